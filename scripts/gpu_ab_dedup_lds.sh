#!/bin/bash
# A/B of dedup_small_lds' workgroup size on C1 (256 threads for <= 256 chunks
# vs 1024), alternating twice on one box, then the small-layer parity tests.
set -u
TAG=${1:-abd}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in 1 2; do
  for v in wide narrow; do
    if [ $v = wide ]; then export NGPU_DEDUP_LDS_THREADS=1024; else unset NGPU_DEDUP_LDS_THREADS; fi
    timeout -k 10 200 python bench.py --workload c1 --steps 400 --warmup 50 --no-cpu-baseline --no-e2e \
      > "$OUT/c1_${v}_$r.json" 2>>"$OUT/err" || exit $?
    python3 -c "import json; d=json.loads(open('$OUT/c1_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'], d['stage_ms'])"
  done
done
unset NGPU_DEDUP_LDS_THREADS
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_guard.py tests/test_gpu_rafs.py -q -p no:cacheprovider --timeout 180 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -2 "$OUT/tests.log"
exit $rc
