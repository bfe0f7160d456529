#!/bin/bash
# r6q: the GPU suite on the in-tree build (B3_QUAD_GROUPS, 134 VGPRs), then
# B3_QUAD_GROUPS=0 / 1 on mid-size layers (l8m, l16m, l32m: 1 MiB chunks,
# the quad_planned path up to 40K leaves) and C1, alternated twice.
set -u
TAG=r6q
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for w in l8m l16m l32m c1; do
    for v in groups0 groups1; do
      NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/abr6/$v.so timeout -k 10 200 python bench.py --workload $w \
        --no-cpu-baseline --no-e2e --steps 100 --warmup 20 > "$OUT/${w}_${v}_$rep.json" 2> "$OUT/${w}_${v}_$rep.err"
      rc=$?; echo "$w $v $rep rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/${w}_${v}_$rep.json" | head -1) $(grep -o '"stage_ms": {[^}]*}' "$OUT/${w}_${v}_$rep.json" | head -1 | cut -c1-70)"
      [ $rc -ne 0 ] && { tail -5 "$OUT/${w}_${v}_$rep.err"; exit $rc; }
    done
  done
done
echo done
