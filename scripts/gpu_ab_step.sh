#!/bin/bash
# Whole-step A/B of two libnydusgpu.so builds on one box: GPU parity tests on
# the new (in-tree) build, then bench.py C2 / C5-shape and the small-file
# layer mix, builds alternated twice.
# usage: scripts/gpu_ab_step.sh OLD.so TAG [skip-tests]
set -u
OLD=$1
TAG=${2:-abstep}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
NEW=$ROOT/nydus-snapshotter_amd/libnydusgpu.so
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ "${3:-}" != skip-tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for v in old new; do
    lib=$OLD
    if [ "$v" = new ]; then lib=$NEW; fi
    for W in c2 c5; do
      NYDUS_GPU_LIB=$lib timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 3 \
        --no-cpu-baseline --no-e2e > "$OUT/${W}_${v}_$r.json" 2>>"$OUT/err" || exit $?
    done
    NYDUS_GPU_LIB=$lib timeout -k 10 200 python tools/mixed_sizes.py 4 4 0x100000 \
      > "$OUT/m4_${v}_$r.json" 2>>"$OUT/err" || exit $?
  done
done
python3 - "$OUT" <<'EOF'
import glob, json, os, sys
out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "c[25]_*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), d["value"], d["ms_per_step"], d["stage_ms"])
for f in sorted(glob.glob(os.path.join(out, "m4_*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), d["lanes0"])
EOF
