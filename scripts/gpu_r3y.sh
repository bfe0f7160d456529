#!/bin/bash
# Full GPU suite (60 s per-test limit) on the 40K quad limit, then the size sweep.
set -u
TAG=${1:-r3y}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 60 --timeout-method thread --durations=10 > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_size_sweep.sh "$TAG"
