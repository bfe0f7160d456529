#!/bin/bash
# Full GPU suite with a 60 s per-test limit: a hang ends with every thread's
# Python stack in the log (pytest-timeout, thread method), not a silent kill.
set -u
TAG=${1:-r3s}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 60 --timeout-method thread --durations=25 > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "rc=$rc"
tail -4 "$OUT/pytest_gpu.log"
exit $rc
