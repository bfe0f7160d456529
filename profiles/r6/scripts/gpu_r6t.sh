#!/bin/bash
# r6t: the closing build (in-wave tree levels) end to end: gpu_r6e.sh's suite,
# smoke, default line, C1, 32-Pack lines, rocprof C2 / C3; then the soaks.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/r6/scripts/gpu_r6e.sh r6t || exit $?
OUT=$ROOT/gpurun_out/r6t
timeout -k 10 600 python -u scripts/gpu_soak.py 1000 24750 > "$OUT/soak_single.log" 2>&1
rc=$?; echo "soak_single rc=$rc"; tail -1 "$OUT/soak_single.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/gpu_soak.py --threads 16 100 24751 > "$OUT/soak_threads.log" 2>&1
rc=$?; echo "soak_threads rc=$rc"; tail -1 "$OUT/soak_threads.log"
exit $rc
