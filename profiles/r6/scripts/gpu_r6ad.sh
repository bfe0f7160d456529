#!/bin/bash
# r6ad: the closing build (in-wave tree levels, narrow tree, dedup scan) end to end: gpu_r6e.sh's suite,
# smoke, default line, C1, 32-Pack lines, rocprof C2 / C3; then the soaks.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/r6/scripts/gpu_r6e.sh r6ad || exit $?
OUT=$ROOT/gpurun_out/r6ad
timeout -k 10 600 python -u scripts/gpu_soak.py 1000 24760 > "$OUT/soak_single.log" 2>&1
rc=$?; echo "soak_single rc=$rc"; tail -1 "$OUT/soak_single.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/gpu_soak.py --threads 16 100 24761 > "$OUT/soak_threads.log" 2>&1
rc=$?; echo "soak_threads rc=$rc"; tail -1 "$OUT/soak_threads.log"
exit $rc
