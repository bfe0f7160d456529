#!/bin/bash
# Round-3 check: full GPU suite (no -x), smoke, C2 bench with the clock settle
# (driver-like flags), then the request-size PMC of C2's dominant kernel.
set -u
TAG=${1:-r3f}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
bash scripts/gpu_tests_all.sh "$TAG" || exit $?
CAL=0 bash scripts/gpu_pmc_req.sh "$TAG" c2 > "$OUT/pmc.log" 2>&1
rc=$?
tail -3 "$OUT/pmc.log"
exit $rc
