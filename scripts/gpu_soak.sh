#!/bin/bash
# GPU soak (scripts/gpu_soak.py): random layers through pack_tar + streaming Pack vs the oracle.
set -u
TAG=${1:-r3z}
CASES=${2:-200}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u scripts/gpu_soak.py "$CASES" "${3:-20560}" > "$OUT/soak.log" 2>&1
rc=$?; echo "soak rc=$rc"; tail -3 "$OUT/soak.log"; exit $rc
