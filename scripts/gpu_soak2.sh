#!/bin/bash
# Both soaks in one call: sequential random layers (CASES, SEED), then the
# concurrent mode (THREADS threads x PER cases).
set -u
TAG=${1:-r3za}
CASES=${2:-1000}
SEED=${3:-7777}
THREADS=${4:-6}
PER=${5:-60}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u scripts/gpu_soak.py "$CASES" "$SEED" > "$OUT/soak.log" 2>&1
rc=$?; echo "soak rc=$rc"; tail -2 "$OUT/soak.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/gpu_soak.py --threads "$THREADS" "$PER" > "$OUT/soak_threads.log" 2>&1
rc=$?; echo "threads rc=$rc"; tail -3 "$OUT/soak_threads.log"; exit $rc
