#!/bin/bash
# C1 layers converted concurrently: K engines on one GPU, one stream each.
# usage: scripts/gpu_c1_concurrent.sh TAG [K...]
set -u
TAG=${1:-r2}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 200 python3 bench.py --workload c1 --steps 300 --warmup 30 --no-cpu-baseline --no-e2e > "$OUT/c1_k1.json" 2> "$OUT/c1_k1.err" || exit $?
cat "$OUT/c1_k1.json"
for K in "${@:-2 4 8}"; do
  timeout -k 10 200 python3 bench.py --workload c1 --streams $K --steps 300 --warmup 30 > "$OUT/c1_k$K.json" 2> "$OUT/c1_k$K.err" || exit $?
  cat "$OUT/c1_k$K.json"
done
for K in "${@:-2 4 8}"; do
  timeout -k 10 200 python3 bench.py --workload c1 --streams $K --threads --steps 300 --warmup 30 > "$OUT/c1_t$K.json" 2> "$OUT/c1_t$K.err" || exit $?
  cat "$OUT/c1_t$K.json"
done
