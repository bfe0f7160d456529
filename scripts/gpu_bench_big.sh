#!/bin/bash
# The multi-layer / dict workloads on one box: C4 (one GPU's share of the
# 1 TiB corpus), C5-1000, C3-64k.  usage: scripts/gpu_bench_big.sh TAG
set -u
TAG=${1:-big}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for W in c5-1000 c4 c4-16 c3-64k; do
  timeout -k 10 400 python bench.py --workload $W --steps 10 --warmup 5 --no-e2e \
    > "$OUT/$W.json" 2>>"$OUT/err" || exit $?
  python3 -c "import json,sys; d=json.load(open('$OUT/$W.json')); print('$W', d['value'], d['ms_per_step'], d['stage_ms'], d['roofline']['frac'], d.get('decisions'))"
done
