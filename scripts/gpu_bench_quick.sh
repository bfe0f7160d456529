#!/bin/bash
# Quick bench lines (no CPU baseline / e2e) for C2, C5-shape, C3 on one box.
# usage: scripts/gpu_bench_quick.sh TAG
set -u
TAG=${1:-quick}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for W in c2 c5 c2 c5 c3; do
  timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-e2e \
    >> "$OUT/$W.jsonl" 2>>"$OUT/err" || exit $?
done
python3 - "$OUT" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.jsonl"))):
    for line in open(f):
        d = json.loads(line)
        print(os.path.basename(f), d["value"], d["ms_per_step"], d["stage_ms"], d["roofline"]["frac"])
PY
