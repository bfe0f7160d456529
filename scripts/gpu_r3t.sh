#!/bin/bash
# Full GPU suite (60 s per-test limit, stacks on a hang), then a same-box A/B
# of the C1 bench: b3_quad_windows (default) vs b3_quad_planned
# (NGPU_B3_WINDOWS=0), alternated twice.
set -u
TAG=${1:-r3t}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 60 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
ok $? pytest-gpu
tail -3 "$OUT/pytest_gpu.log"
for i in 1 2; do
  NGPU_B3_WINDOWS=0 timeout -k 10 300 python3 bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline --no-e2e > "$OUT/c1_planned_$i.json" 2>> "$OUT/bench.err"
  ok $? c1_planned_$i
  timeout -k 10 300 python3 bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline --no-e2e > "$OUT/c1_windows_$i.json" 2>> "$OUT/bench.err"
  ok $? c1_windows_$i
done
python3 - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "c1_*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), d["value"], d["ms_per_step"], d.get("stage_ms"))
PY
