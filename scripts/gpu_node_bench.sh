#!/bin/bash
# Node exchange cost: bench.py --node with W parts of device 0 on C4-16 (one
# process, one engine per listed device), partitioned then replicated dict.
# usage: scripts/gpu_node_bench.sh TAG W...
set -u
TAG=${1:-r3}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
for W in "$@"; do
  DEVS=$(python3 -c "print(','.join(['0']*$W))")
  timeout -k 10 500 python3 bench.py --node "$DEVS" --workload c4-16 --no-e2e --no-cpu-baseline > "$OUT/bench_node_w$W.json" 2> "$OUT/bench_node_w$W.err"
  rc=$?
  echo "node W=$W rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 - "$OUT/bench_node_w$W.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], json.dumps(d.get("extra", {}).get("node", d.get("node", {})))[:800])
PY
done
