#!/bin/bash
# Round-4 node step + Pack-stream check: node / emit / ociref / pack GPU tests,
# the early-emission phase run, and the 8-part node bench (routed, copy and
# the bulk step).  usage: scripts/gpu_r4_step.sh TAG
set -u
TAG=${1:-r4s}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_emit.py tests/test_gpu_ociref.py tests/test_gpu_rafs.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
ok $? pytest
tail -1 "$OUT/pytest_gpu.log"
NGPU_SINK_STATS=1 timeout -k 10 300 python3 tools/e2e_early.py 3 32 512 > "$OUT/e2e_early.json" 2> "$OUT/e2e_early.err"
ok $? early
python3 -c "import json; d=json.load(open('$OUT/e2e_early.json')); print({k: v for k, v in d.items() if k != 'runs'})"
grep sink "$OUT/e2e_early.err" | tail -3
timeout -k 10 400 python3 bench.py --node 0,0,0,0,0,0,0,0 --workload c4-16 --steps 10 --warmup 10 > "$OUT/node_w8.json" 2> "$OUT/node_w8.err"
ok $? node
python3 -c "import json; d=json.load(open('$OUT/node_w8.json')); print(json.dumps(d['node_step'])); print(d['modes']['partition']['value_gbs'], d['modes']['partition']['ms_per_step'])"
