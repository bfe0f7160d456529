#!/bin/bash
# Round-4 extra measurements: fast-path NT-load A/B, the clock diagnostic
# (product vs no-load build), the Pack stream with arenas.  usage: scripts/gpu_r4_extra.sh TAG
set -u
TAG=${1:-r4x}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
NGPU_PACK_TRACE=1 NGPU_SINK_STATS=1 timeout -k 10 300 python3 tools/e2e_early.py 3 32 512 > "$OUT/e2e_early.json" 2> "$OUT/e2e_early.err"
ok $? early
python3 -c "import json; d=json.load(open('$OUT/e2e_early.json')); print({k: v for k, v in d.items() if k != 'runs'})"
bash scripts/gpu_clock_diag.sh "$TAG/clk" > "$OUT/clk.log" 2>&1
ok $? clockdiag
tail -4 "$OUT/clk.log"
bash scripts/gpu_ab_fastnt.sh "$TAG/abnt" > "$OUT/abnt.log" 2>&1
ok $? abnt
tail -8 "$OUT/abnt.log" | cut -c1-300
