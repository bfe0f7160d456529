#!/bin/bash
# Round 5, VERDICT r4 item 4: where the bare BLAKE3 compression stream loses
# 21 % against the linear 2-/4-cycle issue model.
#  1. tools/valu_bank: issue rate by VGPR bank pattern, and the compression
#     stream under three register assignments (s_memtime cycles per wave);
#  2. SQ counters on tools/b3_ceiling at 4 and 8 waves/SIMD (one --pmc pass
#     each, quad-cycle units for the SQ_*_CYCLES / ACTIVE / WAIT counters).
# usage: scripts/gpu_r5_valu.sh TAG
set -u
TAG=${1:-r5v}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 180 ./tools/valu_bank > "$OUT/valu_bank.jsonl" 2> "$OUT/valu_bank.err"
ok $? valu_bank
cat "$OUT/valu_bank.jsonl" | cut -c1-160
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
ok $? list
want="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VALU"
have=""
n=0
for c in $want; do
  if grep -qw "$c" "$OUT/counters.txt" && [ $n -lt 7 ]; then have="$have $c"; n=$((n+1)); fi
done
echo "counters:$have GRBM_GUI_ACTIVE"
for w in 4 8; do
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $have GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_w$w" -o b3c -- "$ROOT/tools/b3_ceiling" $w > "$OUT/pmc_w$w.out" 2>&1)
  ok $? pmc_w$w
  tail -2 "$OUT/pmc_w$w.out"
done
