#!/bin/bash
# Round 5, VERDICT r4 item 4, second pass: where the waves of the compression
# stream sit (HW_ID per wave: waves per SIMD and each SIMD's issue rate), for
# workgroups of 64 / 256 / 1024 threads and one or 8 dispatch rounds; then SQ
# counters of b3_groups on the C2 bench (resident waves, issue stalls).
# usage: scripts/gpu_r5_valu2.sh TAG
set -u
TAG=${1:-r5v2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
for cfg in "256 1" "64 1" "1024 1" "256 8" "64 8"; do
  set -- $cfg
  for v in compiled align xor_diff mix_x4a4_diff; do
    timeout -k 10 120 ./tools/valu_bank $v $1 $2 >> "$OUT/placement.jsonl" 2>> "$OUT/placement.err"
    ok $? "placement $v $1 $2"
  done
done
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_c2" -o c2 -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 --settle-s 0 --no-cpu-baseline --no-e2e --no-sub > "$OUT/pmc_c2.out" 2>&1)
ok $? pmc_c2
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_ceil" -o ceil -- "$ROOT/tools/b3_ceiling" 4 8 > "$OUT/pmc_ceil.out" 2>&1)
ok $? pmc_ceil
