#!/bin/bash
# PMC counter passes on the BLAKE3 digest kernel + variant tuning.
# usage: scripts/gpu_prof.sh TAG
set -u
TAG=${1:-prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 600 python scripts/tune_b3.py --rounds 5 --lanes 4,8 --modes 0,2,4 > "$OUT/tune.jsonl" 2> "$OUT/tune.err"
ok $? tune
cat "$OUT/tune.jsonl"
cd /tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
P=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" \
           "TCC_HIT_sum TCC_MISS_sum" ; do
  P=$((P+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex 'b3_groups' --output-format csv -d "$OUT/pmc$P" -o pmc -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc$P.log" 2>&1
  ok $? "pmc$P"
done
