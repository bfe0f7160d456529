#!/bin/bash
# r6j: LDS bank conflicts of the small-layer kernels (C1: b3_quad_planned,
# b3_tree, dedup_small_lds): one PMC pass, kernel-trace only.
set -u
TAG=r6j
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
K='b3_quad_planned|b3_tree|dedup_small_lds'
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "$K" --output-format csv -d "$OUT/pmc1" -o pmc -- python3 "$ROOT/bench.py" --workload c1 --steps 20 --warmup 5 \
  --no-cpu-baseline --no-e2e > "$OUT/pmc1.log" 2>&1
rc=$?; echo "pmc1 rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/pmc1.log"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "$K" --output-format csv -d "$OUT/kt" -o kt -- python3 "$ROOT/bench.py" --workload c1 --steps 20 --warmup 5 \
  --no-cpu-baseline --no-e2e > "$OUT/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"
find "$OUT" -name '*.csv' | head
exit $rc
