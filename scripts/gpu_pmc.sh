#!/bin/bash
# PMC passes (separate runs, kernel-trace only; no sys/runtime trace) on the
# bench's dominant kernel, summarised into profiles-ready JSON.
# usage: scripts/gpu_pmc.sh TAG [workload]
set -u
TAG=${1:-pmc}
W=${2:-c2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
K='b3_groups|sha256_split|sha256_pair'
P=0
for SET in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES"; do
  P=$((P+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "$K" --output-format csv -d "$OUT/pmc$P" -o pmc -- python3 "$ROOT/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/pmc$P.log" 2>&1
  ok $? "pmc$P"
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_$W.json" "$K" "$OUT"/pmc1 "$OUT"/pmc2 "$OUT"/pmc3
