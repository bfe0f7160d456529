#!/bin/bash
# Held clock of the bench's dominant kernel: GRBM_GUI_ACTIVE / 8 XCDs / kernel
# time (MI355X_MICROARCH.md "DVFS give-back"), one --pmc pass, kernel trace only.
# usage: scripts/gpu_pmc_clock.sh TAG [workload] [steps]
set -u
TAG=${1:-clock}
W=${2:-c2}
STEPS=${3:-40}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
K='b3_groups|b3_quad_leaves|b3_quad_planned|sha256_split|sha256_pair|sha256_lane'
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$K" --output-format csv -d "$OUT/clk" -o pmc -- python3 "$ROOT/bench.py" --workload $W --steps $STEPS --warmup 10 --no-cpu-baseline --no-e2e --no-sub > "$OUT/clk.log" 2>&1
rc=$?; echo "clock pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_clock_$W.json" "$K" "$OUT/clk"
