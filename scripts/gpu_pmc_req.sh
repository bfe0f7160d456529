#!/bin/bash
# Read requests by size (exact fabric bytes) and the DRAM share, for the
# calibration kernels (tools/fetch_calib) and the bench's dominant kernel.
# Separate --pmc passes, kernel trace only.
# usage: scripts/gpu_pmc_req.sh TAG [workload]
set -u
TAG=${1:-req}
W=${2:-c2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
S1="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
S2="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum"
CAL=${CAL:-1}  # CAL=0: the bench kernel only (no tools/fetch_calib build needed)
if [ "$CAL" = 1 ]; then
timeout -s KILL 120 rocprofv3 --pmc $S1 --output-format csv -d "$OUT/cal1" -o pmc -- "$ROOT/tools/fetch_calib" > "$OUT/cal1.log" 2>&1
ok $? cal1
timeout -s KILL 120 rocprofv3 --pmc $S2 --output-format csv -d "$OUT/cal2" -o pmc -- "$ROOT/tools/fetch_calib" > "$OUT/cal2.log" 2>&1
ok $? cal2
fi
K='b3_groups|b3_quad_leaves|b3_quad_planned|sha256_split|sha256_pair|sha256_lane'
timeout -k 10 300 rocprofv3 --pmc $S1 --kernel-include-regex "$K" --output-format csv -d "$OUT/k1" -o pmc -- python3 "$ROOT/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-sub > "$OUT/k1.log" 2>&1
ok $? k1
timeout -k 10 300 rocprofv3 --pmc $S2 --kernel-include-regex "$K" --output-format csv -d "$OUT/k2" -o pmc -- python3 "$ROOT/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-sub > "$OUT/k2.log" 2>&1
ok $? k2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d "$OUT/k3" -o pmc -- python3 "$ROOT/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-sub > "$OUT/k3.log" 2>&1
ok $? k3
if [ "$CAL" = 1 ]; then
for k in coalesced 'lane_stream<0>' 'lane_stream<680>'; do
  python3 "$ROOT/scripts/pmc_summary.py" "$OUT/cal_$(echo $k | tr -dc 'a-z0-9').json" "$k" "$OUT/cal1" "$OUT/cal2"
done
fi
python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_req_$W.json" "$K" "$OUT/k1" "$OUT/k2" "$OUT/k3"
