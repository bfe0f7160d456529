#!/bin/bash
# Non-temporal loads in the whole-leaf fast path (build/ab/fastnt.so,
# -DB3_FAST_NT=1) against the product build: C2 digest time alternated on one
# box (scripts/gpu_ab.sh), then the variant's held clock and read requests.
# usage: scripts/gpu_ab_fastnt.sh TAG
set -u
TAG=${1:-abnt}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
L=$ROOT/nydus-snapshotter_amd
bash scripts/gpu_ab.sh "$L/libnydusgpu.so" "$L/build/ab/fastnt.so" "$TAG" > "$OUT/ab.log" 2>&1
ok $? ab
cat "$OUT/ab.log" | cut -c1-300
K=b3_groups
B="--steps 20 --warmup 10 --no-cpu-baseline --no-e2e --no-sub"
cd /tmp
NYDUS_GPU_LIB=$L/build/ab/fastnt.so timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex $K --output-format csv -d "$OUT/clk" -o pmc -- python3 "$ROOT/bench.py" $B > "$OUT/clk.log" 2>&1
ok $? clk
NYDUS_GPU_LIB=$L/build/ab/fastnt.so timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --kernel-include-regex $K --output-format csv -d "$OUT/req" -o pmc -- python3 "$ROOT/bench.py" $B > "$OUT/req.log" 2>&1
ok $? req
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT/pmc_clock_fastnt.json" $K "$OUT/clk" | cut -c1-300
python3 scripts/pmc_summary.py "$OUT/pmc_req_fastnt.json" $K "$OUT/req" | cut -c1-400
