#!/bin/bash
# Round-3 closing evidence on the final build: full GPU suite, smoke, the
# bench set (C2 default line with CPU baseline + PCIe rates, C1, C3, C5-1000),
# rocprofv3 kernel stats of the C2 command with the HIP-event agreement check,
# the request-size PMC of b3_groups, and a 16-thread concurrent soak.
set -u
TAG=${1:-r3final}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 60 --timeout-method thread --durations=10 > "$OUT/pytest_gpu.log" 2>&1
ok $? pytest-gpu
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
ok $? smoke
bash scripts/gpu_bench_round.sh "$TAG" c3 c5-1000
ok $? bench-round
CAL=0 bash scripts/gpu_pmc_req.sh "$TAG" c2 > "$OUT/pmc.log" 2>&1
ok $? pmc
timeout -k 10 600 python -u scripts/gpu_soak.py --threads 16 150 > "$OUT/soak_threads.log" 2>&1
ok $? soak-threads
tail -1 "$OUT/soak_threads.log"
