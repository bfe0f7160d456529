#!/bin/bash
# r6c: node / batch / bench-launch tests after the prefetch and hits fixes,
# 32-Pack API rates (ReadFrom feed; one engine and a 2-part node), a kernel
# trace of back-to-back C1 steps, and the round-6 PMC traffic profiles.
set -u
TAG=r6c
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_bench_launch.py tests/test_gpu_batch.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
ok $? pytest; tail -3 "$OUT/pytest.log"
timeout -k 10 400 python bench.py --workload c1 --packs 32 --steps 20 --warmup 5 > "$OUT/packs_c1.json" 2> "$OUT/packs_c1.err"
ok $? packs_c1
timeout -k 10 400 python bench.py --workload c1 --packs 32 --steps 20 --warmup 5 --node 0,0 --no-cpu-baseline > "$OUT/packs_c1_node00.json" 2> "$OUT/packs_c1_node00.err"
ok $? packs_c1_node00
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c1trace" -o c1 -- python3 "$ROOT/bench.py" --workload c1 --steps 200 --warmup 20 --no-cpu-baseline --no-e2e --no-sub > "$OUT/c1trace.log" 2>&1
ok $? c1trace
cd "$ROOT"
for W in c1 c2 c3; do
  CAL=0 timeout -k 10 900 bash scripts/gpu_pmc_req.sh $TAG/pmc_$W $W > "$OUT/pmc_$W.log" 2>&1
  ok $? pmc_$W
done
timeout -k 10 900 bash scripts/gpu_pmc_probe.sh $TAG/pmc_probe > "$OUT/pmc_probe.log" 2>&1
ok $? pmc_probe
echo done
