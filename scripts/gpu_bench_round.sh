#!/bin/bash
# Round bench set: default bench line (C2, with CPU baseline + PCIe rates),
# C1, and the rocprofv3 kernel-trace stats of the C2 command with the
# HIP-event agreement check.  usage: scripts/gpu_bench_round.sh TAG [extra workloads...]
set -u
TAG=${1:-r2}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 600 python3 bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
ok $? bench_c2
tail -c 3000 "$OUT/bench_c2.json"
timeout -k 10 300 python3 bench.py --workload c1 --steps 200 --warmup 20 > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"
ok $? bench_c1
for W in "$@"; do
  timeout -k 10 600 python3 bench.py --workload $W --no-e2e > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err"
  ok $? "bench_$W"
done
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o prof -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/prof_c2.log" 2>&1
ok $? prof_c2
python3 "$ROOT/scripts/prof_agree.py" "$OUT/prof_c2" 'b3_groups' "$OUT/prof_c2.log" "$OUT/rocprof_c2_agreement.json"
