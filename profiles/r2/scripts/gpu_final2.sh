#!/bin/bash
# Round-end set, part 2: C1 (one stream), C5-1000 with the host Merge, C4-16,
# the one-process node, the 2-rank torchrun path (gloo) and the native C1
# concurrency driver.  usage: TAG
set -u
TAG=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ok() { echo "$2 rc=$1"; [ "$1" -eq 0 ] || exit "$1"; }
timeout -k 10 300 python3 bench.py --workload c1 --steps 300 --warmup 30 > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"; ok $? c1
timeout -k 10 600 python3 bench.py --workload c5-1000 --steps 10 --no-cpu-baseline > "$OUT/bench_c5-1000.json" 2> "$OUT/bench_c5-1000.err"; ok $? c5-1000
timeout -k 10 600 python3 bench.py --workload c4-16 --no-cpu-baseline > "$OUT/bench_c4-16.json" 2> "$OUT/bench_c4-16.err"; ok $? c4-16
timeout -k 10 600 python3 bench.py --node 0,0 --workload c4-16 --steps 10 --warmup 10 > "$OUT/bench_node_c4-16_w2.json" 2> "$OUT/bench_node.err"; ok $? node
bash scripts/gpu_n2_gloo.sh "$TAG"; ok $? n2
bash scripts/gpu_c1_native.sh "$TAG"; ok $? native
