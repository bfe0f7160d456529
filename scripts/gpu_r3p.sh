#!/bin/bash
# Re-entry check of the tree: full GPU suite, smoke, C2 + C1 bench lines,
# then a kernel trace of the C1 bench (per-kernel durations of a small layer).
# usage: scripts/gpu_r3p.sh TAG
set -u
TAG=${1:-r3p}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
ok $? pytest-gpu
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
ok $? smoke
timeout -k 10 600 python3 bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
ok $? bench_c2
timeout -k 10 300 python3 bench.py --workload c1 --steps 200 --warmup 20 > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"
ok $? bench_c1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c1" -o prof -- python3 "$ROOT/bench.py" --workload c1 --steps 200 --warmup 20 --no-cpu-baseline --no-e2e > "$OUT/prof_c1.log" 2>&1
ok $? prof_c1
