#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, lane sweep, rocprofv3 stats.
# Every GPU step has its own time limit; a crash/timeout code stops the script.
# usage: scripts/gpu_check.sh TAG [quick]
set -u
TAG=${1:-r1}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"

ok() { # test failures (1) are data; anything else ends the session
  local rc=$1 what=$2
  echo "$what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi
}

rocminfo 2>/dev/null | grep -m1 -o 'gfx9[0-9a-z]*' > "$OUT/arch.txt"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
ok $? pytest-gpu
tail -5 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
ok $? smoke
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
ok $? bench
cat "$OUT/bench.json"
for W in c3 c5; do
  timeout -k 10 600 python bench.py --workload $W --steps 20 --warmup 20 > "$OUT/bench_$W.json" 2>> "$OUT/bench.err"
  ok $? bench-$W
  cat "$OUT/bench_$W.json"
done
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$ROOT/bench.py" --steps 10 --warmup 10 --no-cpu-baseline --no-e2e > "$OUT/prof.log" 2>&1
ok $? rocprof
find "$OUT/prof" -name '*stats*' | head
python3 "$ROOT/scripts/prof_agree.py" "$OUT/prof" 'b3_groups' "$OUT/prof.log" "$OUT/rocprof_agreement.json"
