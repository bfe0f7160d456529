#!/bin/bash
# GPU parity suite without -x (every failure listed), then smoke and a short C2
# bench.  Each GPU step has its own limit; a crash/timeout code ends the script.
# usage: scripts/gpu_tests_all.sh TAG [pytest-args...]
set -u
TAG=${1:-r3}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() {
  local rc=$1 what=$2
  echo "$what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi
}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread "$@" > "$OUT/pytest_gpu.log" 2>&1
ok $? pytest-gpu
grep -E "passed|failed|FAILED|ERROR" "$OUT/pytest_gpu.log" | tail -25
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
ok $? smoke
tail -2 "$OUT/smoke.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 10 > "$OUT/bench.json" 2> "$OUT/bench.err"
ok $? bench
cut -c1-600 "$OUT/bench.json"
