#!/bin/bash
# Full GPU suite, then the C1 call timeline (kernel trace) and the C1 bench line.
set -u
TAG=${1:-full}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" "$OUT/pytest_gpu.log" | head -30; exit 1; fi
timeout -k 10 300 python -u bench.py --workload c1 > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"
rc=$?; echo "bench c1 rc=$rc"; cat "$OUT/bench_c1.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o c1 -- \
  python3 "$ROOT/tools/c1_gaps.py" 0 > "$OUT/c1.log" 2>&1 || exit $?
grep us_per_call "$OUT/c1.log"
echo ok
