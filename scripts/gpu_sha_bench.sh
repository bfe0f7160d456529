#!/bin/bash
# SHA-256 parity + C3 / C3-64k bench lines + kernel stats for the C3-64k kernel.
set -u
TAG=${1:-shabench}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dict.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "sha" > "$OUT/pytest_sha.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_sha.log"; [ $rc -eq 0 ] || exit 1
for W in c3-64k c3; do
  timeout -k 10 600 python -u bench.py --workload $W > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err"
  rc=$?; echo "bench $W rc=$rc"; cat "$OUT/bench_$W.json"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c3_64k -- \
  python3 "$ROOT/bench.py" --workload c3-64k --steps 10 --warmup 3 --no-cpu-baseline --no-e2e \
  > "$OUT/prof_c3_64k.json" 2> "$OUT/prof_c3_64k.err" || exit $?
echo ok
