#!/bin/bash
# A/B of the first-call stats race (DESIGN §3 "The digest guard"): the
# regression test on the pre-fix build (build/ab/race.so: null-stream hipMemset
# of a new workspace's stats words) and on the fixed library, 3 runs each,
# alternated.  A test FAILURE here is the expected outcome on the race build
# (wrong digests caught by the test / the guard), not a GPU fault.
set -u
TAG=${1:-race}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
T=tests/test_gpu_guard.py::test_first_call_of_fresh_engines_on_nonblocking_streams
for r in 1 2 3; do
  for b in race fixed; do
    if [ $b = race ]; then L=$ROOT/nydus-snapshotter_amd/build/ab/race.so; else L=$ROOT/nydus-snapshotter_amd/libnydusgpu.so; fi
    NYDUS_GPU_LIB=$L timeout -k 10 180 python -u -m pytest "$T" -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/$b.$r.log" 2>&1
    rc=$?
    echo "$b run $r rc=$rc $(tail -1 $OUT/$b.$r.log)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc $rc"; exit $rc; fi
  done
done
grep -h "assert\|EDEVICE" "$OUT"/race.*.log | head -5
exit 0
