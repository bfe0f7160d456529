#!/bin/bash
# A/B of the first-call stats race (DESIGN §3 "The digest guard") with the
# reproducer that found it: tools/step_diag.py 8 (the first node step of 8
# fresh engines on 8 streams), on the pre-fix build (build/ab/race.so: the
# null-stream hipMemset of a new workspace's stats words) and on the fixed
# library, 3 runs each, alternated.  Wrong or unwritten digests on the race
# build are the expected outcome (caught by the guard: EDEVICE), not a GPU fault.
set -u
TAG=${1:-race}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for r in 1 2 3; do
  for b in race fixed; do
    if [ $b = race ]; then L=$ROOT/nydus-snapshotter_amd/build/ab/race.so; else L=$ROOT/nydus-snapshotter_amd/libnydusgpu.so; fi
    NYDUS_GPU_LIB=$L timeout -k 10 180 python3 tools/step_diag.py 8 > "$OUT/$b.$r.log" 2>&1
    rc=$?
    bad=$(grep -c "EDEVICE\|zero [1-9]" "$OUT/$b.$r.log")
    echo "$b run $r rc=$rc parts_with_unwritten_digests=$bad"
    if [ $rc -ne 0 ]; then echo "stopping: rc $rc"; tail -3 "$OUT/$b.$r.log"; exit $rc; fi
  done
done
exit 0
