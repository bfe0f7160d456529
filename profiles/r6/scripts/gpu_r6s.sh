#!/bin/bash
# r6s: the C1 step on the round-6 leaf kernel (in-wave tree levels): a rocprofv3
# kernel trace of back-to-back steps, and the read-request PMC passes of C1's
# dominant kernel (-> pmc_req_c1.json).
set -u
TAG=r6s
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c1trace" -o c1 -- python3 "$ROOT/bench.py" --workload c1 --steps 200 --warmup 20 --no-cpu-baseline --no-e2e --no-sub > "$OUT/c1trace.log" 2>&1
rc=$?; echo "c1trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"
CAL=0 bash scripts/gpu_pmc_req.sh $TAG c1
