#!/bin/bash
# r6ae: on the closing build, the C1 step's kernel trace (c1_step_trace.py)
# and the 2-rank gloo rehearsal of the N > 1 line (every node extra on 0,0).
set -u
TAG=r6ae
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c1trace" -o c1 -- python3 "$ROOT/bench.py" --workload c1 --steps 200 --warmup 20 --no-cpu-baseline --no-e2e --no-sub > "$OUT/c1trace.log" 2>&1
rc=$?; echo "c1trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"
bash scripts/gpu_n2_gloo.sh $TAG/n2 > "$OUT/n2_call.log" 2>&1
rc=$?; echo "n2 rc=$rc"; exit $rc
