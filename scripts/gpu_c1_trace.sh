#!/bin/bash
# C1 call timeline: kernel trace of back-to-back untimed calls (tools/c1_gaps.py).
set -u
TAG=${1:-c1trace}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o c1 -- \
  python3 "$ROOT/tools/c1_gaps.py" 0 > "$OUT/c1.log" 2>&1 || exit $?
cat "$OUT/c1.log"
echo ok
