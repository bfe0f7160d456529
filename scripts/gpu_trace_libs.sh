#!/bin/bash
# Kernel trace of back-to-back untimed C1 calls (tools/c1_gaps.py) per build.
# usage: scripts/gpu_trace_libs.sh TAG LIB.so [LIB.so ...]
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for lib in "$@"; do
  v=$(basename "$lib" .so)
  NYDUS_GPU_LIB=$ROOT/$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
    -d "$OUT/$v" -o kt -- python3 "$ROOT/tools/c1_gaps.py" 0 > "$OUT/$v.log" 2>&1 || exit $?
  echo "$v $(grep us_per_call "$OUT/$v.log")"
done
