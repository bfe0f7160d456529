#!/bin/bash
# HIP API host cost of one small-layer call (tools/c1_concurrent, K=1):
# rocprofv3 HIP runtime trace + stats.  usage: scripts/gpu_c1_apitrace.sh TAG
set -u
TAG=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
[ -f tools/c1_layer.tar ] || python3 -c "import sys; sys.path.insert(0,'tests/golden'); import layers; open('tools/c1_layer.tar','wb').write(layers.LAYERS['alpine_like']())"
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv -d "$OUT/api" -o c1 -- "$ROOT/tools/c1_concurrent" "$ROOT/tools/c1_layer.tar" 1 1 500 50 > "$OUT/api.log" 2>&1
rc=$?
echo "rc=$rc"
find "$OUT/api" -name '*stats*'
