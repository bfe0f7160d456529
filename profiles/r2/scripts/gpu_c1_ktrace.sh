#!/bin/bash
# Kernel trace of C1 layers on K streams of one engine (tools/c1_concurrent).
set -u
TAG=${1:-r2}
K=${2:-4}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
[ -f tools/c1_layer.tar ] || python3 -c "import sys; sys.path.insert(0,'tests/golden'); import layers; open('tools/c1_layer.tar','wb').write(layers.LAYERS['alpine_like']())"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/kt$K" -o kt -- "$ROOT/tools/c1_concurrent" "$ROOT/tools/c1_layer.tar" $K 1 200 20 > "$OUT/kt$K.log" 2>&1
echo "rc=$?"
