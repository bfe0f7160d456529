#!/bin/bash
# Timeline of concurrent converter.Pack calls on one engine (tools/c1_concurrent
# pack mode, T threads): kernels, memory copies, HIP API.  usage: TAG T
set -u
TAG=${1:-r2}
T=${2:-4}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
[ -f tools/c1_layer.tar ] || python3 -c "import sys; sys.path.insert(0,'tests/golden'); import layers; open('tools/c1_layer.tar','wb').write(layers.LAYERS['alpine_like']())"
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/ptrace" -o p -- "$ROOT/tools/c1_concurrent" "$ROOT/tools/c1_layer.tar" 1 $T 40 5 0x100000 pack > "$OUT/ptrace.log" 2>&1
echo "rc=$?"
tail -2 "$OUT/ptrace.log"
