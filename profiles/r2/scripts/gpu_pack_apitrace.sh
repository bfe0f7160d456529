#!/bin/bash
# HIP API / copy / kernel trace of concurrent streaming Packs of the C1
# layer through one engine (tools/c1_concurrent pack mode), T = 1 and 4.
# usage: scripts/gpu_pack_apitrace.sh TAG
set -u
TAG=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
[ -f tools/c1_layer.tar ] || python3 -c "import sys; sys.path.insert(0,'tests/golden'); import layers; open('tools/c1_layer.tar','wb').write(layers.LAYERS['alpine_like']())"
export TMPDIR=/tmp
for T in 1 4; do
  timeout -k 10 180 rocprofv3 --hip-runtime-trace --memory-copy-trace --kernel-trace --stats --output-format csv -d "$OUT/papi$T" -o p -- "$ROOT/tools/c1_concurrent" "$ROOT/tools/c1_layer.tar" 1 $T 100 10 0x100000 pack > "$OUT/papi$T.log" 2>&1 || { echo "T=$T rc=$?"; exit 1; }
  grep c1_concurrent "$OUT/papi$T.log"
done
find "$OUT" -name '*.csv' | head -20
