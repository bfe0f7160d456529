#!/bin/bash
# C1 layers through one engine from C++ (tools/c1_concurrent): K streams,
# T submitting threads.  usage: scripts/gpu_c1_native.sh TAG
set -u
TAG=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
[ -f tools/c1_layer.tar ] || python3 -c "import sys; sys.path.insert(0,'tests/golden'); import layers; open('tools/c1_layer.tar','wb').write(layers.LAYERS['alpine_like']())"
for KT in "1 1" "2 1" "4 1" "8 1" "16 1" "2 2" "4 4" "8 8" "16 8"; do
  set -- $KT
  timeout -k 10 120 tools/c1_concurrent tools/c1_layer.tar $1 $2 2000 100 >> "$OUT/c1_native.jsonl" 2>> "$OUT/c1_native.err" || { echo "K=$1 T=$2 failed"; exit 1; }
done
cat "$OUT/c1_native.jsonl"
for T in 1 2 4 8 16; do
  timeout -k 10 120 tools/c1_concurrent tools/c1_layer.tar 1 $T 300 20 0x100000 pack >> "$OUT/c1_native_pack.jsonl" 2>> "$OUT/c1_native.err" || { echo "pack T=$T failed"; exit 1; }
done
cat "$OUT/c1_native_pack.jsonl"
