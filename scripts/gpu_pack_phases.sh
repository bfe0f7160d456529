#!/bin/bash
# Concurrent streaming Packs of the C1 layer through one engine: per-layer
# write / close split, beside the host memcpy ceiling of the writes.
# usage: scripts/gpu_pack_phases.sh TAG
set -u
TAG=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
[ -f tools/c1_layer.tar ] || python3 -c "import sys; sys.path.insert(0,'tests/golden'); import layers; open('tools/c1_layer.tar','wb').write(layers.LAYERS['alpine_like']())"
for T in 1 2 4 8 16; do
  timeout -k 10 120 tools/c1_concurrent tools/c1_layer.tar 1 $T 300 20 0x100000 memcpy >> "$OUT/pack_phases.jsonl" 2>> "$OUT/pack_phases.err" || { echo "memcpy T=$T failed"; exit 1; }
  timeout -k 10 120 tools/c1_concurrent tools/c1_layer.tar 1 $T 300 20 0x100000 pack >> "$OUT/pack_phases.jsonl" 2>> "$OUT/pack_phases.err" || { echo "pack T=$T failed"; exit 1; }
done
cat "$OUT/pack_phases.jsonl"
