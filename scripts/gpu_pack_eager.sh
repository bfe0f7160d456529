#!/bin/bash
# Concurrent converter.Pack throughput vs the eager H2D copy granule.
set -u
TAG=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
[ -f tools/c1_layer.tar ] || python3 -c "import sys; sys.path.insert(0,'tests/golden'); import layers; open('tools/c1_layer.tar','wb').write(layers.LAYERS['alpine_like']())"
for G in 1048576 4194304 67108864; do
  for T in 1 4 16; do
    echo -n "{\"eager\": $G, " >> "$OUT/pack_eager.jsonl"
    NGPU_EAGER_COPY=$G timeout -k 10 120 tools/c1_concurrent tools/c1_layer.tar 1 $T 200 10 0x100000 pack | cut -c2- >> "$OUT/pack_eager.jsonl" || exit 1
  done
done
for T in 1 4 16; do
  echo -n "{\"eager\": 1048576, \"sdma\": 0, " >> "$OUT/pack_eager.jsonl"
  HSA_ENABLE_SDMA=0 timeout -k 10 120 tools/c1_concurrent tools/c1_layer.tar 1 $T 200 10 0x100000 pack | cut -c2- >> "$OUT/pack_eager.jsonl" || exit 1
done
cat "$OUT/pack_eager.jsonl"
