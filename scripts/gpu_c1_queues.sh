#!/bin/bash
# C1 on K streams of one engine vs hardware queues (GPU_MAX_HW_QUEUES) and
# workspace slots (NGPU_WS_SLOTS).  usage: TAG
set -u
TAG=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
[ -f tools/c1_layer.tar ] || python3 -c "import sys; sys.path.insert(0,'tests/golden'); import layers; open('tools/c1_layer.tar','wb').write(layers.LAYERS['alpine_like']())"
for HQ in 4 8 16; do
  for SL in 4 8 16; do
    for K in 4 8 16; do
      echo -n "{\"hw_queues\": $HQ, \"ws_slots\": $SL, " >> "$OUT/c1_queues.jsonl"
      GPU_MAX_HW_QUEUES=$HQ NGPU_WS_SLOTS=$SL timeout -k 10 60 tools/c1_concurrent tools/c1_layer.tar $K 1 2000 100 | cut -c2- >> "$OUT/c1_queues.jsonl" || exit 1
    done
  done
done
cat "$OUT/c1_queues.jsonl"
