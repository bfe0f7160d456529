#!/bin/bash
# A/B of two builds of libnydusgpu.so on the same GPU box (box-to-box clock
# spread is a few %, so compare builds inside one call): C2 digest kernel and
# a small-file layer mix, alternating builds twice.
# usage: scripts/gpu_ab.sh OLD.so NEW.so TAG
set -u
OLD=$1
NEW=$2
TAG=${3:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in 1 2; do
  for v in old new; do
    lib=$OLD
    if [ "$v" = new ]; then lib=$NEW; fi
    NYDUS_GPU_LIB=$lib timeout -k 10 200 python scripts/tune_b3.py --rounds 7 --lanes 8 --modes 0 \
      > "$OUT/c2_${v}_$r.jsonl" 2>>"$OUT/err" || exit $?
    NYDUS_GPU_LIB=$lib timeout -k 10 200 python tools/mixed_sizes.py 4 4 0x100000 \
      > "$OUT/m4_${v}_$r.json" 2>>"$OUT/err" || exit $?
  done
done
for f in "$OUT"/c2_*.jsonl; do echo "$f $(cat "$f")"; done
for f in "$OUT"/m4_*.json; do
  echo "$f $(python3 -c "import json; d=json.load(open('$f')); print(d['lanes0'])")"
done
