#!/bin/bash
# A/B/n of several builds of libnydusgpu.so on one GPU box (box-to-box clock
# spread is a few %, so variants are compared inside one call, alternated):
# C2 digest kernel (scripts/tune_b3.py) and a small-file layer mix.
# usage: scripts/gpu_abn.sh TAG ROUNDS LIB.so [LIB.so ...]
set -u
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for lib in "$@"; do
    v=$(basename "$lib" .so)
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
