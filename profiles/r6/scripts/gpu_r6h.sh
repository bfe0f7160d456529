#!/bin/bash
# r6h: eager-copy token sweep (NGPU_EAGER_PACKS) on 32 concurrent C1 Packs
# (ReadFrom feed), alternated twice; 0 = every pack streams (the r6e build).
set -u
TAG=r6h
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for rep in 1 2; do
  for k in 0 4 8 12 16; do
    NGPU_EAGER_PACKS=$k timeout -k 10 240 python bench.py --workload c1 --packs 32 --packs-modes decisions \
      --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/packs_k${k}_rep${rep}.json" 2> "$OUT/packs_k${k}_rep${rep}.err"
    rc=$?
    echo "k=$k rep=$rep rc=$rc $(grep -o '"gbs": [0-9.]*' "$OUT/packs_k${k}_rep${rep}.json" | head -1)"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/packs_k${k}_rep${rep}.err"; exit $rc; fi
  done
done
echo done
