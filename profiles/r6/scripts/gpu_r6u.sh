#!/bin/bash
# r6u: 32 concurrent C1 Packs (ReadFrom feed, decisions) alternated between
# B3_QUAD_GROUPS=0 / 1 builds, three times: does the leaf-kernel change move
# the Pack API line (its small batches take the quad_planned path)?
set -u
TAG=r6u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for rep in 1 2 3; do
  for v in groups0 groups1; do
    NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/abr6/$v.so timeout -k 10 240 python bench.py --workload c1 --packs 32 \
      --packs-modes decisions --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/packs_${v}_$rep.json" 2> "$OUT/packs_${v}_$rep.err"
    rc=$?; echo "packs $v $rep rc=$rc $(grep -o '"gbs": [0-9.]*' "$OUT/packs_${v}_$rep.json" | head -1)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/packs_${v}_$rep.err"; exit $rc; }
  done
done
echo done
