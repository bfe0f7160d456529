#!/bin/bash
# r6k: double-buffered quad message staging (B3_QUAD_DB): the GPU suite on the
# new in-tree build, then C1 (and a 32 MiB quad-path layer) alternated between
# B3_QUAD_DB=0 / 1 builds of the same tree.
set -u
TAG=r6k
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
# (the suite subset ran in the first r6k call: 125 passed; build/ab is gpurun-ignored, so the A/B builds ship from build/abr6)
for rep in 1 2; do
  for v in db0 db1; do
    NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/abr6/$v.so timeout -k 10 200 python bench.py --workload c1 \
      --no-cpu-baseline --no-e2e --steps 200 --warmup 20 > "$OUT/c1_${v}_$rep.json" 2> "$OUT/c1_${v}_$rep.err"
    rc=$?; echo "c1 $v $rep rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/c1_${v}_$rep.json" | head -1) $(grep -o '"digest": [0-9.]*' "$OUT/c1_${v}_$rep.json" | head -1)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/c1_${v}_$rep.err"; exit $rc; }
  done
done
echo done
