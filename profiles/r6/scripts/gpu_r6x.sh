#!/bin/bash
# r6x: realistic small layers (log-normal file sizes, tools/mixed_sizes.py:
# 20-35 MB, median file 2-4 KiB, 1 MiB chunks: the quad_planned path) on the
# B3_QUAD_GROUPS=0 / 1 builds, alternated twice.
set -u
TAG=r6x
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for rep in 1 2; do
  for shape in "0.03 3" "0.02 2" "0.035 4"; do
    for v in groups0 groups1; do
      tag=$(echo $shape | tr ' .' '__')
      NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/abr6/$v.so timeout -k 10 120 python tools/mixed_sizes.py $shape 0x100000 \
        > "$OUT/mixed_${tag}_${v}_$rep.json" 2> "$OUT/mixed_${tag}_${v}_$rep.err"
      rc=$?; echo "$shape $v $rep rc=$rc $(grep -o '"lanes0": {[^}]*}' "$OUT/mixed_${tag}_${v}_$rep.json")"
      [ $rc -ne 0 ] && { tail -5 "$OUT/mixed_${tag}_${v}_$rep.err"; exit $rc; }
    done
  done
done
echo done
