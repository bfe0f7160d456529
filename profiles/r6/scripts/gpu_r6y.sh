#!/bin/bash
# r6y: b3_tree at 256 threads / 512-CV tiles for the planned path's group CVs
# (B3_TREE_NARROW) vs 1024 / 1024: the GPU suite on the in-tree build, then C1,
# l8m, l32m and two log-normal small layers alternated twice.
set -u
TAG=r6y
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for w in c1 l8m l32m; do
    for v in narrow0 narrow1; do
      NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/abr6/$v.so timeout -k 10 200 python bench.py --workload $w \
        --no-cpu-baseline --no-e2e --steps 100 --warmup 20 > "$OUT/${w}_${v}_$rep.json" 2> "$OUT/${w}_${v}_$rep.err"
      rc=$?; echo "$w $v $rep rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/${w}_${v}_$rep.json" | head -1) $(grep -o '"stage_ms": {[^}]*}' "$OUT/${w}_${v}_$rep.json" | head -1 | cut -c1-70)"
      [ $rc -ne 0 ] && { tail -5 "$OUT/${w}_${v}_$rep.err"; exit $rc; }
    done
  done
  for shape in "0.03 3" "0.035 4"; do
    for v in narrow0 narrow1; do
      tag=$(echo $shape | tr ' .' '__')
      NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/abr6/$v.so timeout -k 10 120 python tools/mixed_sizes.py $shape 0x100000 \
        > "$OUT/mixed_${tag}_${v}_$rep.json" 2> "$OUT/mixed_${tag}_${v}_$rep.err"
      rc=$?; echo "$shape $v $rep rc=$rc $(grep -o '"lanes0": {[^}]*}' "$OUT/mixed_${tag}_${v}_$rep.json")"
      [ $rc -ne 0 ] && { tail -5 "$OUT/mixed_${tag}_${v}_$rep.err"; exit $rc; }
    done
  done
done
echo done
