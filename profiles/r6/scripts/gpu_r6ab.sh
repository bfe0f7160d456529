#!/bin/bash
# r6ab: dedup_small_lds without its contended LDS atomics (the first NEW chunk
# by its prefix, dict-hit blob minima reduced per wave): the suite, then C1
# and the two log-normal small layers alternated (old / new dedup builds).
set -u
TAG=r6ab
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in dold dnew; do
    NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/abr6/$v.so timeout -k 10 200 python bench.py --workload c1 \
      --no-cpu-baseline --no-e2e --steps 200 --warmup 20 > "$OUT/c1_${v}_$rep.json" 2> "$OUT/c1_${v}_$rep.err"
    rc=$?; echo "c1 $v $rep rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/c1_${v}_$rep.json" | head -1) $(grep -o '"dedup": [0-9.]*' "$OUT/c1_${v}_$rep.json" | head -1)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/c1_${v}_$rep.err"; exit $rc; }
  done
  for shape in "0.03 3" "0.035 4"; do
    for v in dold dnew; do
      tag=$(echo $shape | tr ' .' '__')
      NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/abr6/$v.so timeout -k 10 120 python tools/mixed_sizes.py $shape 0x100000 \
        > "$OUT/mixed_${tag}_${v}_$rep.json" 2> "$OUT/mixed_${tag}_${v}_$rep.err"
      rc=$?; echo "$shape $v $rep rc=$rc $(grep -o '"lanes0": {[^}]*}' "$OUT/mixed_${tag}_${v}_$rep.json")"
      [ $rc -ne 0 ] && { tail -5 "$OUT/mixed_${tag}_${v}_$rep.err"; exit $rc; }
    done
  done
done
echo done
