#!/bin/bash
# r6p: the two lowest tree levels of multi-leaf chunks inside the leaf kernel
# (B3_QUAD_GROUPS): the GPU suite on the new in-tree build, then C1 and a
# 32 MiB layer alternated between B3_QUAD_GROUPS=0 / 1 builds (build/abr6).
set -u
TAG=r6p
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in groups0 groups1; do
    NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/abr6/$v.so timeout -k 10 200 python bench.py --workload c1 \
      --no-cpu-baseline --no-e2e --steps 200 --warmup 20 > "$OUT/c1_${v}_$rep.json" 2> "$OUT/c1_${v}_$rep.err"
    rc=$?; echo "c1 $v $rep rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/c1_${v}_$rep.json" | head -1) $(grep -o '"stage_ms": {[^}]*}' "$OUT/c1_${v}_$rep.json" | head -1)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/c1_${v}_$rep.err"; exit $rc; }
  done
done
echo done
