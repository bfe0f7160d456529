#!/bin/bash
# r6z: the gated narrow tree (>= 512 chunks) on the in-tree build: the GPU
# suite, then C1, l32m and the two log-normal small layers once each.
set -u
TAG=r6z
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for w in c1 l32m; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e --steps 100 --warmup 20 > "$OUT/$w.json" 2> "$OUT/$w.err"
  rc=$?; echo "$w rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/$w.json" | head -1)"; [ $rc -ne 0 ] && exit $rc
done
for shape in "0.03 3" "0.035 4"; do
  tag=$(echo $shape | tr ' .' '__')
  timeout -k 10 120 python tools/mixed_sizes.py $shape 0x100000 > "$OUT/mixed_$tag.json" 2> "$OUT/mixed_$tag.err"
  rc=$?; echo "$shape rc=$rc $(grep -o '"lanes0": {[^}]*}' "$OUT/mixed_$tag.json")"; [ $rc -ne 0 ] && exit $rc
done
echo done
