#!/bin/bash
# A/B of the quad G's DPP form (B3_QUAD_ADDDPP builds) on latency-bound small
# layers, builds alternated twice on one box; then the parity tests of the
# quad paths on the in-tree (default) build.
set -u
TAG=${1:-r3ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for r in 1 2; do
  for v in dpp0 dpp1; do
    for W in c1 l16m l32m; do
      NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/ab/$v.so timeout -k 10 120 python3 bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline --no-e2e > "$OUT/${W}_${v}_$r.json" 2>> "$OUT/err"
      rc=$?; [ $rc -eq 0 ] || { echo "$W $v rc=$rc"; exit $rc; }
    done
  done
done
python3 - "$OUT" <<'PY'
import json, sys, os, glob
rows = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_dpp*_*.json"))):
    W, v, r = os.path.basename(f)[:-5].split("_")
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows.setdefault((W, v), []).append((d["value"], d["stage_ms"]["digest"], d["stage_ms"]["tree"]))
for k in sorted(rows):
    print(k, rows[k])
PY
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 60 --timeout-method thread -k "kat or golden or random" > "$OUT/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 "$OUT/parity.log"; exit $rc
