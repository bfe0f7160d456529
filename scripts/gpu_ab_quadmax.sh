#!/bin/bash
# A/B of the quad-path leaf limit (B3_QUAD_MAX_LEAVES builds, scripts/build_ab.sh)
# on mid-size layers, builds alternated twice on one box.
set -u
TAG=${1:-r3x}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for r in 1 2; do
  for v in q32k q40k q48k; do
    for W in l24m l32m l48m; do
      NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/ab/$v.so timeout -k 10 120 python3 bench.py --workload $W --steps 200 --warmup 20 --no-cpu-baseline --no-e2e > "$OUT/${W}_${v}_$r.json" 2>> "$OUT/err"
      rc=$?; [ $rc -eq 0 ] || { echo "$W $v rc=$rc"; exit $rc; }
    done
  done
done
python3 - "$OUT" <<'PY'
import json, sys, os, glob
rows = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "l*_q*_*.json"))):
    W, v, r = os.path.basename(f)[:-5].split("_")
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows.setdefault((W, v), []).append((d["value"], d["stage_ms"]["digest"]))
for k in sorted(rows):
    print(k, rows[k])
PY
