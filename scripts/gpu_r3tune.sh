#!/bin/bash
# Group-size check on C2 (leaves per lane 4 / 8 / 16, alternated twice) and
# small layers through one engine on 16 streams (C1, 32 MiB).
set -u
TAG=${1:-r3tune}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for r in 1 2; do
  for L in 4 8 16; do
    timeout -k 10 200 python3 bench.py --lanes $L --steps 30 --warmup 10 --no-cpu-baseline --no-e2e > "$OUT/c2_l${L}_$r.json" 2>> "$OUT/err"
    rc=$?; [ $rc -eq 0 ] || { echo "c2 lanes $L rc=$rc"; exit $rc; }
  done
done
for W in c1; do
  timeout -k 10 200 python3 bench.py --workload $W --streams 16 --steps 200 --warmup 20 > "$OUT/${W}_s16.json" 2>> "$OUT/err"
  rc=$?; [ $rc -eq 0 ] || { echo "$W s16 rc=$rc"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import json, sys, os, glob
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), d.get("value"), d.get("ms_per_step"), (d.get("roofline") or {}).get("frac"))
PY
