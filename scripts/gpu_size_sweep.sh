#!/bin/bash
# Layer-size sweep of the device-resident rate (1 MiB chunks, blake3): where
# the small-layer latency floor gives way to the VALU roofline.
set -u
TAG=${1:-r3w}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for W in l8m l16m l32m l64m l128m small; do
  timeout -k 10 200 python3 bench.py --workload $W --steps 100 --warmup 20 --no-cpu-baseline --no-e2e > "$OUT/sweep_$W.json" 2>> "$OUT/sweep.err"
  rc=$?; echo "$W rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import json, sys, os
for W in ["l8m", "l16m", "l32m", "l64m", "l128m", "small"]:
    d = json.loads(open(os.path.join(sys.argv[1], f"sweep_{W}.json")).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(W, d["value"], d["ms_per_step"], d["stage_ms"], r["kernel"], r["frac"])
PY
