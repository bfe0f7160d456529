#!/bin/bash
# The remaining BASELINE-shaped workloads on the closing build: C4 (one GPU's
# 128 GiB share of the 1 TiB corpus, pool dict), C5-shape 16 GiB at 64 KiB
# chunks, C3 at 64 KiB chunks, C1 with sha256.
set -u
TAG=${1:-r3more}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for W in c4 c5 c3-64k c1-sha256; do
  timeout -k 10 400 python3 bench.py --workload $W --no-e2e --no-cpu-baseline > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err"
  rc=$?; echo "$W rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import json, sys, os
for W in ["c4", "c5", "c3-64k", "c1-sha256"]:
    d = json.loads(open(os.path.join(sys.argv[1], f"bench_{W}.json")).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(W, d["value"], d["ms_per_step"], r["kernel"], r["frac"])
PY
