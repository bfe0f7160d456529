#!/bin/bash
# FETCH_SIZE calibration of b3_groups' access pattern (tools/fetch_calib.hip):
# one --pmc pass (kernel trace only), summarised per kernel.
# usage: scripts/gpu_fetch_calib.sh TAG
set -u
TAG=${1:-fcal}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/p1" -o pmc \
  -- "$ROOT/tools/fetch_calib" > "$OUT/run.log" 2>&1 || { echo "pmc rc=$?"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
from collections import defaultdict
out = sys.argv[1]
v = defaultdict(list)
for f in glob.glob(f"{out}/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        v[k].append(float(r["Counter_Value"]))
bytes_ = 16 << 30
res = {"read_bytes_per_launch": bytes_, "kernels": {}}
for k, xs in v.items():
    fs = sum(xs) / len(xs) * 1024
    res["kernels"][k] = {"launches": len(xs), "fetch_size_bytes": fs,
                         "bytes_over_fetch_size": round(bytes_ / fs, 4)}
json.dump(res, open(f"{out}/fetch_calib.json", "w"), indent=1)
print(json.dumps(res))
PY
