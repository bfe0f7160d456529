#!/bin/bash
# Probe line requests by dict size (tools/probe_sweep.py): a timing run, then one
# request-size PMC pass (kernel trace only); per-size averages by launch order.
# usage: scripts/gpu_probe_sweep.sh TAG [SIZES_M]   (NGPU_PROBE_VARIANT passes through)
set -u
TAG=${1:-psweep}
SIZES=${2:-1,16,64,200}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
cd "$ROOT"
timeout -k 10 300 python3 tools/probe_sweep.py 16 $SIZES > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
ok $? sweep
cat "$OUT/sweep.jsonl"
cd /tmp
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --kernel-include-regex "dict_probe_records|dict_probe_variant|dict_probe_multi" --output-format csv -d "$OUT/pmc" -o pmc -- python3 "$ROOT/tools/probe_sweep.py" 16 $SIZES > "$OUT/pmc.log" 2>&1
ok $? pmc
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
f = glob.glob(f"{out}/pmc/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "dict_probe_records" in r["Kernel_Name"] or "dict_probe_variant" in r["Kernel_Name"] or "dict_probe_multi" in r["Kernel_Name"]]
disp = {}
for r in rows:
    disp.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(disp)
sweep = [json.loads(l) for l in open(f"{out}/sweep.jsonl")]
per = sweep[0]["launches"]
res = []
for i, s in enumerate(sweep):
    ds = [disp[d] for d in ids[i * per:(i + 1) * per]]
    lines = sum(d.get("TCC_EA0_RDREQ_128B_sum", 0) + d.get("TCC_EA0_RDREQ_64B_sum", 0) / 2 +
                d.get("TCC_EA0_RDREQ_32B_sum", 0) / 4 for d in ds) / len(ds)
    s["read_lines_per_probe"] = round(lines / s["queries"], 3)
    s["model_lines_per_probe"] = round(0.25 + 1 + s["hits"] / s["queries"], 3)
    res.append(s)
    print(json.dumps(s))
json.dump(res, open(f"{out}/probe_sweep.json", "w"), indent=1)
PY
