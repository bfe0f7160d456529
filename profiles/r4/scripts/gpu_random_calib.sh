#!/bin/bash
# Line requests of random reads (tools/random_calib.hip) by table size and
# access shape, request-size PMC then DRAM share, separate passes.
# usage: scripts/gpu_random_calib.sh TAG [reads_M] [sizes_MiB]
set -u
TAG=${1:-rcal}
R=${2:-16}
SZ=${3:-16,256,4096,12800}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 120 "$ROOT/tools/random_calib" "$R" "$SZ" > "$OUT/plain.jsonl" 2> "$OUT/plain.err"
ok $? plain
cat "$OUT/plain.jsonl"
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --kernel-include-regex random_reads --output-format csv -d "$OUT/p1" -o pmc -- "$ROOT/tools/random_calib" "$R" "$SZ" > "$OUT/p1.log" 2>&1
ok $? pmc1
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex random_reads --output-format csv -d "$OUT/p2" -o pmc -- "$ROOT/tools/random_calib" "$R" "$SZ" > "$OUT/p2.log" 2>&1
ok $? pmc2
python3 - "$OUT" "$R" <<'PY'
import csv, glob, json, sys
from collections import defaultdict
out, R = sys.argv[1], int(sys.argv[2]) << 20
plain = [json.loads(l) for l in open(f"{out}/plain.jsonl")]
res = []
for p in ("p1", "p2"):
    rows = defaultdict(dict)
    for f in glob.glob(f"{out}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    res.append([rows[k] for k in sorted(rows)])
summary = []
for i, pl in enumerate(plain):
    c = {}
    for pas in res:
        lo = pas[i * pl["launches"]:(i + 1) * pl["launches"]]
        for k in (lo[0] if lo else {}):
            c[k] = sum(x[k] for x in lo) / len(lo)
    lines = (32 * c.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) +
             128 * c.get("TCC_EA0_RDREQ_128B_sum", 0)) / 128
    e = dict(pl, lines_per_read=round(lines / R, 4),
             dram_frac=round(c.get("TCC_EA0_RDREQ_DRAM_sum", 0) / max(1, c.get("TCC_EA0_RDREQ_sum", 1)), 4),
             tcc_hit_per_read=round(c.get("TCC_HIT_sum", 0) / R, 4),
             tcc_miss_per_read=round(c.get("TCC_MISS_sum", 0) / R, 4))
    summary.append(e)
    print(json.dumps(e))
json.dump(summary, open(f"{out}/random_calib.json", "w"), indent=1)
PY
