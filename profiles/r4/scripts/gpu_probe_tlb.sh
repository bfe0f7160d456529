#!/bin/bash
# Is the dict probe's excess read traffic address translation?  Lists the
# counters the box offers, then counts UTCL1 translation hits / misses of
# dict_probe_records by dict size (tools/probe_sweep.py; one warm + 5 timed
# launches per size, sizes in order).  Kernel trace only, own time limits.
# usage: scripts/gpu_probe_tlb.sh TAG [SIZES]
set -u
TAG=${1:-tlb}
SIZES=${2:-1,16,200}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -s KILL 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1
ok $? avail
grep -o -E '\b(TCP_UTCL[A-Z0-9_]*|UTCL2[A-Z0-9_]*|TCP_TCC_[A-Z_]*|TCC_EA0_RD[A-Z0-9_]*|GPUVM[A-Z0-9_]*)\b' "$OUT/avail.txt" | sort -u > "$OUT/avail_tlb.txt"
cat "$OUT/avail_tlb.txt" | tr '\n' ' '; echo
S=""
for c in TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_REQUEST TCP_UTCL1_PERMISSION_MISS; do
  grep -qx "$c" "$OUT/avail_tlb.txt" && S="$S ${c}_sum"
done
echo "pass: $S"
[ -n "$S" ] || exit 0
timeout -s KILL 300 rocprofv3 --pmc $S --kernel-include-regex 'dict_probe_records' --output-format csv -d "$OUT/t1" -o pmc -- python3 "$ROOT/tools/probe_sweep.py" 16 "$SIZES" > "$OUT/t1.log" 2>&1
ok $? tlb1
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
from collections import defaultdict
out = sys.argv[1]
rows = defaultdict(dict)
for f in glob.glob(f"{out}/t1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
seq = [rows[k] for k in sorted(rows)]
res = {"launches": len(seq), "per_launch": seq}
json.dump(res, open(f"{out}/tlb_probe.json", "w"), indent=1)
for i, r in enumerate(seq):
    print(i, {k: round(v / (16 << 20), 4) for k, v in r.items()}, "per query")
PY
