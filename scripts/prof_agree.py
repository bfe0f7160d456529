#!/usr/bin/env python3
"""Check that rocprofv3's per-dispatch durations of the dominant kernel agree
with the HIP-event time bench.py reported in the SAME run (the timed steps are
the last K dispatches; the warmup dispatches before them are excluded).
usage: prof_agree.py PROF_DIR KERNEL_REGEX BENCH_LOG OUT.json"""
import csv
import glob
import json
import re
import sys


def main():
    d, pat, log, out = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3], sys.argv[4]
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if pat.search(r["Kernel_Name"])]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    line = next(json.loads(x) for x in open(log) if x.startswith('{"metric"'))
    k = line["steps"]
    timed = durs[-k:]
    rp = sum(timed) / len(timed)
    bench = line["stage_ms"]["digest"]
    res = {"kernel_regex": sys.argv[2], "dispatches": len(durs), "timed_steps": k,
           "rocprof_avg_ms_timed": round(rp, 4), "bench_hip_event_ms": bench,
           "rel_diff": round(abs(rp - bench) / bench, 4),
           "rocprof_all_ms": [round(x, 4) for x in durs]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
