#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV passes for one kernel into a JSON the bench
reads for roofline.traffic (HBM bytes per launch).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes
of a wide coalesced streaming read -> x2; WRITE_SIZE is exact for 16-B streaming
stores.  Both are in KiB.
usage: pmc_summary.py OUT.json KERNEL_REGEX DIR [DIR ...]"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def main():
    out, pat, dirs = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3:]
    rows = []
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if not pat.search(r["Kernel_Name"]):
                    continue
                m = re.search(r"(b3_groups<[^>]*>|b3_quad_\w+|sha256_\w+)", r["Kernel_Name"])
                rows.append((m.group(1) if m else r["Kernel_Name"], r["Counter_Name"],
                             float(r["Counter_Value"]),
                             (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    # the workload's own launches only: a bench also runs the same kernels on
    # small setup inputs (C5's shared pool, dict fixtures), orders of magnitude
    # shorter; keep the launches within 2x of the longest
    top = max((r[3] for r in rows), default=0.0)
    vals = defaultdict(list)
    durs = []
    name = None
    dropped = 0
    for nm, cn, v, du in rows:
        if du < 0.5 * top:
            dropped += 1
            continue
        name = nm
        vals[cn].append(v)
        durs.append(du)
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    res = {"kernel": name, "launches_sampled": {k: len(v) for k, v in vals.items()},
           "short_launch_rows_dropped": dropped,
           "avg_duration_ms_profiled": round(sum(durs) / max(1, len(durs)), 4), "counters": avg}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        res["traffic_bytes"] = int((2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024)
        res["correction"] = "FETCH_SIZE x2 (gfx950 half-count on wide streams), WRITE_SIZE as is, KiB -> B"
    sized = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
    if all(k in avg for k in sized):
        # read requests by size: the exact bytes the L2 asked of the fabric
        # (Infinity Cache + HBM); no x2 rule needed (tools/fetch_calib.hip)
        rb = 32 * avg[sized[0]] + 64 * avg[sized[1]] + 128 * avg[sized[2]]
        res["read_request_bytes"] = int(rb)
        wr = avg.get("WRITE_SIZE", 0) * 1024
        res["traffic_bytes"] = int(rb + wr)
        res["correction"] = ("TCC_EA0_RDREQ_{32,64,128}B_sum x size (+ WRITE_SIZE KiB if "
                             "collected): exact request bytes, no x2 rule")
    if "TCC_EA0_RDREQ_DRAM_sum" in avg and "TCC_EA0_RDREQ_sum" in avg:
        res["dram_request_frac"] = round(avg["TCC_EA0_RDREQ_DRAM_sum"] /
                                         max(1.0, avg["TCC_EA0_RDREQ_sum"]), 4)
    if "GRBM_GUI_ACTIVE" in avg and durs:
        res["clock_ghz"] = round(avg["GRBM_GUI_ACTIVE"] / 8 / (sum(durs) / len(durs) / 1e3) / 1e9, 3)
    if "SQ_INSTS_VALU" in avg:
        res["valu_busy_est"] = "SQ_INSTS_VALU x 4 cyc / 1024 SIMDs / (duration x clock)"
        if "clock_ghz" in res:
            res["valu_busy_frac"] = round(avg["SQ_INSTS_VALU"] * 4 / 1024 /
                                          (sum(durs) / len(durs) / 1e3 * res["clock_ghz"] * 1e9), 3)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
