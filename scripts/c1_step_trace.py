"""Summarise a rocprofv3 kernel trace of back-to-back C1 steps into the
decomposition bench.py's C1 line cites (`latency_bound.step_decomposition.trace`).

usage: python scripts/c1_step_trace.py KERNEL_TRACE.csv OUT.json [steps]

A step is one ngpu_process_device of the C1 layer (b3_quad_planned, b3_tree,
dedup_small_lds) plus the result table's same-stream D2H, which HIP runs as
the blit kernel __amd_rocclr_copyBuffer.  Over the last `steps` steps (200):
median kernel durations, median gaps between consecutive kernels (a profiled
run adds a few us to every gap) and the median step (first kernel start to the
next step's first kernel start)."""
import csv
import json
import re
import sys

import numpy as np

ORDER = ["b3_quad_planned", "b3_tree", "dedup_small_lds", "copyBuffer"]


def short(name):
    for k in ORDER:
        if k in name:
            return k
    return None


def main():
    path, out = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    rows = []
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r["Queue_Id"]))
    rows.sort()
    # steps: runs of the four kernels in order
    seq = []
    i = 0
    while i + 4 <= len(rows):
        if [x[2] for x in rows[i:i + 4]] == ORDER:
            seq.append(rows[i:i + 4])
            i += 4
        else:
            i += 1
    seq = seq[-(steps + 1):]
    dur = {k: [] for k in ORDER}
    gaps = {f"{a}->{b}": [] for a, b in zip(ORDER, ORDER[1:] + ORDER[:1])}
    step = []
    for s, nxt in zip(seq, seq[1:] + [None]):
        for (t0, t1, k, _) in s:
            dur[k].append((t1 - t0) / 1e3)
        for a, b in zip(s, s[1:]):
            gaps[f"{a[2]}->{b[2]}"].append((b[0] - a[1]) / 1e3)
        if nxt is not None:
            gaps[f"{s[-1][2]}->{nxt[0][2]}"].append((nxt[0][0] - s[-1][1]) / 1e3)
            step.append((nxt[0][0] - s[0][0]) / 1e3)
    med = lambda v: round(float(np.median(v)), 2) if v else None
    res = {"what": "rocprofv3 kernel trace of back-to-back C1 steps (bench.py --workload c1); one step = "
                   "ngpu_process_device of the 108-chunk alpine-like layer + the 7 KB result table D2H on "
                   "the same stream, which HIP runs as the blit kernel __amd_rocclr_copyBuffer",
           "source_csv": re.sub(r".*gpurun_out/", "gpurun_out/", path),
           "steps": len(step), "step_us_median": med(step),
           "kernel_us_median": {k: med(v) for k, v in dur.items()},
           "gap_us_median": {k: med(v) for k, v in gaps.items()},
           "queues": sorted({r[3] for r in rows}),
           "sum_kernels_us": round(sum(med(v) or 0 for v in dur.values()), 2),
           "sum_gaps_us": round(sum(med(v) or 0 for v in gaps.values()), 2)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
