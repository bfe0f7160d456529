#!/usr/bin/env python3
"""Interleaved A/B of BLAKE3 digest-kernel variants in ONE process
(cdna_hip_programming.md §5.4 rule 24): leaves-per-lane x load mode, on the
C2 layer resident in HBM.  Prints one JSON line per variant (median/min of the
digest-kernel time measured with HIP events)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "nydus-snapshotter_amd"))

import torch  # noqa: E402  (torch's HIP runtime first)

import bench  # noqa: E402
import nydus_gpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--lanes", default="4,8,16")
    ap.add_argument("--modes", default="0,1,2,3")
    ap.add_argument("--files", type=int, default=4096)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--digester", default="blake3")
    args = ap.parse_args()
    buf, ch = bench.build_layer_on_gpu(torch, args.files, 4 << 20, args.chunk, seed=7)
    n = len(ch)
    fb = int(ch["length"].sum())
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    d_out = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    ref = None
    engines = {}
    for L in [int(x) for x in args.lanes.split(",")]:
        for M in [int(x) for x in args.modes.split(",")]:
            engines[(L, M)] = nydus_gpu.Engine(chunk_size=args.chunk, digester=args.digester,
                                               leaves_per_lane=L, timing=True, flags=(1 + M) << 8)
    times = {k: [] for k in engines}
    for r in range(args.rounds + 1):
        for k, e in engines.items():
            e.process_device(buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n, d_out.data_ptr())
            t = e.last_timing()
            if r:
                times[k].append(t)
            torch.cuda.synchronize()
            if k[1] == 4:
                continue  # diagnostic no-load variant: digests are meaningless
            if ref is None:
                ref = d_out.clone()
            else:
                assert torch.equal(ref, d_out), f"variant {k} differs"
    for (L, M), ts in times.items():
        dg = np.array([t["digest_ms"] for t in ts])
        tr = np.array([t["tree_ms"] for t in ts])
        tot = np.array([t["total_ms"] for t in ts])
        print(json.dumps({"lanes": L, "mode": M, "digest_ms_med": round(float(np.median(dg)), 3),
                          "digest_ms_min": round(float(dg.min()), 3),
                          "tree_ms": round(float(np.median(tr)), 3),
                          "total_ms": round(float(np.median(tot)), 3),
                          "GBps_total": round(fb / (np.median(tot) / 1e3) / 1e9, 1)}), flush=True)
    for e in engines.values():
        e.close()


if __name__ == "__main__":
    main()
