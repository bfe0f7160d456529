"""Digest+dedup rate on layers whose files follow a realistic size mix
(log-normal sizes, most files a few KiB, a long tail up to tens of MiB), as
opposed to bench.py's uniform 4 MiB files.  Shows how lane imbalance inside a
wave (a small chunk next to a full 8-KiB leaf group) costs throughput.
python tools/mixed_sizes.py [total_GiB] [median_KiB] [chunk_size]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "nydus-snapshotter_amd"))
import nydus_gpu  # noqa: E402


def layout(total, median, chunk, seed=1):
    rng = np.random.default_rng(seed)
    sizes = []
    acc = 0
    while acc < total:
        s = int(min(64 << 20, max(1, rng.lognormal(np.log(median), 1.6))))
        sizes.append(s)
        acc += 512 + (s + 511) // 512 * 512
    sizes = np.array(sizes, np.int64)
    stride = 512 + (sizes + 511) // 512 * 512
    starts = np.concatenate([[0], np.cumsum(stride)[:-1]]) + 512
    per = (sizes + chunk - 1) // chunk
    n = int(per.sum())
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    fi = np.repeat(np.arange(len(sizes)), per)
    k = np.arange(n) - np.repeat(np.cumsum(per) - per, per)
    ch["offset"] = starts[fi] + k * chunk
    ch["length"] = np.minimum(chunk, sizes[fi] - k * chunk)
    ch["file_index"] = fi
    ch["file_offset"] = k * chunk
    return int(stride.sum()) + 1024, ch, sizes


def main():
    total = int(float(sys.argv[1]) * (1 << 30)) if len(sys.argv) > 1 else 4 << 30
    median = int(sys.argv[2]) * 1024 if len(sys.argv) > 2 else 16 * 1024
    chunk = int(sys.argv[3], 0) if len(sys.argv) > 3 else 1 << 20
    nbytes, ch, sizes = layout(total, median, chunk)
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    buf.random_(0, 256)
    n = len(ch)
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    d_out = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    fb = int(ch["length"].sum())
    res = {"files": len(sizes), "chunks": n, "file_bytes": fb, "chunk_size": chunk,
           "median_file": int(np.median(sizes)), "mean_file": int(sizes.mean()),
           "frac_bytes_in_files_lt_64k": round(float(sizes[sizes < 65536].sum() / sizes.sum()), 4)}
    for lanes in (0, 1, 2, 4, 8):
        eng = nydus_gpu.Engine(chunk_size=chunk, leaves_per_lane=lanes, timing=True)
        ts = []
        for r in range(6):
            eng.process_device(buf.data_ptr(), nbytes, d_ch.data_ptr(), n, d_out.data_ptr())
            t = eng.last_timing()
            if r:
                ts.append(t)
        torch.cuda.synchronize()
        tot = float(np.median([t["total_ms"] for t in ts]))
        dig = float(np.median([t["digest_ms"] for t in ts]))
        res[f"lanes{lanes}"] = {"total_ms": round(tot, 3), "digest_ms": round(dig, 3),
                                "tree_ms": round(float(np.median([t["tree_ms"] for t in ts])), 3),
                                "dedup_ms": round(float(np.median([t["dedup_ms"] for t in ts])), 3),
                                "GBps": round(fb / tot / 1e6, 1), "D": ts[-1]["group_log2"]}
        eng.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
