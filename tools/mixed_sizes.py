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
    torch.cuda.synchronize()
    n = len(ch)
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    d_out = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    fb = int(ch["length"].sum())
    res = {"files": len(sizes), "chunks": n, "file_bytes": fb, "chunk_size": chunk,
           "median_file": int(np.median(sizes)), "mean_file": int(sizes.mean()),
           "frac_bytes_in_files_lt_64k": round(float(sizes[sizes < 65536].sum() / sizes.sum()), 4)}
    # argv[4]: comma list of b3_groups load modes to A/B (interleaved rounds,
    # auto leaves-per-lane only); default: mode 0 over the leaves-per-lane sweep
    modes = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0]
    cases = [(lanes, 0) for lanes in (0, 1, 2, 4, 8)] if modes == [0] else [(0, m) for m in modes]
    engines = {c: nydus_gpu.Engine(chunk_size=chunk, leaves_per_lane=c[0], timing=True,
                                   flags=(1 + c[1]) << 8 if c[1] else 0) for c in cases}
    ts = {c: [] for c in cases}
    ref = None
    for r in range(6):
        for c, eng in engines.items():
            eng.process_device(buf.data_ptr(), nbytes, d_ch.data_ptr(), n, d_out.data_ptr())
            if r:
                ts[c].append(eng.last_timing())
            torch.cuda.synchronize()
            if ref is None:
                ref = d_out.clone()
            else:
                assert torch.equal(ref, d_out), f"case {c} differs"
    for (lanes, mode), tl in ts.items():
        tot = float(np.median([t["total_ms"] for t in tl]))
        dig = float(np.median([t["digest_ms"] for t in tl]))
        key = f"lanes{lanes}" + (f"_m{mode}" if mode else "")
        res[key] = {"total_ms": round(tot, 3), "digest_ms": round(dig, 3),
                    "tree_ms": round(float(np.median([t["tree_ms"] for t in tl])), 3),
                    "dedup_ms": round(float(np.median([t["dedup_ms"] for t in tl])), 3),
                    "GBps": round(fb / tot / 1e6, 1), "D": tl[-1]["group_log2"]}
    for eng in engines.values():
        eng.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
