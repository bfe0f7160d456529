#!/usr/bin/env python3
"""Phase timing of converter.Pack end to end: a C2-shaped
tar sample (512 x 4 MiB files of random bytes, 1 MiB chunks) in engine-pinned
host memory, packed to /dev/null three ways, alternated:
  sha     -- hashlib SHA-256 over the sample (the single-stream bound);
  finish  -- retain + finish(dest) after the last write (no early emission);
  early   -- retain + set_output(dest) before the first write, finish(None).
Per run: seconds to the end of the writes and to the end of the call.
usage: tools/e2e_early.py [ROUNDS] [WRITE_MIB] [FILES] [THREADS,...]  -> one JSON line
THREADS: BlobWriter pool sizes for the early mode (0 = the default min(16, CPUs));
each gets its own mode "early_t<N>"."""
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "nydus-snapshotter_amd"))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    piece = (int(sys.argv[2]) if len(sys.argv) > 2 else 32) << 20
    n_files = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    threads = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0]
    import torch
    import nydus_gpu
    import bench
    buf, _ = bench.build_layer_on_gpu(torch, n_files, 4 << 20, 1 << 20, seed=11)
    eng = nydus_gpu.Engine(device=0, chunk_size=1 << 20, staging_bytes=64 << 20)
    L = nydus_gpu.lib()
    hp = ctypes.c_void_p()
    nbytes = buf.numel()
    assert L.ngpu_alloc_pinned(eng._h, nbytes, ctypes.byref(hp)) == 0
    host = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(hp.value))
    host[:] = buf.cpu().numpy()
    del buf
    fd = os.open(os.devnull, os.O_WRONLY)
    res = {"sample_bytes": nbytes, "write_bytes": piece, "runs": []}
    try:
        def run(mode):
            t0 = time.perf_counter()
            if mode == "sha":
                hashlib.sha256(memoryview(host)).digest()
                return {"mode": mode, "total_s": time.perf_counter() - t0}
            w = eng.pack(retain=True)
            t_open = time.perf_counter() - t0
            early = mode.startswith("early")
            if early:
                t = int(mode[7:]) if mode.startswith("early_t") else 0
                w.set_output(nydus_gpu.FdWriter(fd), compressor="none", threads=t)
            t_open = time.perf_counter() - t0
            for a in range(0, nbytes, piece):
                w.write(host[a:a + piece])
            tw = time.perf_counter() - t0
            if early:
                info = w.finish(None)[3]
            else:
                info = w.finish(nydus_gpu.FdWriter(fd), compressor="none")[3]
            return {"mode": mode, "open_s": t_open, "writes_s": tw,
                    "total_s": time.perf_counter() - t0,
                    "stream": info["stream_digest"]}
        run("early")  # warm
        modes = ["sha", "finish"] + (["early"] if threads == [0] else [f"early_t{t}" for t in threads])
        for _ in range(rounds):
            for m in modes:
                res["runs"].append(run(m))
    finally:
        os.close(fd)
        L.ngpu_free_pinned(eng._h, hp)
        eng.close()
    digs = {r["stream"] for r in res["runs"] if "stream" in r}
    res["streams_equal"] = len(digs) == 1
    for m in modes:
        ts = sorted(r["total_s"] for r in res["runs"] if r["mode"] == m)
        res[f"{m}_gbs_med"] = round(nbytes / ts[len(ts) // 2] / 1e9, 3)
    for r in res["runs"]:
        r.pop("stream", None)
        for k in ("open_s", "writes_s", "total_s"):
            if r.get(k) is not None:
                r[k] = round(r[k], 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
