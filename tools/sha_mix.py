"""SHA-256 digest time of one launch by chunk mix (diagnostic, runs on the GPU
box): is a 1 MiB chunk's chain slower when its workgroup also holds short
chunks, or when its bytes are not 16-B aligned?  One JSON line per case:
one digest call's wall ms (enqueue + device sync; the kernel is ms long),
median of 7 launches.

usage: python3 tools/sha_mix.py [sha-mode flags value]
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "nydus-snapshotter_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402  (one HIP runtime per process: torch's, loaded first)
import numpy as np  # noqa: E402

import layers  # noqa: E402
import nydus_gpu  # noqa: E402

MiB = 1 << 20


def run(eng, data, chunks, reps=7):
    # the buffer ends at the last chunk's end, as a layer's data would
    end = int((chunks["offset"] + chunks["length"]).max())
    d = torch.from_numpy(np.frombuffer(data, np.uint8)[:end].copy()).cuda()
    ch = torch.from_numpy(np.ascontiguousarray(chunks).view(np.uint8).copy()).cuda()
    out = torch.zeros(len(chunks) * nydus_gpu.RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    ms = []
    torch.cuda.synchronize()
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        eng.digest_device(d.data_ptr(), d.numel(), ch.data_ptr(), len(chunks), out.data_ptr())
        torch.cuda.synchronize()  # (device-wide: the engine's stream included)
        ms.append((time.perf_counter() - t0) * 1e3)
    return round(statistics.median(ms[1:]), 3)


def chunk_table(spec):
    """spec: [(offset, length)] -> CHUNK_DTYPE array (file index = position)."""
    a = np.zeros(len(spec), dtype=nydus_gpu.CHUNK_DTYPE)
    for i, (o, n) in enumerate(spec):
        a[i]["offset"], a[i]["length"] = o, n
        a[i]["file_index"] = i
    return a


def main():
    flags = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    eng = nydus_gpu.Engine(device=0, digester="sha256", chunk_size=MiB, timing=True,
                           flags=flags)
    rng = np.random.default_rng(7)
    big = rng.integers(0, 256, 80 * MiB, dtype=np.uint8).tobytes()
    cases = {
        "one_1MiB": [(0, MiB)],
        "64x1MiB": [(i * MiB, MiB) for i in range(64)],
        "1MiB_plus_63x4KiB": [(0, MiB)] + [(MiB + i * 4096, 4096) for i in range(63)],
        "1MiB_plus_63x100KiB": [(0, MiB)] + [(MiB + i * 102400, 102400) for i in range(63)],
        "1MiB_at_offset_8": [(8, MiB)],
        "1MiB_at_offset_512": [(512, MiB)],
    }
    for name, spec in cases.items():
        print(json.dumps({"case": name, "flags": flags, "chunks": len(spec),
                          "digest_ms": run(eng, big, chunk_table(spec))}), flush=True)
    tar = layers.alpine_like_tar(0xA1F1E)
    ch = nydus_gpu.tar_chunks(tar, MiB)
    print(json.dumps({"case": "c1_layer", "flags": flags, "chunks": len(ch),
                      "longest": int(ch["length"].max()),
                      "longest_offset_mod16": int(ch["offset"][np.argmax(ch["length"])] % 16),
                      "digest_ms": run(eng, tar, ch)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
