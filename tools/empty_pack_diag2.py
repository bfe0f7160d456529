"""Diagnostic: test_streaming_pack_large_random_layer then the empty pack of
test_streaming_pack_errors in one process.  Not part of the product."""
import io
import os
import sys
import tarfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nydus-snapshotter_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import layers  # noqa: E402
import nydus_gpu  # noqa: E402

tars = {k: fn() for k, fn in layers.LAYERS.items()}
rng = np.random.default_rng(8)
bio = io.BytesIO()
tf = tarfile.open(fileobj=bio, mode="w", format=tarfile.GNU_FORMAT)
blobs = []
for i in range(300):
    n = int(rng.choice([0, 100, 5000, 70000, 1 << 20, 3 << 20]) + rng.integers(0, 3000))
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes() if i % 7 else (blobs[-1] if blobs else b"")
    blobs.append(data)
    ti = tarfile.TarInfo(f"f{i}")
    ti.size = len(data)
    tf.addfile(ti, io.BytesIO(data))
tf.close()
tb = bio.getvalue()
for rep in range(3):
    eng = nydus_gpu.Engine(chunk_size=0x100000, staging_bytes=8 << 20)
    w = eng.pack()
    for a in range(0, len(tb), 1 << 20):
        w.write(tb[a:a + (1 << 20)])
    ch, out, st = w.close()
    print(rep, "big layer", len(ch), st["chunks"], flush=True)
    eng.close()
    for mode in ("plain", "seq"):
        eng = nydus_gpu.Engine(chunk_size=0x100000)
        if mode == "seq":
            w = eng.pack()
            w.write(tars["oci_upper"][: len(tars["oci_upper"]) // 2])
            try:
                w.close()
            except nydus_gpu.NgpuError:
                pass
            w = eng.pack()
            w.write(tars["oci_lower"])
            w.abort()
        ch, out, st = eng.pack().close()
        print(rep, mode, "empty pack chunks", st["chunks"], st, flush=True)
        ch, out, st = eng.pack().close()
        print(rep, mode, "empty pack again chunks", st["chunks"], flush=True)
        eng.close()
