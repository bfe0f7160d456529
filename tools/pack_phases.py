"""Diagnostic: where the streaming Pack's time goes on the C1 layer
(pack open, each 1 MiB write, close), and ngpu_pack_tar beside it.
Not part of the product."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nydus-snapshotter_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import layers  # noqa: E402
import nydus_gpu  # noqa: E402

tar = layers.LAYERS["alpine_like"]()
eng = nydus_gpu.Engine(chunk_size=1 << 20)
L = nydus_gpu.lib()
hp = ctypes.c_void_p()
assert L.ngpu_alloc_pinned(eng._h, len(tar), ctypes.byref(hp)) == 0
host = np.ctypeslib.as_array((ctypes.c_uint8 * len(tar)).from_address(hp.value))
host[:] = np.frombuffer(tar, np.uint8)
plain = np.frombuffer(tar, np.uint8).copy()  # pageable, like a caller's buffer
reps = 200
acc = {"open": 0.0, "writes": 0.0, "close": 0.0}
for it in range(reps + 20):
    t0 = time.perf_counter()
    w = eng.pack()
    t1 = time.perf_counter()
    for a in range(0, plain.size, 1 << 20):
        w.write(plain[a:a + (1 << 20)])
    t2 = time.perf_counter()
    w.close()
    t3 = time.perf_counter()
    if it >= 20:
        acc["open"] += t1 - t0
        acc["writes"] += t2 - t1
        acc["close"] += t3 - t2
out = {k: round(v / reps * 1e6, 1) for k, v in acc.items()}
buf = np.empty_like(plain)
t0 = time.perf_counter()
for _ in range(reps):
    buf[:] = plain
out["numpy_copy_10MB_us"] = round((time.perf_counter() - t0) / reps * 1e6, 1)
for _ in range(20):
    eng.pack_tar(host)
t0 = time.perf_counter()
for _ in range(reps):
    eng.pack_tar(host)
out["pack_tar_us"] = round((time.perf_counter() - t0) / reps * 1e6, 1)
out["layer_bytes"] = len(tar)
print(json.dumps(out))
L.ngpu_free_pinned(eng._h, hp)
eng.close()
