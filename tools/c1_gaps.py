"""Diagnostic: back-to-back ngpu_process_device calls on the C1 layer with the
engine's timing events on or off (argv[1] = 1/0), for a rocprofv3 kernel
trace of the inter-kernel gaps.  Not part of the product."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nydus-snapshotter_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

import layers  # noqa: E402
import nydus_gpu  # noqa: E402

timing = sys.argv[1] == "1"
tar = layers.LAYERS["alpine_like"]()
ch = nydus_gpu.tar_chunks(tar, 1 << 20)
buf = torch.from_numpy(np.frombuffer(tar, np.uint8).copy()).cuda()
d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
out = torch.empty(len(ch) * 64, dtype=torch.uint8, device="cuda")
eng = nydus_gpu.Engine(chunk_size=1 << 20, timing=timing)
s = torch.cuda.Stream()
for it in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        eng.process_device(buf.data_ptr(), buf.numel(), d_ch.data_ptr(), len(ch), out.data_ptr(),
                           stream=s.cuda_stream)
    s.synchronize()
    dt = (time.perf_counter() - t0) / 200
print(f"timing={int(timing)} us_per_call={dt * 1e6:.1f}")
eng.close()
