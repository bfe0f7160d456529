"""SHA-256 kernel timing by variant.  python tools/sha_diag.py [chunk_size]"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "nydus-snapshotter_amd")
import nydus_gpu  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
total = 16 << 30
n = total // S
buf = torch.empty(total, dtype=torch.uint8, device="cuda")
buf.random_(0, 256)
ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
ch["offset"] = np.arange(n, dtype=np.uint64) * S
ch["length"] = S
d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
d_out = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
ref = None
for v, name in [(1, "split"), (2, "pair"), (3, "lane"), (5, "pair-r1"), (6, "pair-r4")]:
    eng = nydus_gpu.Engine(digester="sha256", chunk_size=S, flags=v << 11)
    s = torch.cuda.Stream()
    for _ in range(2):
        eng.digest_device(buf.data_ptr(), total, d_ch.data_ptr(), n, d_out.data_ptr(),
                          stream=s.cuda_stream)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(5):
        eng.digest_device(buf.data_ptr(), total, d_ch.data_ptr(), n, d_out.data_ptr(),
                          stream=s.cuda_stream)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 5
    dig = d_out.view(n, 64)[:, :32].cpu().numpy()
    if ref is None:
        ref = dig.copy()
    print(json.dumps({"variant": name, "chunk": S, "ms": round(ms, 3),
                      "gbs": round(total / ms / 1e6, 1),
                      "us_per_block": round(ms * 1e3 / (S // 64 + 1), 4),
                      "matches_split": bool((dig == ref).all())}), flush=True)
    eng.close()
