"""bench.py's synthetic layer layout equals what the real tar front end
produces on the same bytes (small instance, CPU only)."""
import io
import tarfile

import numpy as np

import bench
import nydus_gpu


def test_synthetic_layout_matches_parser():
    h, stride, total, ch = bench.synthetic_layout(5, 3 * 1024 * 1024 + 100, 1 << 20)
    buf = np.zeros(total, np.uint8)
    rng = np.random.default_rng(0)
    for i in range(5):
        buf[i * stride:i * stride + 512] = h[i]
        buf[i * stride + 512:i * stride + 512 + 3 * 1024 * 1024 + 100] = rng.integers(0, 256, 3 * 1024 * 1024 + 100)
    got = nydus_gpu.tar_chunks(buf, 1 << 20)
    assert got.tobytes() == ch.tobytes()
    names = [m.name for m in tarfile.open(fileobj=io.BytesIO(buf.tobytes())).getmembers()]
    assert len(names) == 5
