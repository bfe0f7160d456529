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


def test_pool_content_is_a_function_of_the_id():
    """C4/C5 pool contents are regenerated per batch on every rank: content i
    must not depend on which batch (or rank) produced it, and distinct ids
    must give distinct contents."""
    import torch
    S = 4096
    a = bench.pool_content(torch, torch.arange(0, 8), S, device="cpu")
    b = bench.pool_content(torch, torch.tensor([5, 3, 7]), S, device="cpu")
    assert a.shape == (8, S) and a.dtype == torch.uint8
    assert torch.equal(a[5], b[0]) and torch.equal(a[3], b[1]) and torch.equal(a[7], b[2])
    assert len({bytes(r.numpy()) for r in a}) == 8
    # bytes look uniform (no constant high bytes from the shifts)
    counts = np.bincount(a.numpy().ravel(), minlength=256)
    assert counts.min() > 0.5 * counts.mean()
