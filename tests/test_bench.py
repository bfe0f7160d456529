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


def test_merge_extra_on_oracle_decisions():
    """bench.merge_extra (C5's host Merge): per-layer bootstraps built from
    dedup decisions, merged against the dict bootstrap -> every layer's own
    blob plus exactly the dict blobs the layers hit.  Decisions come from the
    CPU oracle (no GPU), three layers of 12 chunks."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(bench.__file__), "oracle"))
    import oracle_py
    S, P, L = 4096, 12, 3
    rng = np.random.default_rng(4)
    m = 50
    dg = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    us = np.full(m, S, np.int32)
    bl = (np.arange(m) % 3).astype(np.int32)  # dict blobs 0..2
    ix = np.arange(m, dtype=np.int32)
    ch = np.zeros(P * L, nydus_gpu.CHUNK_DTYPE)
    ch["length"] = S
    ch["offset"] = np.arange(P * L, dtype=np.uint64) * S
    ch["file_offset"] = (np.arange(P * L) % P) * S
    res = np.zeros(P * L, nydus_gpu.RESULT_DTYPE)
    for l in range(L):
        dig = rng.integers(0, 256, (P, 32), dtype=np.uint8)
        dig[0] = dg[l]          # a dict hit on blob l % 3
        dig[5] = dg[3 + l]      # another one
        dig[7] = dig[6]         # INTRA
        dec, _ = oracle_py.dedup(dig, ch["length"][:P], dg, us.view(np.uint32), bl.view(np.uint32),
                                 ix.view(np.uint32))
        sl = slice(l * P, (l + 1) * P)
        for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
            res[f][sl] = dec[f]
        res["digest"][sl] = dig
        res["dict_blob"][sl] = np.where(dec["kind"] == nydus_gpu.DICT, bl[np.minimum(dec["ref"], m - 1)], 0)
    out = bench.merge_extra(nydus_gpu, ch, res, L, P, S, (dg, us, bl, ix))
    hit_blobs = {int(bl[l]) for l in range(L)} | {int(bl[3 + l]) for l in range(L)}
    assert out["own_blobs"] == L
    assert out["dict_blobs"] == len(hit_blobs)
    assert out["layers"] == L and out["merged_bytes"] > 0
