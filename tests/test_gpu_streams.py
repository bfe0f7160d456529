"""Device entry points are stream-ordered with the caller: inputs produced by
PyTorch on its default stream (handle 0 == NULL) and handed straight to the
engine must be complete when the kernels read them (no synchronize between).
Also pins bench.py's C4/C5 pool machinery: planted pool chunks digest to the
pool digests the chunk dict is built from."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def test_null_stream_orders_after_torch_producer():
    import nydus_gpu
    import oracle_py
    S = MiB
    P = 96  # big enough that the producer is still running when the engine starts
    ch = np.zeros(P, nydus_gpu.CHUNK_DTYPE)
    ch["offset"] = np.arange(P, dtype=np.uint64) * S
    ch["length"] = S
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    out = torch.zeros(P * 64, dtype=torch.uint8, device="cuda")
    eng = nydus_gpu.Engine(device=0, digester="blake3", chunk_size=S)
    try:
        for rep in range(3):
            torch.cuda.synchronize()
            data = torch.empty(P * S, dtype=torch.uint8, device="cuda")
            data.random_(0, 256)  # default stream, not synchronised
            for _ in range(4):
                data.add_(1)
            eng.digest_device(data.data_ptr(), data.numel(), d_ch.data_ptr(), P, out.data_ptr(),
                              stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            ref = oracle_py.digest_chunks(data.cpu().numpy(), ch.view(oracle_py.CHUNK_DTYPE), "blake3")
            assert np.array_equal(out.view(P, 64)[:, :32].cpu().numpy(), ref), rep
    finally:
        eng.close()


def test_bench_pool_digests_match_planted_chunks():
    import bench
    import nydus_gpu
    import oracle_py
    S = MiB
    wl = dict(n_files=16, file_size=4 * MiB, chunk=S, digester="blake3", pool=1100)
    buf, ch = bench.build_layer_on_gpu(torch, wl["n_files"], wl["file_size"], S, seed=3)
    _, stride, _, _ = bench.synthetic_layout(1, wl["file_size"], S)
    n = len(ch)
    rng = np.random.default_rng(11)
    sel = np.nonzero(rng.random(n) < 0.5)[0]
    src = rng.integers(0, wl["pool"], len(sel))
    per_file = wl["file_size"] // S
    rows = buf[: wl["n_files"] * stride].view(wl["n_files"], stride)[:, 512:].view(
        wl["n_files"], per_file, S)
    rows[torch.from_numpy(sel // per_file).cuda(), torch.from_numpy(sel % per_file).cuda()] = \
        bench.pool_content(torch, torch.from_numpy(src).cuda(), S)
    pd = bench.pool_digests(torch, nydus_gpu, wl, 0).cpu().numpy()
    host = buf.cpu().numpy()
    ref = oracle_py.digest_chunks(host, ch.view(oracle_py.CHUNK_DTYPE), "blake3")
    assert np.array_equal(ref[sel], pd[src])
    one = bench.pool_content(torch, torch.tensor([1099]).cuda(), S).cpu().numpy().ravel()
    r1 = np.zeros(1, oracle_py.CHUNK_DTYPE)
    r1["length"] = S
    assert np.array_equal(oracle_py.digest_chunks(one, r1, "blake3")[0], pd[1099])
