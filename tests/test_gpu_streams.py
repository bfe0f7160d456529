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


def test_calls_on_different_streams_share_the_workspace_in_order():
    """Back-to-back device-path calls on two different streams (no host sync
    between them) on one engine: whether they share a workspace (ordered on
    the GPU) or take one each (NGPU_WS_SLOTS), every call's results equal
    the oracle's."""
    import nydus_gpu
    import oracle_py
    S = 64 << 10
    layers = []
    for seed in range(2):
        rng = np.random.default_rng(40 + seed)
        P = 900 + 300 * seed  # different chunk counts -> different plans / tiles
        ch = np.zeros(P, nydus_gpu.CHUNK_DTYPE)
        ch["length"] = rng.integers(1, S + 1, P)
        ch["offset"] = np.arange(P, dtype=np.uint64) * S
        dup = rng.choice(P, P // 5, replace=False)
        ch["length"][dup] = S
        data = rng.integers(0, 256, P * S, dtype=np.uint8)
        for d in dup[1:]:  # identical full chunks -> INTRA
            data[int(ch["offset"][d]):int(ch["offset"][d]) + S] = data[int(ch["offset"][dup[0]]):int(ch["offset"][dup[0]]) + S]
        dig = oracle_py.digest_chunks(data, ch.view(oracle_py.CHUNK_DTYPE), "blake3")
        dec, _ = oracle_py.dedup(dig, ch["length"])
        layers.append((torch.from_numpy(data).cuda(), torch.from_numpy(ch.view(np.uint8).copy()).cuda(),
                       P, dig, dec))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    eng = nydus_gpu.Engine(device=0, digester="blake3", chunk_size=S)
    try:
        # outputs zero-filled on torch's stream and complete before any call
        # (the calls run on other streams, unordered with that fill)
        outs = [(k % 2, torch.zeros(layers[k % 2][2] * 64, dtype=torch.uint8, device="cuda"))
                for k in range(6)]
        torch.cuda.synchronize()
        for k, (li, out) in enumerate(outs):
            d_data, d_ch, P, _, _ = layers[li]
            eng.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), P, out.data_ptr(),
                               stream=streams[li].cuda_stream)
        torch.cuda.synchronize()
        for k, (li, out) in enumerate(outs):
            _, _, P, dig, dec = layers[li]
            got = out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
            assert np.array_equal(got["digest"], dig), k
            for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
                assert np.array_equal(got[f], dec[f]), (k, f)
    finally:
        eng.close()


def test_pack_on_engine_stream_interleaved_with_device_calls(oracle):
    """Streaming Pack runs on the engine's own stream, whose stage ends are
    recorded lazily (only when a stage on another stream needs the
    workspace).  Pack writes and device-path calls on a caller stream,
    alternated with no host sync: both results equal the oracle's."""
    import io
    import tarfile
    import nydus_gpu
    S = 64 << 10
    rng = np.random.default_rng(5)
    bio = io.BytesIO()
    tf = tarfile.open(fileobj=bio, mode="w", format=tarfile.GNU_FORMAT)
    for i in range(40):
        n = int(rng.choice([0, 700, 70000, 1 << 20]) + rng.integers(0, 5000))
        ti = tarfile.TarInfo(f"f{i}")
        ti.size = n
        tf.addfile(ti, io.BytesIO(rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
    tf.close()
    tb = bio.getvalue()
    P = 700
    ch = np.zeros(P, nydus_gpu.CHUNK_DTYPE)
    ch["length"] = rng.integers(1, S + 1, P)
    ch["offset"] = np.arange(P, dtype=np.uint64) * S
    data = rng.integers(0, 256, P * S, dtype=np.uint8)
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    dec, _ = oracle.dedup(dig, ch["length"])
    d_data = torch.from_numpy(data).cuda()
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    s = torch.cuda.Stream()
    eng = nydus_gpu.Engine(device=0, digester="blake3", chunk_size=S, staging_bytes=1 << 20)
    try:
        torch.cuda.synchronize()
        w = eng.pack()
        # outputs zero-filled on torch's stream and complete before the calls
        # on `s` (unordered with that fill)
        outs = [torch.zeros(P * 64, dtype=torch.uint8, device="cuda")
                for _ in range(0, len(tb), 300 << 10)]
        torch.cuda.synchronize()
        for pos, out in zip(range(0, len(tb), 300 << 10), outs):
            w.write(tb[pos:pos + (300 << 10)])
            eng.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), P,
                               out.data_ptr(), stream=s.cuda_stream)
        pch, pout, _ = w.close()
        torch.cuda.synchronize()
    finally:
        eng.close()
    for k, out in enumerate(outs):
        got = out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
        assert np.array_equal(got["digest"], dig), k
        for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
            assert np.array_equal(got[f], dec[f]), (k, f)
    ref_ch = oracle.tar_chunks(tb, S)
    assert pch.tobytes() == ref_ch.tobytes()
    pdig = oracle.digest_chunks(tb, ref_ch, "blake3")
    assert np.array_equal(pout["digest"], pdig)
    pdec, _ = oracle.dedup(pdig, ref_ch["length"])
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        assert np.array_equal(pout[f], pdec[f]), f
