"""One engine serving concurrent layer conversions (SURVEY.md §8(b)
Threading: containerd converts an image's layers concurrently, one
LayerConvertFunc per layer, convert_unix.go:822, through one cached engine).

Calls on distinct streams take distinct workspace slots (NGPU_WS_SLOTS) and
run side by side on the GPU; packs open at once each run on their own compute
stream and write their blob streams outside the engine lock.  Whatever the
overlap, every result must equal the oracle's, and every pack's output
stream must equal the one the same tar gives alone."""
import io
import os
import tarfile
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FIELDS = ("kind", "index", "ref", "blob_index", "uncompressed_offset")


def _layer(seed, P, S):
    import oracle_py
    import nydus_gpu
    rng = np.random.default_rng(seed)
    ch = np.zeros(P, nydus_gpu.CHUNK_DTYPE)
    ch["length"] = rng.integers(1, S + 1, P)
    ch["offset"] = np.arange(P, dtype=np.uint64) * S
    dup = rng.choice(P, max(2, P // 5), replace=False)
    ch["length"][dup] = S
    data = rng.integers(0, 256, P * S, dtype=np.uint8)
    a = int(ch["offset"][dup[0]])
    for d in dup[1:]:  # identical full chunks -> INTRA
        o = int(ch["offset"][d])
        data[o:o + S] = data[a:a + S]
    dig = oracle_py.digest_chunks(data, ch.view(oracle_py.CHUNK_DTYPE), "blake3")
    dec, _ = oracle_py.dedup(dig, ch["length"])
    return dict(d_data=torch.from_numpy(data).cuda(),
                d_ch=torch.from_numpy(ch.view(np.uint8).copy()).cuda(), P=P, dig=dig, dec=dec)


@pytest.mark.parametrize("slots", [1, 2, 4])
def test_calls_on_many_streams_of_one_engine(slots, monkeypatch):
    """Six layers of different sizes (one to two small-call sizes, a grid-path
    size) on six streams, three rounds, no host sync: with fewer slots than
    streams the engine waits for a slot's last stage before reusing it."""
    import nydus_gpu
    monkeypatch.setenv("NGPU_WS_SLOTS", str(slots))
    S = 64 << 10
    layers = [_layer(70 + i, P, S) for i, P in enumerate((37, 300, 4096, 5000, 120, 2500))]
    streams = [torch.cuda.Stream() for _ in layers]
    eng = nydus_gpu.Engine(device=0, digester="blake3", chunk_size=S)
    try:
        # outputs zero-filled on torch's stream before any call is enqueued
        # (the calls run on other streams, unordered with that fill)
        outs = [(i, r, torch.zeros(L["P"] * 64, dtype=torch.uint8, device="cuda"))
                for r in range(3) for i, L in enumerate(layers)]
        torch.cuda.synchronize()
        for i, r, out in outs:
            L = layers[i]
            eng.process_device(L["d_data"].data_ptr(), L["d_data"].numel(), L["d_ch"].data_ptr(),
                               L["P"], out.data_ptr(), stream=streams[i].cuda_stream)
        torch.cuda.synchronize()
        for i, r, out in outs:
            L = layers[i]
            got = out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
            assert np.array_equal(got["digest"], L["dig"]), (i, r)
            for f in FIELDS:
                assert np.array_equal(got[f], L["dec"][f]), (i, r, f)
    finally:
        eng.close()


def test_stats_follow_the_stream_of_the_call():
    """ngpu_process_device with host stats on interleaved streams: each call
    reads back its own layer's stats (the slot its stream used)."""
    import nydus_gpu
    S = 64 << 10
    layers = [_layer(90 + i, P, S) for i, P in enumerate((50, 700, 3000))]
    streams = [torch.cuda.Stream() for _ in layers]
    eng = nydus_gpu.Engine(device=0, digester="blake3", chunk_size=S)
    try:
        out = torch.zeros(max(L["P"] for L in layers) * 64, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        for r in range(4):
            for i, L in enumerate(layers):
                st = eng.process_device(L["d_data"].data_ptr(), L["d_data"].numel(),
                                        L["d_ch"].data_ptr(), L["P"], out.data_ptr(),
                                        stream=streams[i].cuda_stream, want_stats=True)
                dec = L["dec"]
                assert st["chunks"] == L["P"], (i, r, st)
                assert st["new_chunks"] == int((dec["kind"] == nydus_gpu.NEW).sum()), (i, r, st)
                assert st["intra_chunks"] == int((dec["kind"] == nydus_gpu.INTRA).sum()), (i, r, st)
    finally:
        eng.close()


def _tar(seed, files):
    rng = np.random.default_rng(seed)
    bio = io.BytesIO()
    tf = tarfile.open(fileobj=bio, mode="w", format=tarfile.GNU_FORMAT)
    pool = [rng.integers(0, 256, 200_000, dtype=np.uint8).tobytes() for _ in range(3)]
    for i in range(files):
        if i % 7 == 3:
            body = pool[i % 3]  # repeated file -> INTRA chunks
        else:
            n = int(rng.choice([0, 900, 70_000, 1 << 20, 3 << 20]) + rng.integers(0, 4000))
            body = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        ti = tarfile.TarInfo(f"d{seed}/f{i}")
        ti.size = len(body)
        tf.addfile(ti, io.BytesIO(body))
    tf.close()
    return bio.getvalue()


def _pack(eng, tb, compressor):
    w = eng.pack(retain=True)
    for pos in range(0, len(tb), 256 << 10):
        w.write(tb[pos:pos + (256 << 10)])
    dest = io.BytesIO()
    ch, rs, st, info = w.finish(dest, compressor=compressor)
    return ch, rs, st, dest.getvalue()


@pytest.mark.parametrize("compressor", ["none", "zstd"])
def test_concurrent_packs_from_threads_equal_sequential(compressor, oracle):
    """Six Packs on one engine from six threads at once (staging slots small
    enough that every pack dispatches several times while the others run):
    chunk lists, decisions and the whole output stream equal each tar packed
    alone, and the decisions equal the oracle's."""
    import nydus_gpu
    S = 1 << 20
    tars = [_tar(200 + i, 14 + 3 * i) for i in range(6)]
    solo = nydus_gpu.Engine(device=0, digester="blake3", chunk_size=S, staging_bytes=4 << 20)
    try:
        alone = [_pack(solo, tb, compressor) for tb in tars]
    finally:
        solo.close()
    eng = nydus_gpu.Engine(device=0, digester="blake3", chunk_size=S, staging_bytes=4 << 20)
    got = [None] * len(tars)
    errs = []
    start = threading.Barrier(len(tars))

    def run(i):
        try:
            start.wait()
            for _ in range(2):
                got[i] = _pack(eng, tars[i], compressor)
        except Exception as ex:  # reported below
            errs.append((i, ex))

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(tars))]
    try:
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in th)
    finally:
        eng.close()
    assert not errs, errs
    for i, tb in enumerate(tars):
        ch, rs, st, blob = got[i]
        ach, ars, ast, ablob = alone[i]
        assert ch.tobytes() == ach.tobytes(), i
        assert rs.tobytes() == ars.tobytes(), i
        assert st == ast, i
        assert blob == ablob, i
        ref = oracle.tar_chunks(tb, S)
        dig = oracle.digest_chunks(tb, ref, "blake3")
        dec, _ = oracle.dedup(dig, ref["length"])
        assert np.array_equal(rs["digest"], dig), i
        for f in FIELDS:
            assert np.array_equal(rs[f], dec[f]), (i, f)


def test_ws_slots_env_is_validated(monkeypatch):
    """NGPU_WS_SLOTS outside 1..64 falls back to the default (the engine is
    still created and works)."""
    import nydus_gpu
    S = 64 << 10
    L = _layer(5, 64, S)
    for v in ("0", "65", "x"):
        monkeypatch.setenv("NGPU_WS_SLOTS", v)
        eng = nydus_gpu.Engine(device=0, digester="blake3", chunk_size=S)
        try:
            out = torch.zeros(L["P"] * 64, dtype=torch.uint8, device="cuda")
            eng.process_device(L["d_data"].data_ptr(), L["d_data"].numel(), L["d_ch"].data_ptr(),
                               L["P"], out.data_ptr())
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
            assert np.array_equal(got["digest"], L["dig"]), v
        finally:
            eng.close()
    os.environ.pop("NGPU_WS_SLOTS", None)
