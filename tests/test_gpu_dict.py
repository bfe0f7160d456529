"""GPU: per-Pack chunk-dict handles (PackOption.ChunkDictPath,
pkg/converter/tool/builder.go:122-124), their compatibility checks, lifetimes
and cancellation, and BASELINE configs[2] (C3: sha256 digester against a chunk
dict in HBM) -- every decision bit-exact against the CPU oracle."""
import os
import threading
import time

import numpy as np
import pytest

import nydus_gpu
from nydus_gpu import rafs

pytestmark = pytest.mark.gpu

FLAG_BLAKE3, FLAG_SHA256 = 0x4, 0x8  # RafsSuperFlags HASH_*


def _pack_records(eng, tar):
    """Pack a tar with no dict -> (chunk records of its own blob, blob table)."""
    ch, out, st = eng.pack_tar(tar)
    tab = nydus_gpu.chunk_table(ch, out).view(rafs.CHUNK_INFO_DTYPE).reshape(-1)
    return tab


def _bootstrap(path, recs, chunk_size, digester="blake3", n_blobs=None):
    nb = int(recs["blob_index"].max()) + 1 if len(recs) else 1
    blobs = rafs.make_blob_table([f"{i:064x}" for i in range(n_blobs or nb)], chunk_size,
                                 digester=digester)
    flags = (FLAG_SHA256 if digester == "sha256" else FLAG_BLAKE3) | 0x1
    with open(path, "wb") as f:
        f.write(rafs.write_v6_bootstrap(recs, chunk_size, flags=flags, blobs=blobs))
    return blobs


def _oracle_expect(oracle, tar, chunk, digester, recs=None):
    ch = oracle.tar_chunks(tar, chunk)
    dig = oracle.digest_chunks(tar, ch, digester)
    kw = {}
    if recs is not None:
        kw = dict(dict_digests=recs["block_id"], dict_sizes=recs["uncompressed_size"],
                  dict_blob=recs["blob_index"], dict_index=recs["index"],
                  dict_uoff=recs["uncompressed_offset"])
    dec, own = oracle.dedup(dig, ch["length"], **kw)
    return ch, dig, dec


def _same(out, dig, dec, what=""):
    assert np.array_equal(out["digest"], dig), what
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        assert np.array_equal(out[f], dec[f]), (what, f)


def test_two_packs_with_different_dicts_open_at_once(tars, oracle, tmp_path):
    """Packs on ONE engine with dict P1, dict P2 and no dict, writes
    interleaved, plus a pack that captured the default dict while the default
    is replaced: each equals the oracle against its own dict (the reference
    runs one nydus-image per Pack, convert_unix.go:467-538)."""
    cs = 0x10000
    eng = nydus_gpu.Engine(chunk_size=cs, staging_bytes=4 * cs)
    try:
        r1 = _pack_records(eng, tars["chunk_dict"])
        # P2: every other record of P1, in a second inner blob at other offsets
        r2 = r1[::2].copy()
        r2["blob_index"] = 1
        r2["index"] += 5000
        r2["uncompressed_offset"] += 1 << 30
        p1, p2 = str(tmp_path / "p1"), str(tmp_path / "p2")
        _bootstrap(p1, r1, cs)
        _bootstrap(p2, r2, cs, n_blobs=2)
        d1, d2 = eng.dict_open(p1), eng.dict_open(p2)
        assert d1.entries == len(r1) and d2.entries == len(r2)
        eng.set_dict(d1)
        wd = eng.pack()  # captures the default (d1) now
        eng.dict_load_bootstrap(p2)  # replacing the default must not touch wd
        ws = [(eng.pack(dict=d1), r1), (eng.pack(dict=d2), r2), (eng.pack(dict=None), None), (wd, r1)]
        d1.release()
        d2.release()  # the packs hold their own references
        tar = tars["oci_lower"] + b""
        rng = np.random.default_rng(3)
        pos = 0
        while pos < len(tar):
            k = int(rng.integers(1, 150_000))
            for w, _ in ws:
                w.write(tar[pos:pos + k])
            pos += k
        for i, (w, recs) in enumerate(ws):
            ch, out, st = w.close()
            ech, dig, dec = _oracle_expect(oracle, tar, cs, "blake3", recs)
            assert ch.tobytes() == ech.tobytes()
            _same(out, dig, dec, i)
            if recs is not None:
                assert st["dict_chunks"] == int((dec["kind"] == 2).sum()) > 0
            else:
                assert st["dict_chunks"] == 0
        # the default now is P2
        ch, out, _ = eng.pack_tar(tar)
        _same(out, *_oracle_expect(oracle, tar, cs, "blake3", r2)[1:], "default P2")
    finally:
        eng.close()


def test_dict_open_is_cached_per_unchanged_file(tars, oracle, tmp_path):
    """1000 Packs against one ChunkDictPath load it once: ngpu_dict_open of an
    unchanged file returns the same dict; a rewritten file is loaded anew."""
    from nydus_gpu import converter as cv
    cs = 0x10000
    eng = nydus_gpu.Engine(chunk_size=cs)
    try:
        recs = _pack_records(eng, tars["chunk_dict"])
        path = str(tmp_path / "dict")
        _bootstrap(path, recs, cs)
        a = eng.dict_open(path)
        handles = {a.handle}
        for _ in range(50):
            d = eng.dict_open(path)
            handles.add(d.handle)
            d.release()
        assert handles == {a.handle}
        time.sleep(0.01)
        r2 = recs[: len(recs) // 2].copy()
        _bootstrap(path, r2, cs)
        b = eng.dict_open(path)
        assert b.handle != a.handle and b.entries == len(r2) and a.entries == len(recs)
        a.release()
        b.release()
    finally:
        eng.close()
    # through the converter mirror: many Packs, one dict load
    _bootstrap(path, recs, cs)
    opt = cv.PackOption(ChunkDictPath=path, ChunkSize=hex(cs), Compressor="none")
    import io
    first = None
    for i in range(200):
        out = io.BytesIO()
        w = cv.Pack(out, opt)
        w.write(tars["oci_lower"])
        res = w.close()
        if first is None:
            first = out.getvalue()
        assert out.getvalue() == first
        assert (res["results"]["kind"] == nydus_gpu.DICT).all()
    e = cv._engine(opt)
    d = e.dict_open(path)
    try:
        again = e.dict_open(path)
        assert again.handle == d.handle
        again.release()
    finally:
        d.release()


def test_dict_reload_does_not_stall_concurrent_packs(tars, oracle, tmp_path):
    """A thread rewrites the ChunkDictPath file and reopens it (a 2M-entry
    bootstrap: parse, upload and table build) while 3 threads run Packs on the
    same engine against the dict they opened first.  Every Pack equals the
    oracle, and Pack closes complete while a reload is in flight: the load runs
    outside the engine lock on its own stream (round 3 held e->mu across it and
    its stream syncs)."""
    cs = 0x10000
    eng = nydus_gpu.Engine(chunk_size=cs)
    try:
        recs = _pack_records(eng, tars["chunk_dict"])
        rng = np.random.default_rng(11)

        def with_filler(seed):
            f = np.zeros(2_000_000, dtype=recs.dtype)
            f["block_id"] = np.random.default_rng(seed).integers(0, 256, (len(f), 32), dtype=np.uint8)
            f["uncompressed_size"] = cs
            f["index"] = np.arange(len(f), dtype=np.uint32) + 100_000
            return np.concatenate([recs, f])

        path = str(tmp_path / "dict")
        _bootstrap(path, with_filler(1), cs)
        d0 = eng.dict_open(path)
        tar = tars["oci_lower"]
        _, dig, dec = _oracle_expect(oracle, tar, cs, "blake3", recs)
        stop = threading.Event()
        reloads, closes, errors = [], [], []

        def reloader():
            try:
                k = 2
                while not stop.is_set() and len(reloads) < 6:
                    _bootstrap(path, with_filler(k), cs)
                    t0 = time.monotonic()
                    d = eng.dict_open(path)
                    reloads.append((t0, time.monotonic()))
                    assert d.entries == len(recs) + 2_000_000
                    d.release()
                    k += 1
            except Exception as ex:  # pragma: no cover - reported below
                errors.append(repr(ex))

        def packer(i):
            try:
                r = np.random.default_rng(100 + i)
                while not stop.is_set():
                    w = eng.pack(dict=d0)
                    pos = 0
                    while pos < len(tar):
                        k = int(r.integers(1, 300_000))
                        w.write(tar[pos:pos + k])
                        pos += k
                    t0 = time.monotonic()
                    ch, out, st = w.close()
                    closes.append((t0, time.monotonic()))
                    _same(out, dig, dec, f"packer {i}")
            except Exception as ex:  # pragma: no cover - reported below
                errors.append(repr(ex))

        ts = [threading.Thread(target=packer, args=(i,)) for i in range(3)]
        rt = threading.Thread(target=reloader)
        for t in ts:
            t.start()
        rt.start()
        rt.join(timeout=90)
        stop.set()
        for t in ts:
            t.join(timeout=30)
        d0.release()
        assert not errors, errors
        assert not rt.is_alive() and not any(t.is_alive() for t in ts)
        assert len(reloads) == 6 and len(closes) >= 6
        inside = sum(1 for a, b in closes for r0, r1 in reloads if r0 <= a and b <= r1)
        longest = max(b - a for a, b in reloads)
        print(f"reloads {len(reloads)} (longest {longest * 1e3:.0f} ms), closes {len(closes)}, "
              f"{inside} completed inside a reload")
        assert inside >= 1, "every Pack close waited for the dict reload"
    finally:
        eng.close()


def test_incompatible_dict_is_rejected(tars, tmp_path):
    """nydus-image rejects a chunk-dict bootstrap whose digester / chunk size /
    RAFS version differs from the build's ([nydus v2.3.0]
    RafsSuperConfig::check_compatibility, VERIFY): NGPU_EINVAL here."""
    cs = 0x10000
    eng = nydus_gpu.Engine(chunk_size=cs)
    try:
        recs = _pack_records(eng, tars["chunk_dict"])
    finally:
        eng.close()
    pb, ps = str(tmp_path / "b3"), str(tmp_path / "sha")
    _bootstrap(pb, recs, cs, "blake3")
    _bootstrap(ps, recs, cs, "sha256")
    cases = [(dict(digester="sha256", chunk_size=cs), pb),
             (dict(digester="blake3", chunk_size=cs), ps),
             (dict(digester="blake3", chunk_size=0x20000), pb),
             (dict(digester="blake3", chunk_size=cs, fs_version=5), pb)]
    for kw, path in cases:
        e = nydus_gpu.Engine(**kw)
        try:
            with pytest.raises(nydus_gpu.NgpuError) as x:
                e.dict_open(path)
            assert x.value.code == nydus_gpu.EINVAL, kw
            with pytest.raises(nydus_gpu.NgpuError):
                e.dict_load_bootstrap(path)
        finally:
            e.close()
    # a dict opened on one engine cannot serve a pack of an incompatible one
    a = nydus_gpu.Engine(chunk_size=cs)
    b = nydus_gpu.Engine(chunk_size=cs, digester="sha256")
    try:
        d = a.dict_open(pb)
        with pytest.raises(nydus_gpu.NgpuError):
            b.pack(dict=d)
        with pytest.raises(nydus_gpu.NgpuError):
            b.set_dict(d)
        w = nydus_gpu.Engine.pack(a, dict=d)  # fine on its own engine
        w.write(tars["oci_lower"])
        assert (w.close()[1]["kind"] == nydus_gpu.DICT).all()
        d.release()
    finally:
        a.close()
        b.close()


def test_engine_destroyed_with_pack_open(tars, oracle):
    """ngpu_destroy with packs still open only drops the creator's reference:
    the packs finish normally and free the engine last."""
    import io
    cs = 0x10000
    eng = nydus_gpu.Engine(chunk_size=cs, staging_bytes=4 * cs)
    w = eng.pack(retain=True)
    w2 = eng.pack()
    tar = tars["oci_upper"]
    w.write(tar[: len(tar) // 3])
    eng.close()
    w.write(tar[len(tar) // 3:])
    w2.write(tar)
    out = io.BytesIO()
    ch, res, st, info = w.finish(out, compressor="none")
    ech, dig, dec = _oracle_expect(oracle, tar, cs, "blake3")
    _same(res, dig, dec)
    w2.abort()


def test_pack_cancel_and_timeout(tars):
    """ctx.Done() / PackOption.Timeout: a cancelled pack fails with
    ECANCELED at its next write or in close (builder.go:153-174)."""
    import io
    from nydus_gpu import converter as cv
    eng = nydus_gpu.Engine(chunk_size=0x10000, staging_bytes=1 << 20)
    try:
        w = eng.pack()
        w.write(tars["oci_upper"][:100_000])
        w.cancel()
        with pytest.raises(nydus_gpu.NgpuError) as x:
            w.write(tars["oci_upper"][100_000:])
        assert x.value.code == nydus_gpu.ECANCELED
        w = eng.pack(retain=True)
        w.write(tars["oci_upper"])
        w.cancel()
        with pytest.raises(nydus_gpu.NgpuError) as x:
            w.finish(io.BytesIO())
        assert x.value.code == nydus_gpu.ECANCELED
        # cancelled from another thread while the writer is busy
        big = tars["oci_upper"] * 20
        w = eng.pack()
        t = threading.Timer(0.05, w.cancel)
        t.start()
        with pytest.raises(nydus_gpu.NgpuError) as x:
            for _ in range(200):
                w.write(big)
        assert x.value.code == nydus_gpu.ECANCELED
        t.join()
        ch, out, st = eng.pack_tar(tars["oci_lower"])  # the engine is fine
        assert st["chunks"] == len(ch) > 0
    finally:
        eng.close()
    w = cv.Pack(io.BytesIO(), cv.PackOption(ChunkSize="0x10000", Timeout=0.05))
    time.sleep(0.2)
    with pytest.raises(cv.ConverterError, match="signal: killed"):
        w.write(tars["oci_upper"])
        w.close()
    w = cv.Pack(io.BytesIO(), cv.PackOption(ChunkSize="0x10000", Timeout=30))
    w.write(tars["oci_upper"])
    assert w.close()["stats"]["chunks"] > 0


def _random_layer(rng, total, chunk_size):
    data = rng.integers(0, 256, total, dtype=np.uint8)
    chunks, off = [], 0
    while True:
        ln = int(rng.integers(1, chunk_size + 1)) if rng.random() < 0.3 else chunk_size
        if off + ln > total:
            break
        chunks.append((off, ln, len(chunks), 0))
        off = (off + ln + 511) // 512 * 512
    return data, np.array(chunks, dtype=nydus_gpu.CHUNK_DTYPE)


@pytest.mark.parametrize("m", [1_200_000, 4_000_000])
def test_c3_sha256_dict_bootstrap_1m_entries_vs_oracle(oracle, tmp_path, m):
    """BASELINE configs[2] shape at test size: sha256 digester, 1 MiB chunks,
    a chunk dict of >= 1M entries loaded from a sha256 RAFS v6 bootstrap (4M
    entries = 320 MB of chunk table: the streamed load, csrc/dict.hip
    dict_stream_v6, four 1M-record pieces; the later duplicates sit in
    other pieces than their first rows), with
    planted layer digests, keys duplicated later in the table (first wins),
    usize == 0 wildcards, size mismatches (miss) and 9 inner blobs; every
    decision, index, offset and blob equals the oracle's."""
    S = 0x100000
    rng = np.random.default_rng(0xC3)
    data, ch = _random_layer(rng, 192 << 20, S)
    dup = rng.choice(len(ch), len(ch) // 5, replace=False)  # intra-layer duplicates
    for i in dup:
        j = int(rng.integers(0, len(ch)))
        ln = min(int(ch["length"][i]), int(ch["length"][j]))
        ch["length"][i] = ln
        data[ch["offset"][i]:ch["offset"][i] + ln] = data[ch["offset"][j]:ch["offset"][j] + ln]
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "sha256")
    recs = np.zeros(m, rafs.CHUNK_INFO_DTYPE)
    recs["block_id"] = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    recs["uncompressed_size"] = S
    recs["blob_index"] = rng.integers(0, 9, m)
    recs["index"] = np.arange(m)
    recs["uncompressed_offset"] = np.arange(m, dtype=np.uint64) * S
    recs["compressed_size"] = S
    recs["compressed_offset"] = np.arange(m, dtype=np.uint64) * S
    n = len(ch)
    pick = rng.choice(n, n // 2, replace=False)
    rows = rng.choice(m, len(pick) + 40, replace=False)
    recs["block_id"][rows[: len(pick)]] = dig[pick]
    recs["uncompressed_size"][rows[: len(pick)]] = ch["length"][pick]
    wild, bad = rows[:10], rows[10:20]
    recs["uncompressed_size"][wild] = 0           # wildcard size
    recs["uncompressed_size"][bad] += 1           # size mismatch: a miss
    later = np.sort(rng.choice(np.arange(m // 2, m), 30, replace=False))
    src = pick[:30]
    recs["block_id"][later] = dig[src]            # duplicate keys: the first entry wins
    recs["uncompressed_size"][later] = ch["length"][src]
    path = str(tmp_path / "c3-dict")
    _bootstrap(path, recs, S, "sha256", n_blobs=9)
    exp, own = oracle.dedup(dig, ch["length"], recs["block_id"], recs["uncompressed_size"],
                            recs["blob_index"], recs["index"], dict_uoff=recs["uncompressed_offset"])
    assert (exp["kind"] == 2).sum() > n // 3 and (exp["kind"] == 1).sum() > 0
    for fl in (0, 1 << 11, 2 << 11):
        eng = nydus_gpu.Engine(digester="sha256", chunk_size=S, flags=fl)
        try:
            d = eng.dict_open(path)
            assert d.entries == m
            out, st = eng.process(data, ch, dict=d)
            d.release()
        finally:
            eng.close()
        _same(out, dig, exp, fl)
        assert st["dict_chunks"] == int((exp["kind"] == 2).sum())
        assert st["blobs"] == len(set(exp["blob_index"].tolist()))


def test_c3_200m_entry_device_dict_properties(oracle):
    """BASELINE configs[2] at full dict size: a 200,000,000-entry chunk dict
    built in HBM (2^29 slots), probed by a sha256 layer (1 GiB here) --
    size-independent properties: every planted chunk is DICT with ref = its
    FIRST table row (a key planted twice resolves to the earlier row), copied
    index / uncompressed offset; unplanted chunks are NEW; sampled digests
    equal the oracle's."""
    import torch
    S = 0x100000
    n = 1024
    g = torch.Generator(device="cuda").manual_seed(0xD1C7)
    d_data = torch.randint(0, 256, (n * S,), dtype=torch.uint8, device="cuda", generator=g)
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    ch["offset"] = np.arange(n, dtype=np.uint64) * S
    ch["length"] = S
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    m = 200_000_000
    eng = nydus_gpu.Engine(digester="sha256", chunk_size=S)
    try:
        eng.digest_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), n, d_out.data_ptr())
        torch.cuda.synchronize()
        dig = d_out.view(n, 64)[:, :32].clone()
        dd = torch.empty((m, 32), dtype=torch.uint8, device="cuda")
        dd.random_(0, 256, generator=g)
        planted = np.arange(0, n, 2)                         # even chunks planted
        rows = torch.randperm(m, device="cuda", generator=g)[: len(planted) + 64]
        prow = rows[: len(planted)]
        dd[prow] = dig[torch.from_numpy(planted).cuda()]
        twice = rows[len(planted):]                          # chunk 0..63 planted again
        earlier = prow[:32] > twice[:32]
        dd[twice[:32]] = dig[torch.from_numpy(planted[:32]).cuda()]
        us = torch.full((m,), S, dtype=torch.int32, device="cuda")
        bl = torch.zeros(m, dtype=torch.int32, device="cuda")
        ix = torch.arange(m, dtype=torch.int32, device="cuda")
        uo = torch.arange(m, dtype=torch.int64, device="cuda") * 4096
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = eng.dict_create_device(dd.data_ptr(), us.data_ptr(), bl.data_ptr(), ix.data_ptr(), m, 1,
                                   d_uoff=uo.data_ptr())
        build_s = time.perf_counter() - t0
        del dd, us, bl, ix, uo
        torch.cuda.empty_cache()
        assert d.entries == m
        st = eng.process_dict_device(d, d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), n,
                                     d_out.data_ptr(), want_stats=True)
        d.release()
    finally:
        eng.close()
    out = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
    prow = prow.cpu().numpy().astype(np.int64)
    twice = twice.cpu().numpy().astype(np.int64)
    earlier = earlier.cpu().numpy()
    first = prow.copy()
    first[:32] = np.where(earlier, twice[:32], prow[:32])  # the earlier row of a key planted twice
    assert (out["kind"][planted] == nydus_gpu.DICT).all()
    assert np.array_equal(out["ref"][planted], first)
    assert np.array_equal(out["index"][planted], first)
    assert np.array_equal(out["uncompressed_offset"][planted], first * 4096)
    odd = np.arange(1, n, 2)
    assert (out["kind"][odd] == nydus_gpu.NEW).all()
    assert np.array_equal(out["index"][odd], np.arange(len(odd)))
    assert st["dict_chunks"] == len(planted) and st["new_chunks"] == len(odd)
    for i in np.random.default_rng(1).choice(n, 8, replace=False):
        blob = d_data[i * S:(i + 1) * S].cpu().numpy().tobytes()
        assert out["digest"][i].tobytes() == oracle.sha256(blob), i
    print(f"200M-entry dict built in {build_s:.3f} s")


def test_aligned_chunk_v5(oracle):
    """PackOption.AlignedChunk (types.go:73-74, --aligned-chunk): RAFS v5 NEW
    chunks at 4 KiB-aligned uncompressed offsets (v5 without it: packed)."""
    rng = np.random.default_rng(73)
    data, ch = _random_layer(rng, 8 << 20, 0x10000)
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    for aligned, align in ((True, 4096), (False, 1)):
        exp, _ = oracle.dedup(dig, ch["length"], align=align)
        eng = nydus_gpu.Engine(chunk_size=0x10000, fs_version=5, aligned_chunk=aligned)
        try:
            out, st = eng.process(data, ch)
        finally:
            eng.close()
        _same(out, dig, exp, aligned)


def test_probe_walks_tag_collisions_and_keeps_first_row():
    """The probe's record compare (dict_find, dedup.hip): entries sharing the
    bucket words AND the tag word (digest words 0-2) but not the rest sit in
    one probe chain with equal tags, so the probe must read and compare each
    record and walk past the unequal ones; a digest listed twice resolves to
    its earlier row (ht_insert_min; the oracle's first-occurrence rule,
    oracle_py.dedup); a query that shares words 0-2 with the chain but equals
    none of it walks the chain to the empty slot (a miss).  Expected values
    are computed here by a plain scan of the table rows."""
    import torch
    rng = np.random.default_rng(0x7A6)
    m = 4096
    dd = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    coll = [100, 200, 300, 400, 500, 600, 700, 800, 1000, 1100, 1200, 1300]
    for r in coll:
        dd[r, :12] = dd[100, :12]           # same bucket words and tag, tails differ
    dd[900] = dd[300]                        # a later duplicate: row 300 wins
    dd[50] = dd[700]                         # an earlier duplicate: row 50 wins
    miss_chain = dd[100].copy()
    miss_chain[12:] = rng.integers(0, 256, 20, dtype=np.uint8)
    near = dd[400].copy()
    near[31] ^= 1                            # equal in 31 bytes, bucket and tag included
    q = np.stack([dd[r] for r in coll] + [dd[900], dd[50], miss_chain, near] +
                 [rng.integers(0, 256, 32, dtype=np.uint8) for _ in range(8)] +
                 [dd[r] for r in rng.choice(m, 64, replace=False)])
    exp = []
    for row in q:
        eq = np.flatnonzero((dd == row).all(axis=1))
        exp.append(int(eq[0]) if len(eq) else nydus_gpu.MISS)
    exp = np.array(exp, np.uint32)
    idx = (np.arange(m, dtype=np.int32) * 7 + 3)
    usz = (np.arange(m, dtype=np.int32) % 5 + 1) * 4096
    blb = (np.arange(m, dtype=np.int32) % 3)
    d_dd = torch.from_numpy(dd).cuda()
    d_us, d_bl, d_ix = (torch.from_numpy(a).cuda() for a in (usz, blb, idx))
    d_q = torch.from_numpy(q).cuda()
    d_hits = torch.zeros(len(q) * 24, dtype=torch.uint8, device="cuda")
    eng = nydus_gpu.Engine(chunk_size=0x10000)
    try:
        torch.cuda.synchronize()             # the build reads the arrays from its own stream
        eng.dict_load_device(d_dd.data_ptr(), d_us.data_ptr(), d_bl.data_ptr(), d_ix.data_ptr(), m, 3)
        eng.dict_probe_device(d_q.data_ptr(), 32, len(q), d_hits.data_ptr(),
                              stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        eng.close()
    hits = d_hits.cpu().numpy().view(nydus_gpu.HIT_DTYPE)
    assert np.array_equal(hits["entry"], exp), (hits["entry"][:20], exp[:20])
    hit = exp != nydus_gpu.MISS
    assert hit.sum() == len(coll) + 2 + 64 and not hit[len(coll) + 2:len(coll) + 12].any()
    assert np.array_equal(hits["index"][hit], idx[exp[hit]].astype(np.uint32))
    assert np.array_equal(hits["usize"][hit], usz[exp[hit]].astype(np.uint32))
    assert np.array_equal(hits["blob"][hit], blb[exp[hit]].astype(np.uint32))
