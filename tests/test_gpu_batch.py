"""Concurrent small Packs closed as ONE launch set (csrc/batch.hip, VERDICT
r4 item 3): containerd converting an image's layers concurrently, one
LayerConvertFunc per layer (pkg/converter/convert_unix.go:467-538, :822),
through one engine.  Every pack of a batch must give exactly its own layer's
oracle decisions (per-layer semantics inside the multi-layer dedup), with
and without a chunk dict, for blake3 and sha256, and a batched pack's nydus
stream must equal the unbatched one (NGPU_FLAG_NO_BATCH)."""
import io
import threading

import numpy as np
import pytest

import layers
import nydus_gpu
from nydus_gpu import rafs

pytestmark = pytest.mark.gpu

FIELDS = ("kind", "index", "ref", "blob_index", "uncompressed_offset")


def _run_packs(eng, tars, dict_=nydus_gpu.DEFAULT_DICT, out=None, compressor="zstd"):
    """One thread per tar: open, write in 1 MiB pieces, meet at a barrier,
    close together.  -> [(chunks, results, stats, stream bytes)]"""
    K = len(tars)
    res = [None] * K
    errs = []
    meet = threading.Barrier(K)

    def one(i):
        try:
            w = eng.pack(retain=out is not None, dict=dict_)
            sink = io.BytesIO() if out is not None else None
            if sink is not None:
                w.set_output(sink, compressor=compressor)
            t = tars[i]
            for a in range(0, len(t), 1 << 20):
                w.write(t[a:a + (1 << 20)])
            meet.wait()
            if sink is not None:
                ch, rs, st, _ = w.finish(None)
            else:
                ch, rs, st = w.close()
            res[i] = (ch, rs, st, sink.getvalue() if sink is not None else None)
        except Exception as ex:  # reported below
            errs.append(repr(ex))
            meet.abort()
    th = [threading.Thread(target=one, args=(i,)) for i in range(K)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    return res


def _check(oracle, tar, chunk, digester, got, recs=None):
    ch, rs = got[0], got[1]
    ref_ch = oracle.tar_chunks(tar, chunk)
    assert ch.tobytes() == ref_ch.tobytes()
    dig = oracle.digest_chunks(tar, ref_ch, digester)
    kw = {}
    if recs is not None:
        kw = dict(dict_digests=recs["block_id"], dict_sizes=recs["uncompressed_size"],
                  dict_blob=recs["blob_index"], dict_index=recs["index"],
                  dict_uoff=recs["uncompressed_offset"])
    dec, _ = oracle.dedup(dig, ref_ch["length"], **kw)
    assert np.array_equal(rs["digest"], dig)
    for f in FIELDS:
        assert np.array_equal(rs[f], dec[f]), f
    return dec


@pytest.mark.parametrize("digester", ["blake3", "sha256"])
def test_32_concurrent_c1_packs_share_launch_sets(oracle, digester):
    """32 distinct alpine-like (C1-size) layers, closed at once on one engine:
    the closes coalesce into batched launch sets, every layer equals the
    oracle, per-layer NEW numbering and offsets included."""
    S = 0x100000
    tars = [layers.alpine_like_tar(0xA1F1E + i) for i in range(32)]
    eng = nydus_gpu.Engine(device=0, digester=digester, chunk_size=S, staging_bytes=16 << 20)
    try:
        got = _run_packs(eng, tars)
        bs = eng.batch_stats()
    finally:
        eng.close()
    for t, g in zip(tars, got):
        _check(oracle, t, S, digester, g)
    assert bs["packs"] >= 2 and bs["max_packs"] >= 2, bs  # closes really coalesced
    assert bs["packs"] <= 32


def _big_layer(seed):
    """~49 MiB (one 64 MiB staging slot): two 20 MiB files (one shared by every layer: per-layer NEW
    semantics across a batch), 300 small files with in-layer duplicates."""
    rng = np.random.default_rng(seed)
    shared = np.random.default_rng(1).integers(0, 256, 20 << 20, dtype=np.uint8).tobytes()
    t = layers._TarBuilder()
    t.dir("d")
    t.file("d/shared.bin", shared)
    t.file("d/own.bin", rng.integers(0, 256, 20 << 20, dtype=np.uint8).tobytes())
    small = [rng.integers(0, 256, int(rng.integers(1, 60_000)), dtype=np.uint8).tobytes()
             for _ in range(150)]
    for i in range(300):
        t.file(f"d/s{i}", small[i % 150])
    return t.bytes()


def test_sha256_batch_beyond_one_gib(oracle):
    """24 layers of ~49 MiB (1.15 GiB) closed together on a sha256 engine:
    batches may now hold 2 GiB (csrc/batch.hip kMaxBytes), so a launch set
    can cover more than 1 GiB of gathered layers (r5x2: one batch of all 24,
    1.14 GiB).  Every layer equals the oracle."""
    S = 0x100000
    tars = [_big_layer(0xB16 + i) for i in range(24)]
    eng = nydus_gpu.Engine(device=0, digester="sha256", chunk_size=S, staging_bytes=64 << 20)
    try:
        got = _run_packs(eng, tars)
        bs = eng.batch_stats()
    finally:
        eng.close()
    for t, g in zip(tars, got):
        _check(oracle, t, S, "sha256", g)
    print("batch_stats", bs, "layer MiB", round(len(tars[0]) / 2**20, 1))
    assert bs["packs"] >= 2 and bs["max_packs"] >= 2, bs


def test_batched_packs_against_a_chunk_dict(oracle, tars):
    """The same layer set against one ChunkDict (records of a packed layer,
    planted into half of the others): DICT decisions, blob order and the
    dict's first-row rule per layer inside the batch."""
    S = 0x10000
    eng = nydus_gpu.Engine(device=0, chunk_size=S)
    try:
        base = layers.alpine_like_tar(0xBEEF)
        ch, out, _ = eng.pack_tar(base)
        recs = nydus_gpu.chunk_table(ch, out).view(rafs.CHUNK_INFO_DTYPE).reshape(-1).copy()
        recs["blob_index"] = np.arange(len(recs)) % 3
        d = eng.dict_create(recs, rafs.make_blob_table([f"{b:064x}" for b in range(3)], S))
        ts = [base if i % 2 == 0 else layers.alpine_like_tar(0x5EED + i) for i in range(12)]
        ts.append(tars["oci_lower"])
        got = _run_packs(eng, ts, dict_=d)
        bs = eng.batch_stats()
        d.release()
    finally:
        eng.close()
    for i, (t, g) in enumerate(zip(ts, got)):
        dec = _check(oracle, t, S, "blake3", g, recs)
        if i % 2 == 0 and i < 12:  # the dict's own layer: every chunk a DICT hit
            assert (dec["kind"] == nydus_gpu.DICT).all()
    assert bs["max_packs"] >= 2, bs


def test_batched_stream_equals_unbatched():
    """converter.Pack with early emission (set_output, zstd): the nydus
    stream of every batched pack equals the stream the same tar gives with
    NGPU_FLAG_NO_BATCH (same chunk list, digests, blob, bootstrap, TOC)."""
    S = 0x100000
    tars = [layers.alpine_like_tar(0x7A + i) for i in range(8)]
    streams = {}
    for name, flags in (("batched", 0), ("unbatched", nydus_gpu.FLAG_NO_BATCH)):
        eng = nydus_gpu.Engine(device=0, chunk_size=S, flags=flags, staging_bytes=16 << 20)
        try:
            got = _run_packs(eng, tars, out=True)
            streams[name] = [g[3] for g in got]
            streams[name + "_stats"] = eng.batch_stats()
        finally:
            eng.close()
    assert streams["unbatched_stats"]["packs"] == 0
    assert streams["batched_stats"]["max_packs"] >= 2, streams["batched_stats"]
    for a, b in zip(streams["batched"], streams["unbatched"]):
        assert a == b


def test_native_threads_drive_concurrent_packs(oracle):
    """tools/packs_drive.cpp (bench.py --packs's caller: K native threads, one
    Pack each, as cgo goroutines would): decisions and early-emission streams
    of 8 concurrent layers, fed by Write and by ReadFrom (reserve / commit),
    on one engine and on a 2-part node (least-loaded placement: both parts take Packs),
    counted per layer, equal the oracle's."""
    import ctypes
    import os
    lib_path = os.path.join(os.path.dirname(nydus_gpu._lib.LIB_PATH), "build", "libpacks_drive.so")
    drive = ctypes.CDLL(lib_path).packs_drive
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    drive.argtypes = [vp, u32, ctypes.POINTER(vp), ctypes.POINTER(u64), u64, u32, u32, u32, u32,
                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64),
                      ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, u64, vp,
                      ctypes.POINTER(ctypes.c_int32)]
    S, K = 0x100000, 8
    tars = [np.frombuffer(layers.alpine_like_tar(0xD0 + i), np.uint8) for i in range(K)]
    want = []
    for t in tars:
        ch = oracle.tar_chunks(t.tobytes(), S)
        dec, _ = oracle.dedup(oracle.digest_chunks(t.tobytes(), ch, "blake3"), ch["length"])
        want.append(np.bincount(dec["kind"], minlength=3)[:3])
    for mode in (0, 1, 2, 3):  # bit 0: stream, bit 1: ReadFrom feed
        for on_node in (False, True):
            node = nydus_gpu.Node([0, 0], chunk_size=S, staging_bytes=16 << 20) if on_node else None
            eng = None if on_node else nydus_gpu.Engine(device=0, chunk_size=S, staging_bytes=16 << 20)
            part = (ctypes.c_int32 * K)()
            try:
                rs = (ctypes.c_double * 3)()
                per = (u64 * (4 * K))()
                err = ctypes.create_string_buffer(256)
                rc = drive(None if on_node else eng._h, K, (vp * K)(*[t.ctypes.data for t in tars]),
                           (u64 * K)(*[t.size for t in tars]), 1 << 20, mode, 0, S, 3, rs, per, None,
                           err, 256, node._h if on_node else None, part)
                assert rc == 0, err.value
                engs = node.engines if on_node else [eng]
                bs = [e.batch_stats() for e in engs]
            finally:
                (node or eng).close()
            got = np.array(per, np.uint64).reshape(K, 4)
            for k in range(K):
                assert list(got[k, :3]) == list(want[k]), (mode, on_node, k)
                assert (got[k, 3] > 0) == (mode & 1 == 1)
            assert all(x > 0 for x in rs)
            assert sum(b["packs"] for b in bs) >= 2, bs
            if on_node:  # placement follows load (open Packs per engine): not an exact split
                placed = np.bincount(np.array(part), minlength=2).tolist()
                assert len(placed) == 2 and min(placed) > 0 and sum(placed) == K, list(part)


@pytest.mark.parametrize("digester", ["blake3", "sha256"])
def test_batch_lanes_stress_timed_engine(oracle, digester):
    """32 native threads, 4 rounds each of decisions then streams, on ONE
    timed engine (NGPU_FLAG_TIMING, as bench.py --packs): batches on the 4
    lanes overlap, lanes are freed by the first pack back and retaken.  Every
    layer's NEW / INTRA / DICT counts equal the oracle's in every mode (a lane
    freed under its running batch once faulted exactly here, r5n)."""
    import ctypes
    import os
    lib_path = os.path.join(os.path.dirname(nydus_gpu._lib.LIB_PATH), "build", "libpacks_drive.so")
    drive = ctypes.CDLL(lib_path).packs_drive
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    drive.argtypes = [vp, u32, ctypes.POINTER(vp), ctypes.POINTER(u64), u64, u32, u32, u32, u32,
                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64),
                      ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, u64, vp,
                      ctypes.POINTER(ctypes.c_int32)]
    S, K, R = 0x100000, 32, 4
    tars = [np.frombuffer(layers.alpine_like_tar(0x5150 + i), np.uint8) for i in range(K)]
    want = []
    for t in tars:
        ch = oracle.tar_chunks(t.tobytes(), S)
        dec, _ = oracle.dedup(oracle.digest_chunks(t.tobytes(), ch, digester), ch["length"])
        want.append(list(np.bincount(dec["kind"], minlength=3)[:3]))
    eng = nydus_gpu.Engine(device=0, digester=digester, chunk_size=S, timing=True,
                           staging_bytes=16 << 20)
    try:
        for mode in (0, 1):
            rs = (ctypes.c_double * R)()
            per = (u64 * (4 * K))()
            err = ctypes.create_string_buffer(256)
            rc = drive(eng._h, K, (vp * K)(*[t.ctypes.data for t in tars]),
                       (u64 * K)(*[t.size for t in tars]), 1 << 20, mode | 2,
                       nydus_gpu._lib.DIGESTERS[digester], S, R, rs, per, None, err, 256, None, None)
            assert rc == 0, err.value
            got = np.array(per, np.uint64).reshape(K, 4)
            for k in range(K):
                assert list(got[k, :3]) == want[k], (mode, k)
        bs = eng.batch_stats()
    finally:
        eng.close()
    assert bs["packs"] >= 2 * K and bs["batches"] >= 2, bs


def test_batch_per_layer_error_words():
    """a batched launch set's error words go only to the layer that
    raised them, with its own chunk id (tests/cpp/batch_stats_test.hip runs
    csrc/batch_stats.hpp's kernel on a 3-layer set with one faulty layer)."""
    import os
    import subprocess
    from conftest import ROOT
    exe = os.path.join(ROOT, "nydus-snapshotter_amd", "build", "batch_stats_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "PASS", r.stdout + r.stderr


def test_batch_leader_waits_only_for_packs_that_can_join(oracle):
    """a batch leader waits for the open packs that may still join
    (engine counter batch_waitable): a pack whose tar outgrew one staging slot
    leaves the count at that moment, an OCIRef pack never enters it, and each
    pack leaves it when it ends; the small packs still batch and still equal
    the oracle."""
    cs = 0x10000
    eng = nydus_gpu.Engine(chunk_size=cs, staging_bytes=4 << 20)
    try:
        base = eng.counters()
        assert base["open_packs"] == 0 and base["batch_waitable"] == 0
        big = eng.pack()
        small = [eng.pack() for _ in range(3)]
        assert eng.counters()["batch_waitable"] == 4
        tar_big = layers.alpine_like_tar()  # 10 MB > one 4 MiB slot
        big.write(tar_big)
        c = eng.counters()
        assert c["open_packs"] == 4 and c["batch_waitable"] == 3
        tars = [layers.oci_upper_tar(), layers.oci_lower_tar(), layers.chunk_dict_tar()]
        got = [None] * 3
        meet = threading.Barrier(3)

        def one(i):
            small[i].write(tars[i])
            meet.wait()
            got[i] = small[i].close()
        th = [threading.Thread(target=one, args=(i,)) for i in range(3)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for t, g in zip(tars, got):
            _check(oracle, t, cs, "blake3", g)
        assert eng.batch_stats()["max_packs"] >= 2
        assert eng.counters()["batch_waitable"] == 0
        gb = big.close()
        _check(oracle, tar_big, cs, "blake3", gb)
        end = eng.counters()
        assert end["open_packs"] == 0 and end["batch_waitable"] == 0
    finally:
        eng.close()
