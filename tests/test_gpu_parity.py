"""GPU parity: the HIP path (through the C ABI) against the golden fixtures
and the CPU oracle, bit-exact.  Run on a gfx950 box: pytest -m gpu."""
import os
import struct
import tempfile

import numpy as np
import pytest

import nydus_gpu
from nydus_gpu import rafs

from conftest import kat_input

import layers

pytestmark = pytest.mark.gpu

LANES = [1, 2, 4, 8, 16]
# SHA-256 kernels, forced through ngpu_config.flags bits 11..12 (1 + variant):
# 0 = auto, one lane per chunk ("split": schedule/round waves; "lane": one wave
# does both), two lanes per chunk ("pair").
# "pair" runs two chunk groups per workgroup; 5 forces one group, 6 four groups.
SHA_SPLIT, SHA_PAIR, SHA_LANE = 1 << 11, 2 << 11, 3 << 11
SHA_PAIR_R1, SHA_PAIR_R4 = 5 << 11, 6 << 11
SHA_FLAGS = [0, SHA_SPLIT, SHA_PAIR, SHA_LANE, SHA_PAIR_R1, SHA_PAIR_R4]
# Calls with <= 4096 chunks plan and dedup in one fused workgroup; this flag
# forces the multi-kernel grid path, so both are checked on the same inputs.
GRID = nydus_gpu.FLAG_GRID_STAGES


@pytest.fixture(scope="module")
def engines():
    cache = {}

    def get(digester="blake3", chunk_size=0x100000, lanes=0, fs_version=6, flags=0):
        k = (digester, chunk_size, lanes, fs_version, flags)
        if k not in cache:
            cache[k] = nydus_gpu.Engine(digester=digester, chunk_size=chunk_size,
                                        leaves_per_lane=lanes, fs_version=fs_version,
                                        flags=flags)
        return cache[k]
    yield get
    for e in cache.values():
        e.close()


def one_chunk(n, off=0):
    ch = np.zeros(1, nydus_gpu.CHUNK_DTYPE)
    ch["offset"], ch["length"] = off, n
    return ch


@pytest.mark.parametrize("digester", ["blake3", "sha256"])
def test_kat_single_chunk(engines, kat, digester):
    for lanes, fl in ([(l, 0) for l in LANES] if digester == "blake3" else
                      [(0, f) for f in SHA_FLAGS]):
        eng = engines(digester, 0x1000000, lanes, flags=fl)
        for v in kat["vectors"]:
            if v["len"] == 0:
                continue  # nydus never emits empty chunks
            out, st = eng.process(kat_input(v["len"]), one_chunk(v["len"]))
            assert out["digest"][0].tobytes().hex() == v[digester], (lanes, fl, v["len"])
            assert st["new_chunks"] == 1


def test_kat_batched_all_lengths(engines, kat):
    """All KAT inputs in ONE call, packed back to back at odd offsets."""
    vecs = [v for v in kat["vectors"] if v["len"]]
    parts, chunks, off = [], [], 0
    for v in vecs:
        pad = 7
        parts.append(b"\x55" * pad)
        off += pad
        parts.append(kat_input(v["len"]))
        chunks.append((off, v["len"], 0, 0))
        off += v["len"]
    data = b"".join(parts)
    ch = np.array(chunks, dtype=nydus_gpu.CHUNK_DTYPE)
    for digester in ("blake3", "sha256"):
        for lanes, fl in ([(l, 0) for l in LANES] if digester == "blake3" else
                          [(0, f) for f in SHA_FLAGS]) + [(0, GRID)]:
            out, _ = engines(digester, 0x1000000, lanes, flags=fl).process(data, ch)
            got = [o.tobytes().hex() for o in out["digest"]]
            assert got == [v[digester] for v in vecs], (digester, lanes, fl)


def _decisions(out):
    return [(int(o["kind"]), int(o["index"]), int(o["ref"]), int(o["blob_index"]),
             int(o["uncompressed_offset"])) for o in out]


def _expected(dec):
    kinds = {"NEW": 0, "INTRA": 1, "DICT": 2}
    return [(kinds[k], i, r, b, u) for (k, i, r, b, u) in dec]


def test_golden_layers(engines, golden_layers, tars):
    for case in golden_layers["cases"]:
        for lanes in (LANES if case["digester"] == "blake3" else [0]):
            eng = engines(case["digester"], case["chunk_size"], lanes)
            ch, out, st = eng.pack_tar(tars[case["layer"]])
            assert [tuple(int(x) for x in c) for c in ch] == [tuple(c) for c in case["chunks"]]
            got = [d.tobytes().hex() for d in out["digest"]]
            bad = [i for i, (g, x) in enumerate(zip(got, case["digests"])) if g != x]
            # the path that produced it (the r2end zero digest named only the layer)
            where = (f"{case['layer']} {case['digester']} chunk_size={case['chunk_size']:#x} "
                     f"leaves_per_lane={lanes} n={len(got)} bad={bad[:8]} "
                     f"kinds={[int(out['kind'][i]) for i in bad[:8]]} "
                     f"lengths={[int(ch['length'][i]) for i in bad[:8]]}")
            assert len(got) == len(case["digests"]) and not bad, where
            assert _decisions(out) == _expected(case["decisions"]), where
            own = st["own_blob_index"]
            assert (None if own == 0xFFFFFFFF else own) == case["own_blob"]


def _dict_arrays(tp):
    dd = np.frombuffer(b"".join(bytes.fromhex(e[0]) for e in tp["dict"]), np.uint8).reshape(-1, 32)
    return (dd, np.array([e[1] for e in tp["dict"]], np.uint32),
            np.array([e[2] for e in tp["dict"]], np.uint32), np.array([e[3] for e in tp["dict"]], np.uint32))


def test_testpack_with_chunk_dict(engines, golden_layers, tars):
    """tests/converter_test.go:459-528 outcome: lower all-DICT, upper own blob,
    merged blob list [dict, upper]."""
    tp = golden_layers["testpack"]
    eng = nydus_gpu.Engine(chunk_size=0x100000)
    try:
        eng.dict_load(*_dict_arrays(tp))
        assert eng.dict_size == len(tp["dict"])
        blobs = []
        for name, lay in tp["layers"].items():
            ch, out, st = eng.pack_tar(tars[name])
            assert _decisions(out) == _expected(lay["decisions"]), name
            for o in out:
                tag = "dict" if o["kind"] == nydus_gpu.DICT else name
                if tag not in blobs:
                    blobs.append(tag)
        assert blobs == tp["expected_blobs"]
    finally:
        eng.close()


def test_chunk_dict_bootstrap_roundtrip(tars, oracle):
    """Pack the dict layer, write its chunk table into a RAFS v6 bootstrap,
    load it as ChunkDictPath, pack the lower layer: every chunk is a DICT hit."""
    eng = nydus_gpu.Engine(chunk_size=0x1000)
    try:
        ch, out, _ = eng.pack_tar(tars["chunk_dict"])
        tab = nydus_gpu.chunk_table(ch, out)
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "dict-bootstrap")
            with open(p, "wb") as f:
                f.write(rafs.write_v6_bootstrap(tab.view(rafs.CHUNK_INFO_DTYPE).reshape(-1), 0x1000))
            eng.dict_load_bootstrap(p)
        ch2, out2, st2 = eng.pack_tar(tars["oci_lower"])
        assert (out2["kind"] == nydus_gpu.DICT).all()
        assert st2["own_blob_index"] == 0xFFFFFFFF and st2["blobs"] == 1
        # oracle agrees on every field
        dig = oracle.digest_chunks(tars["oci_lower"], ch2.view(oracle.CHUNK_DTYPE), "blake3")
        recs = tab.view(rafs.CHUNK_INFO_DTYPE).reshape(-1)
        dec, _ = oracle.dedup(dig, ch2["length"], recs["block_id"], recs["uncompressed_size"],
                              recs["blob_index"], recs["index"])
        assert np.array_equal(out2["digest"], dig)
        for f in ("kind", "index", "ref", "blob_index"):
            assert np.array_equal(out2[f], dec[f]), f
    finally:
        eng.close()


def _random_layer(rng, total, chunk_size, dup_frac=0.2, unaligned=False):
    """Random data + chunk list (random lengths, some duplicated contents)."""
    data = bytearray(rng.integers(0, 256, total, dtype=np.uint8).tobytes())
    chunks, off = [], 0
    while True:
        ln = int(rng.integers(1, chunk_size + 1)) if rng.random() < 0.5 else chunk_size
        if unaligned:
            off += int(rng.integers(0, 16))
        if off + ln > total:
            break
        chunks.append([off, ln, 0, 0])
        off += ln
        off = (off + 511) // 512 * 512 if not unaligned else off
    # plant duplicates: copy an earlier chunk's bytes over a later same-length one
    n = len(chunks)
    for _ in range(int(n * dup_frac)):
        a, b = sorted(rng.integers(0, n, 2))
        la = chunks[a][1]
        if a != b and la <= chunks[b][1]:
            chunks[b][1] = la
            data[chunks[b][0]:chunks[b][0] + la] = data[chunks[a][0]:chunks[a][0] + la]
    return bytes(data), np.array([tuple(c) for c in chunks], dtype=nydus_gpu.CHUNK_DTYPE)


@pytest.mark.parametrize("seed,chunk_size,unaligned,total", [
    (1, 0x1000, False, 8 << 20), (2, 0x4000, True, 8 << 20), (3, 0x10000, False, 8 << 20),
    (4, 0x100000, False, 48 << 20), (5, 0x100000, True, 48 << 20), (6, 0x1000000, False, 48 << 20),
    # just under the 40K-leaf limit of the quad-lane BLAKE3 path, unaligned; and a
    # 32 MiB layer, quad since round 3
    (7, 0x100000, True, 39 << 20), (8, 0x100000, False, 32 << 20)])
def test_random_vs_oracle(engines, oracle, seed, chunk_size, unaligned, total):
    rng = np.random.default_rng(seed)
    data, ch = _random_layer(rng, total, chunk_size, unaligned=unaligned)
    for digester in ("blake3", "sha256"):
        exp_d = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), digester)
        exp, own = oracle.dedup(exp_d, ch["length"])
        for lanes, fl in ([(0, 0), (1, 0), (16, 0)] if digester == "blake3" else
                          [(0, f) for f in SHA_FLAGS]) + [(0, GRID)]:
            out, st = engines(digester, chunk_size, lanes, flags=fl).process(data, ch)
            assert np.array_equal(out["digest"], exp_d), (digester, lanes, fl)
            for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
                assert np.array_equal(out[f], exp[f]), (digester, lanes, fl, f)
            assert st["intra_chunks"] == int((exp["kind"] == 1).sum())
            assert st["new_chunks"] == int((exp["kind"] == 0).sum())


def test_quad_groups_every_ragged_shape(engines, oracle):
    """b3_quad_planned's in-wave tree levels (round 6): multi-leaf chunks padded
    to groups of 4 slots, parents from adjacent LDS rows, chunks of <= 4 leaves
    finished in the leaf kernel, the rest continued by b3_tree over group CVs.
    Every leaf count 1..13 at k KiB - 1 / k KiB / k KiB + 1 bytes (ragged last
    groups of 1, 2 and 3 leaves; roots at 2, 3 and 4 leaves), single-leaf chunks
    interleaved so multi-leaf slots and single slots alternate in chunk order,
    a few 64-leaf chunks, ~4,000 chunks (the planned path's limit is 4,096),
    odd offsets; against the oracle and the grid-stage path."""
    rng = np.random.default_rng(66)
    lens = []
    while len(lens) < 3900:
        k = int(rng.integers(1, 14))
        lens.append(max(1, 1024 * k + int(rng.integers(-1, 2))))
        if rng.random() < 0.6:
            lens.append(int(rng.integers(1, 1025)))
        if rng.random() < 0.01:
            lens.append(65536 + int(rng.integers(-1, 2)))
    chunks, off = [], 0
    for ln in lens:
        off += int(rng.integers(0, 4))
        chunks.append((off, ln, 0, 0))
        off += ln
    data = rng.integers(0, 256, off + 16, dtype=np.uint8).tobytes()
    ch = np.array(chunks, dtype=nydus_gpu.CHUNK_DTYPE)
    assert len(ch) <= 4096 and off // 1024 + len(ch) <= 40960  # the planned quad path
    exp_d = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    exp, _ = oracle.dedup(exp_d, ch["length"])
    for fl in (0, GRID):
        out, _ = engines("blake3", 0x100000, 0, flags=fl).process(data, ch)
        bad = np.nonzero((out["digest"] != exp_d).any(1))[0]
        assert not len(bad), (fl, bad[:8], ch["length"][bad[:8]])
        for f in ("kind", "index", "ref"):
            assert np.array_equal(out[f], exp[f]), (fl, f)


@pytest.mark.parametrize("fl", [SHA_SPLIT, SHA_PAIR, SHA_LANE, SHA_PAIR_R1, SHA_PAIR_R4])
def test_sha256_ragged_wave(engines, oracle, fl):
    """Chunks of very different block counts in one wave (lanes finish at
    different blocks), lengths around the 55/56/64-byte padding edges, odd
    offsets (byte-load path), a count that is not a multiple of 32/64, and a
    bad descriptor in the middle of a wave."""
    rng = np.random.default_rng(21)
    lens = [1, 55, 56, 63, 64, 65, 119, 120, 128, 4096, 70000, 1 << 20, 3, 200000]
    lens += [int(x) for x in rng.integers(1, 300000, 83)]
    parts, chunks, off = [], [], 0
    for i, n in enumerate(lens):
        pad = int(rng.integers(0, 20)) if i % 3 == 0 else (-off) % 16
        parts.append(rng.integers(0, 256, pad, dtype=np.uint8).tobytes())
        off += pad
        parts.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        chunks.append((off, n, i, 0))
        off += n
    data = b"".join(parts)
    ch = np.array(chunks, dtype=nydus_gpu.CHUNK_DTYPE)
    exp_d = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "sha256")
    eng = engines("sha256", 0x1000000, 0, flags=fl)
    out, _ = eng.process(data, ch)
    assert np.array_equal(out["digest"], exp_d)
    bad = ch.copy()
    bad[40]["length"] = len(data)  # runs past the buffer
    with pytest.raises(nydus_gpu.NgpuError):
        eng.process(data, bad)


@pytest.mark.parametrize("fl", [0, GRID])
def test_random_dict_vs_oracle(oracle, fl):
    """Dict with duplicates (first wins), usize 0 wildcard, size mismatches and
    several inner blobs: decisions and blob allocation order match the oracle."""
    rng = np.random.default_rng(11)
    data, ch = _random_layer(rng, 16 << 20, 0x10000, dup_frac=0.3)
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    n = len(ch)
    pick = rng.choice(n, n // 2, replace=False)
    dd = np.concatenate([dig[pick], rng.integers(0, 256, (5000, 32), dtype=np.uint8), dig[pick[:50]]])
    ds = np.concatenate([ch["length"][pick], rng.integers(1, 1 << 16, 5000).astype(np.uint32),
                         np.zeros(50, np.uint32)]).astype(np.uint32)
    ds[: n // 20] = 0  # wildcard sizes
    ds[n // 20: n // 10] += 1  # size mismatch -> miss
    db = rng.integers(0, 7, len(dd)).astype(np.uint32)
    di = rng.integers(0, 1 << 20, len(dd)).astype(np.uint32)
    exp, own = oracle.dedup(dig, ch["length"], dd, ds, db, di)
    eng = nydus_gpu.Engine(chunk_size=0x10000, flags=fl)
    try:
        eng.dict_load(dd, ds, db, di)
        out, st = eng.process(data, ch)
    finally:
        eng.close()
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        assert np.array_equal(out[f], exp[f]), f
    assert st["dict_chunks"] == int((exp["kind"] == 2).sum()) > 0


def test_device_path_matches_host_path(engines):
    import torch
    rng = np.random.default_rng(5)
    data, ch = _random_layer(rng, 32 << 20, 0x100000)
    eng = engines("blake3", 0x100000, 0)
    out_h, st_h = eng.process(data, ch)
    d_data = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(len(ch) * 64, dtype=torch.uint8, device="cuda")
    st = eng.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), len(ch),
                            d_out.data_ptr(), stream=torch.cuda.current_stream().cuda_stream,
                            want_stats=True)
    out_d = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
    assert out_d.tobytes() == out_h.tobytes()
    assert st == st_h


def test_bad_descriptor_device_path(engines):
    import torch
    eng = engines("blake3", 0x100000, 0)
    d_data = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    ch = one_chunk(4096, off=1024)  # runs past the end of the buffer
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(nydus_gpu.NgpuError):
        eng.process_device(d_data.data_ptr(), 4096, d_ch.data_ptr(), 1, d_out.data_ptr(),
                           want_stats=True)
    with pytest.raises(nydus_gpu.NgpuError):
        eng.process(bytes(4096), ch)


@pytest.mark.parametrize("fl", [0, GRID])
def test_overlapping_descriptors(engines, oracle, fl):
    """Chunks that overlap (a tar's file extents never do) can hold more leaves
    than the buffer bounds a launch by: the call fails (NGPU_EINVAL) instead
    of leaving leaves unhashed.  A mild overlap inside the bound still hashes
    every chunk exactly."""
    S = 0x10000
    data = np.random.default_rng(3).integers(0, 256, S, dtype=np.uint8).tobytes()
    eng = engines("blake3", S, fl)
    many = np.zeros(2000, nydus_gpu.CHUNK_DTYPE)
    many["length"] = S  # 2000 x the whole buffer: 128,000 leaves
    with pytest.raises(nydus_gpu.NgpuError, match="overlap"):
        eng.process(data, many)
    mild = np.zeros(40, nydus_gpu.CHUNK_DTYPE)
    mild["offset"] = np.arange(40, dtype=np.uint64) * 1024
    mild["length"] = 2048  # each chunk shares 1 KiB with the next
    out, _ = eng.process(data, mild)
    assert np.array_equal(out["digest"], oracle.digest_chunks(data, mild.view(oracle.CHUNK_DTYPE), "blake3"))


def test_empty_layer(engines):
    out, st = engines().process(b"", np.zeros(0, nydus_gpu.CHUNK_DTYPE))
    assert len(out) == 0 and st["chunks"] == 0 and st["own_blob_index"] == 0xFFFFFFFF


def test_large_layer_properties(oracle):
    """BASELINE configs[1]-shaped at 4 GiB (device resident): planted duplicates
    are INTRA, NEW indices/offsets are the prefix sums, and a sample of chunks
    digests equal the oracle's (size-independent properties)."""
    import torch
    S = 0x100000
    n = 4096
    g = torch.Generator(device="cuda").manual_seed(1234)
    d_data = torch.randint(0, 256, (n * S,), dtype=torch.uint8, device="cuda", generator=g)
    # every 10th chunk copies chunk i-7
    for i in range(10, n, 10):
        d_data[i * S:(i + 1) * S] = d_data[(i - 7) * S:(i - 6) * S]
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    ch["offset"] = np.arange(n, dtype=np.uint64) * S
    ch["length"] = S
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    eng = nydus_gpu.Engine(chunk_size=S)
    try:
        st = eng.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), n,
                                d_out.data_ptr(), want_stats=True)
    finally:
        eng.close()
    out = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
    dup = np.zeros(n, bool)
    dup[10::10] = True
    assert (out["kind"][dup] == nydus_gpu.INTRA).all()
    assert (out["ref"][dup] == np.nonzero(dup)[0] - 7).all()
    assert (out["kind"][~dup] == nydus_gpu.NEW).all()
    assert np.array_equal(out["index"][~dup], np.arange((~dup).sum()))
    assert np.array_equal(out["uncompressed_offset"][~dup], np.arange((~dup).sum(), dtype=np.uint64) * S)
    assert st["new_chunks"] == (~dup).sum() and st["intra_chunks"] == dup.sum()
    rng = np.random.default_rng(0)
    for i in rng.choice(n, 24, replace=False):
        blob = d_data[i * S:(i + 1) * S].cpu().numpy().tobytes()
        assert out["digest"][i].tobytes() == oracle.blake3(blob), i


# ---- split stages and the digest-prefix partitioned dict ---------------------

def _to_dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


def test_split_stages_equal_process(oracle):
    """digest + dict probe + dedup as separate calls equal one process call."""
    import torch
    rng = np.random.default_rng(21)
    data, ch = _random_layer(rng, 24 << 20, 0x10000, dup_frac=0.3)
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    pick = rng.choice(len(ch), len(ch) // 3, replace=False)
    dd, ds = dig[pick], ch["length"][pick].astype(np.uint32)
    db = (np.arange(len(pick)) % 3).astype(np.uint32)
    di = np.arange(len(pick), dtype=np.uint32) + 7
    eng = nydus_gpu.Engine(chunk_size=0x10000)
    try:
        keep = [_to_dev(x) for x in (dd, ds, db, di)]  # alive until the engine has copied them
        torch.cuda.synchronize()
        eng.dict_load_device(*(t.data_ptr() for t in keep), len(pick), 3)
        torch.cuda.synchronize()
        d_data, d_ch = _to_dev(np.frombuffer(data, np.uint8)), _to_dev(ch)
        n = len(ch)
        o1 = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        st1 = eng.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), n, o1.data_ptr(),
                                 want_stats=True)
        o2 = torch.zeros_like(o1)
        eng.digest_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), n, o2.data_ptr())
        hits = torch.empty((n, 6), dtype=torch.int32, device="cuda")  # ngpu_dict_hit, 24 B
        eng.dict_probe_device(o2.data_ptr(), 64, n, hits.data_ptr())
        st2 = eng.dedup_device(d_ch.data_ptr(), n, o2.data_ptr(), hits.data_ptr(), 3, want_stats=True)
        torch.cuda.synchronize()
        assert torch.equal(o1, o2) and st1 == st2
        out = o1.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
        exp, _ = oracle.dedup(dig, ch["length"], dd, ds, db, di)
        for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
            assert np.array_equal(out[f], exp[f]), f
        # probe records vs a first-occurrence map
        h = hits.cpu().numpy()
        first = {}
        for i, row in enumerate(dd):
            first.setdefault(row.tobytes(), i)
        for i in range(n):
            e = first.get(dig[i].tobytes(), -1)
            assert h[i, 0] == e and (e < 0 or (h[i, 1] == di[e] and h[i, 2] == db[e] and h[i, 3] == ds[e]))
    finally:
        eng.close()


def _sharded_worker(rank, world, port, ret, equal=False):
    import os
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_py as oracle
        from nydus_gpu.dist import ShardedChunkDict, engine_load_fn, engine_probe_fn, sharded_process
        layers = [_random_layer(np.random.default_rng(500 + r), 16 << 20, 0x10000, dup_frac=0.2)
                  for r in range(world)]
        digs = [oracle.digest_chunks(d, c.view(oracle.CHUNK_DTYPE), "blake3") for d, c in layers]
        rng = np.random.default_rng(9)
        dd = np.concatenate([digs[0][::3], digs[1][1::4], rng.integers(0, 256, (3000, 32), dtype=np.uint8),
                             digs[0][::6]])
        ds = np.concatenate([layers[0][1]["length"][::3], layers[1][1]["length"][1::4],
                             rng.integers(1, 65536, 3000), np.zeros(len(digs[0][::6]))]).astype(np.uint32)
        db = (np.arange(len(dd)) % 4).astype(np.uint32)
        di = np.arange(len(dd), dtype=np.uint32)
        eng = nydus_gpu.Engine(chunk_size=0x10000)
        cap = max(len(c) for _, c in layers) if equal else 0  # equal padded splits
        sd = ShardedChunkDict(rank, world, comm_device="cpu", cap=cap)
        sd.load(torch.from_numpy(dd).cuda(), torch.from_numpy(ds.view(np.int32)).cuda(),
                torch.from_numpy(db.view(np.int32)).cuda(), torch.from_numpy(di.view(np.int32)).cuda(),
                4, engine_load_fn(eng, 4))
        sd.probe_fn = engine_probe_fn(eng)
        data, ch = layers[rank]
        n = len(ch)
        d_data, d_ch = _to_dev(np.frombuffer(data, np.uint8)), _to_dev(ch)
        out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        sharded_process(eng, sd, d_data, d_ch, n, out)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
        exp, _ = oracle.dedup(digs[rank], ch["length"], dd, ds, db, di)
        ok = np.array_equal(got["digest"], digs[rank])
        for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
            ok = ok and np.array_equal(got[f], exp[f])
        ret[rank] = (bool(ok), int((exp["kind"] == 2).sum()))
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("equal", [False, True])
def test_sharded_dict_two_ranks_one_gpu(equal):
    """Two ranks (processes) on the one GPU: dict partitioned by digest prefix,
    probes routed by all-to-all (gloo carries the exchange here; RCCL on a
    multi-GPU node), decisions identical to the oracle with the whole dict.
    equal: equal padded splits (no host sync in the probe)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_sharded_worker, args=(2, port, ret, equal), nprocs=2, join=True)
    assert ret[0][0] and ret[1][0]
    assert ret[0][1] > 0 and ret[1][1] > 0


# ---- streaming Pack (converter.Pack mirror) --------------------------------

def _stream(eng, tb, rng, zero_copy):
    w = eng.pack()
    pos = 0
    while pos < len(tb):
        k = int(rng.integers(1, 300_000))
        piece = tb[pos:pos + k]
        (w.write_zero_copy if zero_copy else w.write)(piece)
        pos += len(piece)
    return w.close()


def test_streaming_pack_matches_pack_tar(golden_layers, tars):
    rng = np.random.default_rng(77)
    for case in golden_layers["cases"]:
        cs = case["chunk_size"]
        # staging = 4 chunks: forces many slot switches and carried chunks
        eng = nydus_gpu.Engine(digester=case["digester"], chunk_size=cs, staging_bytes=4 * cs)
        try:
            tb = tars[case["layer"]]
            ref = eng.pack_tar(tb)
            for zc in (False, True):
                ch, out, st = _stream(eng, tb, rng, zc)
                assert ch.tobytes() == ref[0].tobytes(), case["layer"]
                assert out.tobytes() == ref[1].tobytes(), case["layer"]
                assert st == ref[2]
                assert [d.tobytes().hex() for d in out["digest"]] == case["digests"]
        finally:
            eng.close()


def test_streaming_pack_large_random_layer(oracle):
    """~200 MiB tar of random files through 8 MiB staging slots."""
    import io
    import tarfile
    rng = np.random.default_rng(8)
    bio = io.BytesIO()
    tf = tarfile.open(fileobj=bio, mode="w", format=tarfile.GNU_FORMAT)
    blobs = []
    for i in range(300):
        n = int(rng.choice([0, 100, 5000, 70000, 1 << 20, 3 << 20]) + rng.integers(0, 3000))
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes() if i % 7 else (blobs[-1] if blobs else b"")
        blobs.append(data)
        ti = tarfile.TarInfo(f"f{i}")
        ti.size = len(data)
        tf.addfile(ti, io.BytesIO(data))
    tf.close()
    tb = bio.getvalue()
    eng = nydus_gpu.Engine(chunk_size=0x100000, staging_bytes=8 << 20)
    try:
        ch, out, st = _stream(eng, tb, rng, True)
    finally:
        eng.close()
    ref_ch = oracle.tar_chunks(tb, 0x100000)
    assert ch.tobytes() == ref_ch.tobytes()
    dig = oracle.digest_chunks(tb, ref_ch, "blake3")
    assert np.array_equal(out["digest"], dig)
    dec, _ = oracle.dedup(dig, ref_ch["length"])
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        assert np.array_equal(out[f], dec[f]), f
    assert st["intra_chunks"] > 0


def test_streaming_pack_errors(tars):
    eng = nydus_gpu.Engine(chunk_size=0x100000)
    try:
        tb = tars["oci_upper"]
        w = eng.pack()
        w.write(tb[: len(tb) // 2])
        with pytest.raises(nydus_gpu.NgpuError) as e:
            w.close()
        assert e.value.code == -4  # truncated inside file data
        w = eng.pack()
        with pytest.raises(nydus_gpu.NgpuError):
            w.write(b"z" * 2048)  # bad header checksum
        w = eng.pack()
        w.write(tars["oci_lower"])
        w.abort()
        ch, out, st = eng.pack().close()  # empty stream is an empty layer
        assert len(ch) == 0 and st["chunks"] == 0
    finally:
        eng.close()


def test_host_reads_see_fresh_results_on_recycled_memory(tars):
    """Device memory recycled from a previous engine holds stale stats and
    results; a pack on a fresh engine (engine stream, no stage-end events)
    must still hand the host its own (host_fence before every D2H)."""
    import torch
    tb = tars["oci_lower"]
    for it in range(12):
        junk = torch.full((64 << 20,), 0x5A, dtype=torch.uint8, device="cuda")
        del junk
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        eng = nydus_gpu.Engine(chunk_size=0x10000)
        try:
            ch, out, st = eng.pack().close()  # empty layer first: all-zero stats
            assert len(ch) == 0 and st["chunks"] == 0 and st["new_chunks"] == 0, it
            ref = eng.pack_tar(tb)
            w = eng.pack()
            w.write(tb)
            ch2, out2, st2 = w.close()
            assert ch2.tobytes() == ref[0].tobytes() and out2.tobytes() == ref[1].tobytes(), it
            assert st2 == ref[2] and st2["chunks"] == len(ch2), it
        finally:
            eng.close()


def test_staging_pool_reuse_across_packs(golden_layers, tars, oracle):
    """The engine keeps streaming-Pack staging slots between packs (pack.hip
    release / ngpu_pack_open_ex). Slots move between plain and retained packs
    (a retained pack leaves no device copy behind), survive an aborted pack and
    are shared by two packs open at once; every result still equals
    pack_tar / the host writer fed with the oracle's decisions."""
    import io as _io
    from test_blob import cpu_stream
    rng = np.random.default_rng(31)
    cases = [c for c in golden_layers["cases"] if c["chunk_size"] == 0x10000]
    assert cases
    case = cases[0]
    cs, dg = case["chunk_size"], case["digester"]
    names = sorted(tars)
    tb, tb2 = tars[case["layer"]], tars[names[0] if names[0] != case["layer"] else names[1]]
    eng = nydus_gpu.Engine(digester=dg, chunk_size=cs, staging_bytes=4 * cs)
    try:
        ref, ref2 = eng.pack_tar(tb), eng.pack_tar(tb2)

        def same(got, want):
            assert got[0].tobytes() == want[0].tobytes()
            assert got[1].tobytes() == want[1].tobytes()
            assert got[2] == want[2]

        def retained(t):
            w = eng.pack(retain=True)
            w.write(t)
            out = _io.BytesIO()
            ch, res, st, info = w.finish(out, compressor="none")
            want = cpu_stream(oracle, t, cs, "none", dg)
            assert ch.tobytes() == want[2].tobytes()
            assert out.getvalue() == want[0]

        for rnd in range(3):
            same(_stream(eng, tb, rng, rnd % 2 == 1), ref)
            retained(tb)
            same(_stream(eng, tb, rng, False), ref)  # slots from the retained pack
            w = eng.pack()
            w.write(tb[: len(tb) // 2])
            w.abort()
            same(_stream(eng, tb2, rng, True), ref2)
            # two packs open at once, writes interleaved
            wa, wb = eng.pack(), eng.pack()
            pa = pb = 0
            while pa < len(tb) or pb < len(tb2):
                k = int(rng.integers(1, 200_000))
                if pa < len(tb):
                    wa.write(tb[pa:pa + k])
                    pa += k
                if pb < len(tb2):
                    wb.write(tb2[pb:pb + k])
                    pb += k
            same(wb.close(), ref2)
            same(wa.close(), ref)
    finally:
        eng.close()


@pytest.mark.parametrize("L,fl", [(40, 0), (40, GRID), (64, 0), (80, 0)])
def test_multi_layer_dedup_matches_per_layer(oracle, L, fl):
    """One launch set over L layers == each layer packed alone (oracle per
    layer), with a shared chunk dict and cross-layer duplicate contents (<= 64
    layers of a small call: the fused one-workgroup dedup; 80 layers and
    GRID: the multi-kernel path)."""
    import torch
    rng = np.random.default_rng(31)
    data, ch = _random_layer(rng, 40 << 20, 0x10000, dup_frac=0.4)
    n = len(ch)
    assert n <= 4096
    cuts = np.sort(rng.choice(np.arange(1, n), L - 1, replace=False))
    first = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    first[5] = first[4]  # an empty layer
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    pick = rng.choice(n, n // 5, replace=False)
    dd, ds = dig[pick], ch["length"][pick].astype(np.uint32)
    db = (np.arange(len(pick)) % 5).astype(np.uint32)
    di = np.arange(len(pick), dtype=np.uint32)
    eng = nydus_gpu.Engine(chunk_size=0x10000, flags=fl)
    try:
        eng.dict_load(dd, ds, db, di)
        d_data, d_ch = _to_dev(np.frombuffer(data, np.uint8)), _to_dev(ch)
        d_first = torch.from_numpy(first.view(np.int64).copy()).cuda()
        out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        st = torch.zeros(L * nydus_gpu.LAYER_STATS_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        eng.process_layers_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), n, out.data_ptr(),
                                  d_first.data_ptr(), L, st.data_ptr())
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
        stats = st.cpu().numpy().view(nydus_gpu.LAYER_STATS_DTYPE)
    finally:
        eng.close()
    assert np.array_equal(got["digest"], dig)
    for l in range(L):
        a, b = int(first[l]), int(first[l + 1])
        exp, own = oracle.dedup(dig[a:b], ch["length"][a:b], dd, ds, db, di)
        g = got[a:b]
        assert np.array_equal(g["kind"], exp["kind"]), l
        assert np.array_equal(g["index"], exp["index"]), l
        assert np.array_equal(g["blob_index"], exp["blob_index"]), l
        assert np.array_equal(g["uncompressed_offset"], exp["uncompressed_offset"]), l
        # refs: DICT -> dict entry, INTRA/NEW -> chunk id (global in the call)
        r = exp["ref"].astype(np.int64)
        r[exp["kind"] != 2] += a
        assert np.array_equal(g["ref"].astype(np.int64), r), l
        assert stats[l]["chunks"] == b - a
        assert stats[l]["new_chunks"] == (exp["kind"] == 0).sum()
        assert stats[l]["intra_chunks"] == (exp["kind"] == 1).sum()
        assert stats[l]["dict_chunks"] == (exp["kind"] == 2).sum()
        assert stats[l]["own_blob_index"] == (0xFFFFFFFF if own is None else own)


@pytest.mark.parametrize("fs", ["5", "6"])
def test_converter_testpack_flow(tars, oracle, tmp_path, fs):
    """tests/converter_test.go:459-528 (testPack for FsVersion "5" and "6")
    through the converter mirror on the GPU: buildChunkDict (Pack + Merge ->
    [sha256(dict Pack output)], :446-448), Pack lower/upper against the dict
    bootstrap, Merge -> [dict blob, sha256(upper Pack output)] (:513-519), and
    verify (:358-418) restated: the merged bootstrap reads back the expected
    overlay file tree from the dict and upper blobs alone (the lower layer's
    chunks are all in the dict: its blob is never read, :526).  v6 Pack
    outputs are byte-equal to the host writer fed with the CPU oracle's
    decisions."""
    import hashlib
    import io as _io
    import rafs_fixtures as rf
    from nydus_gpu import converter as cv
    from test_blob import check_stream, cpu_stream

    def pack(tar, dict_path=""):
        out = _io.BytesIO()
        w = cv.Pack(out, cv.PackOption(FsVersion=fs, ChunkDictPath=dict_path))
        for a in range(0, len(tar), 100_000):
            w.write(tar[a:a + 100_000])
        res = w.close()
        s = out.getvalue()
        assert res["digest"] == "sha256:" + hashlib.sha256(s).hexdigest()
        return s, res

    dstream, dres = pack(tars["chunk_dict"])
    if fs == "6":
        assert dstream == cpu_stream(oracle, tars["chunk_dict"], 0x100000, "zstd")[0]
    merged = _io.BytesIO()
    blobs = cv.Merge([cv.Layer(dres["digest"], dstream)], merged, cv.MergeOption())
    assert blobs == [dres["digest"]]
    dict_path = str(tmp_path / "dict-bootstrap")
    with open(dict_path, "wb") as f:
        f.write(merged.getvalue())

    lstream, lres = pack(tars["oci_lower"], dict_path)
    ustream, ures = pack(tars["oci_upper"], dict_path)
    assert (lres["results"]["kind"] == nydus_gpu.DICT).all()
    if fs == "6":
        from nydus_gpu import inspect as ni
        for tar, stream, res in ((tars["oci_lower"], lstream, lres), (tars["oci_upper"], ustream, ures)):
            ref = cpu_stream(oracle, tar, 0x100000, "zstd", dict_boot=merged.getvalue())
            assert stream == ref[0]
            # the layer bootstrap lists its dict chunks under the dict blob, copied
            # from the dict's records (check_stream compares them to the expectation)
            check_stream(oracle, stream, res["info"], tar, res["chunks"], res["results"], "zstd",
                         dict_boot=merged.getvalue())
            a, b = tmp_path / "gpu.stream", tmp_path / "oracle.stream"
            a.write_bytes(stream)
            b.write_bytes(ref[0])
            assert ni.main(["--diff", str(a), str(b)]) == 0
            assert ni.canonical(ni.load_bootstrap(stream)) == ni.canonical(ni.load_bootstrap(ref[0]))
        assert lres["info"]["dict_records"] == len({bytes(d) for d in lres["results"]["digest"]}) > 0
    out = _io.BytesIO()
    blobs = cv.Merge([cv.Layer(lres["digest"], lstream), cv.Layer(ures["digest"], ustream)], out,
                     cv.MergeOption(ChunkDictPath=dict_path))
    assert blobs == [dres["digest"], ures["digest"]]
    boot = out.getvalue()
    assert (struct.unpack_from("<I", boot, 0)[0] == 0x52414653) == (fs == "5")
    if fs == "6":
        assert rafs.read_v6(boot)["blob_ids"] == [dres["digest"][7:], ures["digest"][7:]]
    # verify: the blob directory holds the dict and upper blobs only
    blob_dir = {d["digest"][7:]: nydus_gpu.unpack_entry(st, "image.blob")[0]
                for d, st in ((dres, dstream), (ures, ustream))}
    view = rf.mount_view(boot, blob_dir)
    from test_rafs import tar_overlay
    assert view == tar_overlay([tars["oci_lower"], tars["oci_upper"]])


@pytest.mark.parametrize("compressor", ["none", "zstd", "lz4_block"])
def test_pack_stream_matches_host_writer(golden_layers, tars, oracle, compressor):
    """GPU Pack with the layer retained in HBM (NEW chunks gathered on the GPU,
    copied to the host window by window) writes exactly the stream the host
    writer produces from the oracle's decisions; tiny staging forces many
    segments and blob windows."""
    import io as _io
    from test_blob import check_stream, cpu_stream
    rng = np.random.default_rng(5)
    for case in golden_layers["cases"]:
        cs, dg = case["chunk_size"], case["digester"]
        tb = tars[case["layer"]]
        ref, rinfo, rch, rres, _ = cpu_stream(oracle, tb, cs, compressor, dg)
        eng = nydus_gpu.Engine(digester=dg, chunk_size=cs, staging_bytes=4 * cs)
        try:
            w = eng.pack(retain=True)
            pos = 0
            while pos < len(tb):
                k = int(rng.integers(1, 300_000))
                w.write(tb[pos:pos + k])
                pos += k
            out = _io.BytesIO()
            ch, res, st, info = w.finish(out, compressor=compressor)
        finally:
            eng.close()
        assert ch.tobytes() == rch.tobytes(), case["layer"]
        assert out.getvalue() == ref, (case["layer"], compressor)
        assert info == rinfo
        check_stream(oracle, out.getvalue(), info, tb, ch, res, compressor, dg)


def test_pack_stream_large_random_layer(oracle):
    """~200 MiB tar (random + repeated + compressible files) through 8 MiB
    staging slots with the blob stream written at the end."""
    import io
    import tarfile
    from test_blob import check_stream
    rng = np.random.default_rng(18)
    bio = io.BytesIO()
    tf = tarfile.open(fileobj=bio, mode="w", format=tarfile.GNU_FORMAT)
    prev = b""
    for i in range(260):
        n = int(rng.choice([0, 100, 5000, 70000, 1 << 20, 3 << 20]) + rng.integers(0, 3000))
        if i % 7 == 0:
            data = prev
        elif i % 5 == 0:
            data = bytes(n)  # compressible
        else:
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        prev = data
        ti = tarfile.TarInfo(f"f{i}")
        ti.size = len(data)
        tf.addfile(ti, io.BytesIO(data))
    tf.close()
    tb = bio.getvalue()
    eng = nydus_gpu.Engine(chunk_size=0x100000, staging_bytes=8 << 20)
    try:
        w = eng.pack(retain=True)
        for a in range(0, len(tb), 5 << 20):
            w.write_zero_copy(tb[a:a + (5 << 20)])
        out = io.BytesIO()
        ch, res, st, info = w.finish(out, compressor="zstd")
    finally:
        eng.close()
    ref_ch = oracle.tar_chunks(tb, 0x100000)
    assert ch.tobytes() == ref_ch.tobytes()
    dig = oracle.digest_chunks(tb, ref_ch, "blake3")
    assert np.array_equal(res["digest"], dig)
    check_stream(oracle, out.getvalue(), info, tb, ch, res, "zstd")
    assert 0 < info["compressed_chunks"] < info["blob_chunks"]


def test_pack_finish_needs_retain(tars):
    import io
    eng = nydus_gpu.Engine(chunk_size=0x100000)
    try:
        w = eng.pack()
        w.write(tars["oci_lower"])
        with pytest.raises(nydus_gpu.NgpuError) as e:
            w.finish(io.BytesIO())
        assert e.value.code == -1
    finally:
        eng.close()


def test_fs_version_5_offsets(oracle):
    """RAFS v5 (FsVersion "5"): NEW chunks packed without 4 KiB alignment."""
    rng = np.random.default_rng(55)
    data, ch = _random_layer(rng, 8 << 20, 0x10000, dup_frac=0.2)
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    exp, _ = oracle.dedup(dig, ch["length"], align=1)
    eng = nydus_gpu.Engine(chunk_size=0x10000, fs_version=5)
    try:
        out, st = eng.process(data, ch)
    finally:
        eng.close()
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        assert np.array_equal(out[f], exp[f]), f
    assert st["uncompressed_size"] == int(ch["length"][exp["kind"] == 0].sum())


def test_plain_c_client(tars, golden_layers, tmp_path):
    """A plain-C program (what the cgo binding does) links libnydusgpu.so and
    gets the golden digests and decisions (built in-tree by make)."""
    import subprocess
    from conftest import ROOT
    exe = os.path.join(ROOT, "nydus-snapshotter_amd", "build", "abi_client")
    case = next(c for c in golden_layers["cases"] if c["layer"] == "edge_pax" and c["chunk_size"] == 0x10000)
    tp = tmp_path / "l.tar"
    tp.write_bytes(tars["edge_pax"])
    out = subprocess.check_output([exe, str(tp), str(0x10000), "0"], text=True, timeout=60).splitlines()
    rows = [line.split(",") for line in out[:-1]]
    assert [r[2] for r in rows] == case["digests"]
    kinds = {"NEW": 0, "INTRA": 1, "DICT": 2}
    assert [int(r[3]) for r in rows] == [kinds[d[0]] for d in case["decisions"]]
    assert out[-1].startswith(f"STATS {len(rows)} ")


@pytest.mark.parametrize("compressor", ["", "none", "lz4_block"])
def test_cpp_converter_mirror_testpack(tars, tmp_path, compressor):
    """TestPack (converter_test.go:420-528) restated in C++ against the C++
    pkg/converter mirror (host/converter.hpp); its REQUIREs run in the binary,
    the digests it reports are re-checked here from the files it wrote."""
    import hashlib
    import subprocess
    from conftest import ROOT
    exe = os.path.join(ROOT, "nydus-snapshotter_amd", "build", "converter_test")
    paths = []
    for k in ("chunk_dict", "oci_lower", "oci_upper"):
        p = tmp_path / f"{k}.tar"
        p.write_bytes(tars[k])
        paths.append(str(p))
    work = tmp_path / "work"
    work.mkdir()
    go = tmp_path / "oci_upper_go.tar"  # TestUnpack's input in Go's tar encoding
    go.write_bytes(layers.oci_upper_tar_go(3))
    r = subprocess.run([exe, *paths, str(work), compressor, str(go)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[-1] == "PASS" and "unpack ok" in lines
    dig = dict(line.split()[1:] for line in lines if line.startswith("digest "))
    dict_file = work / dig["dict"][7:]
    assert "sha256:" + hashlib.sha256(dict_file.read_bytes()).hexdigest() == dig["dict"]
    merged = rafs.read_v6((work / "bootstrap").read_bytes())
    assert merged["blob_ids"] == [dig["dict"][7:], dig["upper"][7:]]
    # verify (converter_test.go:358-418) of both merged images from the dict
    # and upper blobs the binary wrote
    import rafs_fixtures as rf
    from test_rafs import tar_overlay
    dig5 = dict(line.split()[1:] for line in lines if line.startswith("digest5 "))
    want = tar_overlay([tars["oci_lower"], tars["oci_upper"]])
    for boot, dg in (("bootstrap", dig), ("bootstrap-v5", dig5)):
        blob_dir = {dg[k][7:]: nydus_gpu.unpack_entry((work / dg[k][7:]).read_bytes(), "image.blob")[0]
                    for k in ("dict", "upper")}
        assert rf.mount_view((work / boot).read_bytes(), blob_dir) == want, boot


def test_engine_thread_safety(oracle):
    """Concurrent calls on one engine serialise internally (threads as
    goroutines sharing an engine)."""
    import threading
    rng = np.random.default_rng(90)
    layers = [_random_layer(rng, 6 << 20, 0x10000) for _ in range(4)]
    eng = nydus_gpu.Engine(chunk_size=0x10000)
    errs = []

    def run(i):
        try:
            data, ch = layers[i]
            for _ in range(3):
                out, _ = eng.process(data, ch)
                exp = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
                if not np.array_equal(out["digest"], exp):
                    errs.append(i)
        except Exception as e:  # pragma: no cover
            errs.append(repr(e))
    ts = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    eng.close()
    assert not errs


@pytest.mark.parametrize("chunk_size,median,files", [(0x100000, 4096, 4000), (0x10000, 16384, 1200),
                                                     (0x100000, 1500, 4000)])
def test_small_file_mix_vs_oracle(engines, oracle, chunk_size, median, files):
    """Log-normal file sizes (most files a few KiB, a long tail): single-group
    chunks go through the block-count-sorted lane path of b3_groups, the rest
    through the chunk-ordered groups; every lanes-per-thread setting must give
    the oracle's digests and decisions."""
    rng = np.random.default_rng(median)
    sizes = np.minimum(8 << 20, np.maximum(1, rng.lognormal(np.log(median), 1.6, files))).astype(np.int64)
    stride = 512 + (sizes + 511) // 512 * 512
    starts = np.concatenate([[0], np.cumsum(stride)[:-1]]) + 512
    total = int(stride.sum()) + 1024
    data = bytearray(rng.integers(0, 256, total, dtype=np.uint8).tobytes())
    for i in range(7, len(sizes), 9):  # whole-file duplicates -> INTRA chunks
        j = i - 5
        if sizes[j] == sizes[i]:
            continue
        sizes[i] = sizes[j]
        data[starts[i]:starts[i] + sizes[i]] = data[starts[j]:starts[j] + sizes[j]]
    per = (sizes + chunk_size - 1) // chunk_size
    n = int(per.sum())
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    fi = np.repeat(np.arange(len(sizes)), per)
    k = np.arange(n) - np.repeat(np.cumsum(per) - per, per)
    ch["offset"] = starts[fi] + k * chunk_size
    ch["length"] = np.minimum(chunk_size, sizes[fi] - k * chunk_size)
    ch["file_index"] = fi
    ch["file_offset"] = k * chunk_size
    data = bytes(data)
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    dec, _ = oracle.dedup(dig, ch["length"])
    assert (dec["kind"] == 1).sum() > 0
    for lanes, fl in [(l, 0) for l in LANES] + [(0, GRID)]:
        out, st = engines("blake3", chunk_size, lanes, flags=fl).process(data, ch)
        assert np.array_equal(out["digest"], dig), (lanes, fl)
        for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
            assert np.array_equal(out[f], dec[f]), (lanes, fl, f)


def test_many_tiles_multi_layer_vs_oracle(oracle):
    """600K small chunks in 53 layers (one empty) with duplicates and a chunk
    dict: the BLAKE3 plan scan runs over > 512 tiles of 1024 chunks, so its
    look-back needs more than one round, and the dedup scan over ~300 tiles;
    every decision and every per-layer stat (derived from scan differences)
    must equal the oracle's per-layer pack."""
    import torch
    rng = np.random.default_rng(600)
    data = rng.integers(0, 256, 8 << 20, dtype=np.uint8).tobytes()
    n = 600_000
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    ch["length"] = rng.integers(1, 3000, n)
    ch["offset"] = rng.integers(0, len(data) - 3000, n)
    dup = rng.choice(n, n // 4, replace=False)  # same bytes as an earlier-or-later chunk
    src = rng.integers(0, n, len(dup))
    ch["offset"][dup], ch["length"][dup] = ch["offset"][src], ch["length"][src]
    ch["file_index"] = np.arange(n)
    first = np.concatenate([[0], np.sort(rng.choice(np.arange(1, n), 52, replace=False)), [n]])
    first[7] = first[6]  # an empty layer
    first = first.astype(np.uint64)
    L = len(first) - 1
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    pick = rng.choice(n, n // 10, replace=False)
    dd, ds = dig[pick], ch["length"][pick].astype(np.uint32)
    ds[::7] = 0  # wildcard sizes
    db = (np.arange(len(pick)) % 3).astype(np.uint32)
    di = np.arange(len(pick), dtype=np.uint32)
    eng = nydus_gpu.Engine(chunk_size=0x100000)
    try:
        eng.dict_load(dd, ds, db, di)
        d_data, d_ch = _to_dev(np.frombuffer(data, np.uint8)), _to_dev(ch)
        d_first = torch.from_numpy(first.view(np.int64).copy()).cuda()
        out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        st = torch.zeros(L * nydus_gpu.LAYER_STATS_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        eng.process_layers_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), n,
                                  out.data_ptr(), d_first.data_ptr(), L, st.data_ptr())
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
        stats = st.cpu().numpy().view(nydus_gpu.LAYER_STATS_DTYPE)
    finally:
        eng.close()
    assert np.array_equal(got["digest"], dig)
    for l in range(L):
        a, b = int(first[l]), int(first[l + 1])
        exp, own = oracle.dedup(dig[a:b], ch["length"][a:b], dd, ds, db, di)
        g = got[a:b]
        for f in ("kind", "index", "blob_index", "uncompressed_offset"):
            assert np.array_equal(g[f], exp[f]), (l, f)
        new = exp["kind"] == 0
        assert stats[l]["chunks"] == b - a
        assert stats[l]["new_chunks"] == new.sum()
        assert stats[l]["intra_chunks"] == (exp["kind"] == 1).sum()
        assert stats[l]["dict_chunks"] == (exp["kind"] == 2).sum()
        assert stats[l]["new_bytes"] == ch["length"][a:b][new].astype(np.int64).sum()
        ends = exp["uncompressed_offset"][new] + (ch["length"][a:b][new] + 4095) // 4096 * 4096
        assert stats[l]["uncompressed_size"] == (ends.max() if new.any() else 0)
        assert stats[l]["own_blob_index"] == (0xFFFFFFFF if own is None else own)
        assert stats[l]["blobs"] == len(set(exp["blob_index"].tolist())), l


_SCAN_N = [1, 2, 255, 256, 257, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097,
           64 * 1024 + 1, 512 * 1024 + 3]


@pytest.mark.parametrize("n,fl", [(n, 0) for n in _SCAN_N] + [(n, GRID) for n in _SCAN_N if n <= 4097])
def test_scan_tile_boundaries_vs_oracle(engines, oracle, n, fl):
    """Chunk counts at the single-pass scans' tile edges (256, 1024, 2048 and
    the 512-tile look-back window) and at the fused small-call limit (4096):
    decisions, indices and offsets equal the oracle's, for the single-layer
    path and a 3-layer call, on the fused and the grid path."""
    import torch
    rng = np.random.default_rng(n)
    data = rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    ch["length"] = rng.integers(1, 2500, n)
    ch["offset"] = rng.integers(0, len(data) - 2500, n)
    dup = rng.random(n) < 0.3
    src = rng.integers(0, n, n)
    ch["offset"][dup], ch["length"][dup] = ch["offset"][src[dup]], ch["length"][src[dup]]
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    dec, _ = oracle.dedup(dig, ch["length"])
    out, st = engines("blake3", 0x100000, flags=fl).process(data, ch)
    assert np.array_equal(out["digest"], dig)
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        assert np.array_equal(out[f], dec[f]), f
    # three layers, the middle one empty when n allows a cut
    cut = n // 2
    first = np.array([0, cut, cut, n], dtype=np.int64)
    eng = engines("blake3", 0x100000, flags=fl)
    d_data, d_ch = _to_dev(np.frombuffer(data, np.uint8)), _to_dev(ch)
    d_first = torch.from_numpy(first.copy()).cuda()
    d_out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(3 * nydus_gpu.LAYER_STATS_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    eng.process_layers_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), n, d_out.data_ptr(),
                              d_first.data_ptr(), 3, d_st.data_ptr())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
    stats = d_st.cpu().numpy().view(nydus_gpu.LAYER_STATS_DTYPE)
    for l in range(3):
        a, b = int(first[l]), int(first[l + 1])
        exp, _ = oracle.dedup(dig[a:b], ch["length"][a:b])
        for f in ("kind", "index", "blob_index", "uncompressed_offset"):
            assert np.array_equal(got[a:b][f], exp[f]), (l, f)
        assert stats[l]["chunks"] == b - a
        assert stats[l]["new_chunks"] == (exp["kind"] == 0).sum()
        assert stats[l]["intra_chunks"] == (exp["kind"] == 1).sum()


@pytest.mark.parametrize("fs", [5, 6])
def test_fixture_replay_through_gpu_dedup(fs):
    """The reference's real nydus-image bootstraps
    (pkg/filesystem/testdata/v5-bootstrap-file-size-736032.tar.gz,
    v6-bootstrap-chunk-pos-438272.tar.gz): their chunk streams (digests +
    sizes, file by file in inode order) through the GPU dedup stage
    (ngpu_dedup_device, FsVersion 5 / 6) give nydus-image's own index and
    uncompressed offset for every one of the 2,624 chunk references."""
    import torch
    import rafs_fixtures
    from test_oracle import V5_FIXTURE, V6_FIXTURE
    if fs == 5:
        d = rafs_fixtures.read_v5(rafs_fixtures.boot_from_targz(V5_FIXTURE))
        fx = np.concatenate([f[4] for f in d["files"]])
        count, usize, _ = d["ext_blobs"][0]
    else:
        files = rafs_fixtures.read_v6_files(rafs_fixtures.boot_from_targz(V6_FIXTURE))
        fx = np.concatenate([f[3] for f in files])
        b = rafs.read_v6_from_targz(V6_FIXTURE)["blobs"][0]
        count, usize = int(b["chunk_count"]), int(b["uncompressed_size"])
    n = len(fx)
    res = np.zeros(n, nydus_gpu.RESULT_DTYPE)
    res["digest"] = fx["block_id"]
    res["kind"] = nydus_gpu.DIGESTED  # caller-supplied digests enter dedup marked
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    ch["length"] = fx["uncompressed_size"]
    ch["file_offset"] = fx["file_offset"]
    eng = nydus_gpu.Engine(chunk_size=0x100000, fs_version=fs)
    try:
        d_out, d_ch = _to_dev(res), _to_dev(ch)
        st = eng.dedup_device(d_ch.data_ptr(), n, d_out.data_ptr(), want_stats=True)
        got = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
    finally:
        eng.close()
    assert np.array_equal(got["index"], fx["index"])
    assert np.array_equal(got["uncompressed_offset"], fx["uncompressed_offset"])
    assert np.array_equal(got["blob_index"], fx["blob_index"])
    assert st["new_chunks"] == count == 2515 and st["intra_chunks"] == n - count
    if fs == 5:
        assert st["uncompressed_size"] == usize
    else:  # v6: the blob's uncompressed size is 4K-rounded
        assert (st["uncompressed_size"] + 4095) // 4096 * 4096 == usize


def test_reference_v6_bootstrap_as_chunk_dict(tmp_path):
    """The reference's v6 fixture as PackOption.ChunkDictPath: the dict loads
    from a real nydus-image bootstrap (blake3, 1 MiB, its blob table), and the
    fixture's own chunk stream replayed against it is all DICT, each result
    carrying the dict record's entry, index and uncompressed offset."""
    import rafs_fixtures
    from test_oracle import V6_FIXTURE
    boot = rafs_fixtures.boot_from_targz(V6_FIXTURE)
    path = tmp_path / "image.boot"
    path.write_bytes(boot)
    table = rafs.read_v6(boot)["chunks"]
    fx = np.concatenate([f[3] for f in rafs_fixtures.read_v6_files(boot)])
    n = len(fx)
    res = np.zeros(n, nydus_gpu.RESULT_DTYPE)
    res["digest"] = fx["block_id"]
    res["kind"] = nydus_gpu.DIGESTED  # caller-supplied digests enter dedup marked
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    ch["length"] = fx["uncompressed_size"]
    eng = nydus_gpu.Engine(chunk_size=0x100000)
    try:
        d = eng.dict_open(str(path))
        assert d.entries == len(table) == 2515
        eng.set_dict(d)
        d.release()
        d_out, d_ch = _to_dev(res), _to_dev(ch)
        st = eng.dedup_device(d_ch.data_ptr(), n, d_out.data_ptr(), want_stats=True)
        got = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
    finally:
        eng.close()
    assert (got["kind"] == nydus_gpu.DICT).all() and st["dict_chunks"] == n
    pos = {bytes(r["block_id"]): i for i, r in enumerate(table)}
    assert np.array_equal(got["ref"], [pos[bytes(b)] for b in fx["block_id"]])
    assert np.array_equal(got["index"], fx["index"])
    assert np.array_equal(got["uncompressed_offset"], fx["uncompressed_offset"])
    assert st["own_blob_index"] == 0xFFFFFFFF and st["blobs"] == 1


def test_reference_v5_bootstrap_as_chunk_dict(tmp_path, oracle):
    """FsVersion "5" with ChunkDictPath = the reference's real v5 nydus-image
    bootstrap (RAFS v5 keeps each file's chunk infos after its inode; the dict
    is every file's chunks in inode-table order, first insertion wins).  The
    fixture's chunk stream replayed against it (plus random chunks) equals
    the oracle dedup against the same records; a v5 dict on a FsVersion 6
    engine and a v6 dict on a FsVersion 5 engine are rejected."""
    import rafs_fixtures
    from test_oracle import V5_FIXTURE, V6_FIXTURE
    boot = rafs_fixtures.boot_from_targz(V5_FIXTURE)
    path = tmp_path / "v5.boot"
    path.write_bytes(boot)
    v5 = rafs_fixtures.read_v5(boot)
    recs = np.concatenate([f[4] for f in v5["files"]])
    rng = np.random.default_rng(55)
    n = 3000
    pick = rng.integers(0, len(recs), n)
    res = np.zeros(n, nydus_gpu.RESULT_DTYPE)
    res["digest"] = recs["block_id"][pick]
    res["digest"][::7] = rng.integers(0, 256, (len(res["digest"][::7]), 32), dtype=np.uint8)
    res["kind"] = nydus_gpu.DIGESTED  # caller-supplied digests enter dedup marked
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    ch["length"] = recs["uncompressed_size"][pick]
    ch["length"][::7] = rng.integers(1, 0x100000, len(ch["length"][::7]))
    eng = nydus_gpu.Engine(chunk_size=v5["block_size"], fs_version=5)
    try:
        d = eng.dict_open(str(path))
        assert d.entries == len(recs)
        eng.set_dict(d)
        d.release()
        d_out, d_ch = _to_dev(res), _to_dev(ch)
        st = eng.dedup_device(d_ch.data_ptr(), n, d_out.data_ptr(), want_stats=True)
        got = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
    finally:
        eng.close()
    exp, _ = oracle.dedup(res["digest"], ch["length"], recs["block_id"], recs["uncompressed_size"],
                          recs["blob_index"], recs["index"], align=1,
                          dict_uoff=recs["uncompressed_offset"])
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        assert np.array_equal(got[f], exp[f]), f
    assert st["dict_chunks"] == int((exp["kind"] == nydus_gpu.DICT).sum()) > n // 2
    # version pairing
    v6path = tmp_path / "v6.boot"
    v6path.write_bytes(rafs_fixtures.boot_from_targz(V6_FIXTURE))
    for fs, pth in ((6, path), (5, v6path)):
        e2 = nydus_gpu.Engine(chunk_size=0x100000, fs_version=fs)
        try:
            with pytest.raises(nydus_gpu.NgpuError, match="inconsistent version"):
                e2.dict_open(str(pth))
        finally:
            e2.close()


@pytest.mark.parametrize("blobs", [1000, 1500])
def test_small_layer_dict_with_many_blobs(oracle, blobs):
    """A small single-layer call against a dict of many inner blobs: up to
    1023 the whole dedup stage stays in LDS (dedup_small_lds ranks the blobs
    there), beyond it the global small path takes over; both equal the oracle,
    blob allocation order included."""
    rng = np.random.default_rng(21 + blobs)
    data, ch = _random_layer(rng, 6 << 20, 0x10000, dup_frac=0.3)
    dig = oracle.digest_chunks(data, ch.view(oracle.CHUNK_DTYPE), "blake3")
    n = len(ch)
    pick = rng.choice(n, n // 2, replace=False)
    dd = np.concatenate([rng.integers(0, 256, (3000, 32), dtype=np.uint8), dig[pick]])
    ds = np.concatenate([rng.integers(1, 1 << 16, 3000), ch["length"][pick]]).astype(np.uint32)
    db = (np.arange(len(dd)) * 7919 % blobs).astype(np.uint32)
    di = np.arange(len(dd), dtype=np.uint32)
    exp, _ = oracle.dedup(dig, ch["length"], dd, ds, db, di)
    eng = nydus_gpu.Engine(chunk_size=0x10000)
    try:
        eng.dict_load(dd, ds, db, di)
        out, st = eng.process(data, ch)
    finally:
        eng.close()
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        assert np.array_equal(out[f], exp[f]), f
    assert st["dict_chunks"] == int((exp["kind"] == 2).sum()) > 0
    assert st["blobs"] == len(set(out["blob_index"].tolist()))


@pytest.mark.parametrize("fs", [5, 6])
def test_dict_bootstrap_fuzz(tmp_path, fs):
    """Corrupted RAFS v5 / v6 chunk-dict bootstraps (the file is untrusted
    input): every mutation either loads or fails with an NgpuError -- never a
    crash or a hang.  Mutations: truncation at random points, random bytes
    over the super blocks, the inode / blob / chunk tables."""
    import rafs_fixtures
    from test_oracle import V5_FIXTURE, V6_FIXTURE
    boot = bytearray(rafs_fixtures.boot_from_targz(V5_FIXTURE if fs == 5 else V6_FIXTURE))
    rng = np.random.default_rng(77 + fs)
    eng = nydus_gpu.Engine(chunk_size=0x100000, fs_version=fs)
    loaded = failed = 0
    try:
        for k in range(150):
            b = bytearray(boot)
            if k % 3 == 0:
                b = b[: int(rng.integers(0, len(b)))]
            else:
                lo = 0 if k % 3 == 1 else (8192 if fs == 5 else 1024)
                for _ in range(int(rng.integers(1, 8))):
                    p = int(rng.integers(lo, len(b) - 8))
                    b[p:p + 8] = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
            path = tmp_path / f"f{k}.boot"
            path.write_bytes(bytes(b))
            try:
                d = eng.dict_open(str(path))
                d.release()
                loaded += 1
            except nydus_gpu.NgpuError:
                failed += 1
    finally:
        eng.close()
    assert loaded + failed == 150 and failed > 0
