"""BASELINE.json configs at their full sizes (VERDICT r2 "configs_untested"):

* C2 -- the 16 GiB layer (4096 x 4 MiB files, 1 MiB chunks, real tar headers,
  offsets up to 2^34), blake3 at the auto setting (b3_groups<3>) and at one
  leaf per lane (b3_groups<0>): digests of every chunk that crosses a 4 GiB
  boundary, the last chunk and random chunks past 2^32 against the oracle;
  the dedup decisions by size-independent properties.
* C3 -- the same 16 GiB layer with the sha256 digester (sha256_pair) against a
  200,000,000-entry chunk dict in HBM: planted chunks DICT with their first
  table row, the rest NEW, digests past 2^32 against the oracle.
* C5 -- one multi-layer call of 1000 layers x 64 MiB (64 KiB chunks,
  1,024,000 chunks) against a pool dict: per-layer stats and decisions by
  properties, full oracle comparison on a sample of layers.

Each test builds its layer on the GPU (bench.py's generators, the bench's
exact layouts) and frees it before the next."""
import numpy as np
import pytest

import nydus_gpu

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _sample_ids(ch, k=24, seed=11):
    import bench
    ids = bench.high_offset_sample(ch, k=k, seed=seed)
    return np.unique(np.concatenate([ids, [0, 1]]))


def _check_digests(oracle, buf, ch, out, ids, digester):
    for i in ids:
        o, ln = int(ch["offset"][i]), int(ch["length"][i])
        blob = buf[o:o + ln].cpu().numpy().tobytes()
        want = oracle.sha256(blob) if digester == "sha256" else oracle.blake3(blob)
        assert out["digest"][i].tobytes() == want, (int(i), o, ln)


@pytest.mark.parametrize("lanes", [0, 1])
def test_c2_16gib_layer_digests_past_4gib(lanes, oracle):
    import torch
    import bench
    buf, ch = bench.build_layer_on_gpu(torch, 4096, 4 * MiB, MiB, seed=0x6E79647573)
    try:
        assert buf.numel() > (1 << 34) and int(ch["offset"].max()) > (1 << 34)
        n = len(ch)
        d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
        d_out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        eng = nydus_gpu.Engine(chunk_size=MiB, leaves_per_lane=lanes)
        try:
            st = eng.process_device(buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n, d_out.data_ptr(),
                                    want_stats=True)
        finally:
            eng.close()
        out = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
        ids = _sample_ids(ch)
        assert len(ids) >= 28 and int(ch["offset"][ids].max()) > (1 << 34)
        _check_digests(oracle, buf, ch, out, ids, "blake3")
        # random 4 MiB files: every chunk NEW, indices / v6 offsets are prefix sums
        assert (out["kind"] == nydus_gpu.NEW).all()
        assert np.array_equal(out["index"], np.arange(n))
        assert np.array_equal(out["uncompressed_offset"], np.arange(n, dtype=np.uint64) * MiB)
        assert st["chunks"] == st["new_chunks"] == n and st["new_bytes"] == n * MiB
        # all 16384 digests distinct (no INTRA could hide a bad high-offset digest)
        assert len({d.tobytes() for d in out["digest"]}) == n
    finally:
        del buf
        torch.cuda.empty_cache()


def test_c3_16gib_sha256_vs_200m_entry_dict(oracle):
    import torch
    import bench
    S = MiB
    buf, ch = bench.build_layer_on_gpu(torch, 4096, 4 * MiB, S, seed=0x6E79647573)
    n = len(ch)
    m = 200_000_000
    eng = nydus_gpu.Engine(digester="sha256", chunk_size=S)
    try:
        d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
        d_out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        eng.digest_device(buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n, d_out.data_ptr())
        torch.cuda.synchronize()
        dig = d_out.view(n, 64)[:, :32].clone()
        g = torch.Generator(device="cuda").manual_seed(0xD1C7)
        dd = torch.empty((m, 32), dtype=torch.uint8, device="cuda")
        dd.random_(0, 256, generator=g)
        rng = np.random.default_rng(3)
        planted = np.sort(rng.choice(n, int(0.3 * n), replace=False))
        rows = torch.randperm(m, device="cuda", generator=g)[: len(planted)]
        dd[rows] = dig[torch.from_numpy(planted).cuda()]
        us = torch.full((m,), S, dtype=torch.int32, device="cuda")
        bl = torch.zeros(m, dtype=torch.int32, device="cuda")
        ix = torch.arange(m, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        d = eng.dict_create_device(dd.data_ptr(), us.data_ptr(), bl.data_ptr(), ix.data_ptr(), m, 1)
        del dd, us, bl, ix
        torch.cuda.empty_cache()
        try:
            d_out.zero_()
            st = eng.process_dict_device(d, buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n,
                                         d_out.data_ptr(), want_stats=True)
        finally:
            d.release()
        out = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
        rows = rows.cpu().numpy().astype(np.int64)
        assert (out["kind"][planted] == nydus_gpu.DICT).all()
        assert np.array_equal(out["ref"][planted], rows)
        assert np.array_equal(out["index"][planted], rows)
        rest = np.setdiff1d(np.arange(n), planted)
        assert (out["kind"][rest] == nydus_gpu.NEW).all()
        assert np.array_equal(out["index"][rest], np.arange(len(rest)))
        assert st["dict_chunks"] == len(planted) and st["new_chunks"] == len(rest)
        _check_digests(oracle, buf, ch, out, _sample_ids(ch, k=12), "sha256")
    finally:
        eng.close()
        del buf
        torch.cuda.empty_cache()


def test_c5_1000_layers_one_call(oracle):
    """configs[4] at its real layer count: 1000 layers x 64 MiB (16 x 4 MiB
    files each), 64 KiB chunks = 1,024,000 chunks in one multi-layer call,
    30 % of the chunks drawn from a 1024-content pool whose digests (plus
    filler) form the chunk dict.  Per layer: pool chunks are DICT (or INTRA to
    an earlier NEW copy never, since the dict takes every pool digest), the
    rest NEW with indices 0.. in stream order; stats equal the decisions.  A
    sample of layers is compared field by field with the oracle's dedup of
    that layer alone."""
    import torch
    import bench
    wl = dict(bench.WORKLOADS["c5-1000"])
    S, L = wl["chunk"], 1000
    wl["n_files"] = wl["n_files"] * L
    buf, ch = bench.build_layer_on_gpu(torch, wl["n_files"], wl["file_size"], S, seed=0xC5)
    try:
        _, stride, _, _ = bench.synthetic_layout(1, wl["file_size"], S)
        _, planted = bench.plant_pool(torch, buf, ch, stride, wl, seed=1)
        n = len(ch)
        assert n == 1_024_000
        pool = bench.pool_digests(torch, nydus_gpu, wl, 0)  # (1024, 32) on the GPU
        filler = torch.randint(0, 256, (wl["dict_entries"], 32), dtype=torch.uint8, device="cuda",
                               generator=torch.Generator(device="cuda").manual_seed(5))
        dd = torch.cat([pool, filler]).contiguous()
        m = dd.shape[0]
        us = torch.full((m,), S, dtype=torch.int32, device="cuda")
        bl = (torch.arange(m, dtype=torch.int32, device="cuda") % 8).contiguous()
        ix = torch.arange(m, dtype=torch.int32, device="cuda")
        per_layer = n // L
        first = np.arange(L + 1, dtype=np.int64) * per_layer
        eng = nydus_gpu.Engine(chunk_size=S)
        try:
            torch.cuda.synchronize()
            d = eng.dict_create_device(dd.data_ptr(), us.data_ptr(), bl.data_ptr(), ix.data_ptr(), m, 8)
            d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
            d_out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
            d_first = torch.from_numpy(first).cuda()
            d_st = torch.zeros(L * nydus_gpu.LAYER_STATS_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
            eng.process_dict_device(d, buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n,
                                    d_out.data_ptr(), d_layer_first=d_first.data_ptr(),
                                    n_layers=L, d_stats=d_st.data_ptr())
            torch.cuda.synchronize()
            eng.device_status()
            d.release()
        finally:
            eng.close()
        out = d_out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
        stats = d_st.cpu().numpy().view(nydus_gpu.LAYER_STATS_DTYPE)
        kinds = np.bincount(out["kind"], minlength=5)
        assert kinds[3] == kinds[4] == 0
        assert kinds[2] >= planted * 0.999  # every pool chunk is a dict hit (filler may add a few)
        assert stats["chunks"].sum() == n
        assert stats["new_chunks"].sum() == kinds[0] and stats["dict_chunks"].sum() == kinds[2]
        for l in range(L):
            a, b = first[l], first[l + 1]
            k = out["kind"][a:b]
            new = k == nydus_gpu.NEW
            assert np.array_equal(out["index"][a:b][new], np.arange(new.sum())), l
            assert stats["new_chunks"][l] == new.sum()
        # full field-by-field comparison for a sample of layers (dict = pool + filler)
        dig_all = out["digest"]
        dd_h = dd.cpu().numpy()
        us_h, bl_h, ix_h = np.full(m, S, np.uint32), (np.arange(m) % 8).astype(np.uint32), \
            np.arange(m, dtype=np.uint32)
        for l in (0, 1, 499, 998, 999):
            a, b = first[l], first[l + 1]
            blob = buf[int(ch["offset"][a]):int(ch["offset"][b - 1] + ch["length"][b - 1])]
            sub = ch[a:b].copy()
            sub["offset"] -= ch["offset"][a]
            dig = oracle.digest_chunks(blob.cpu().numpy().tobytes(), sub.view(oracle.CHUNK_DTYPE),
                                       "blake3")
            assert np.array_equal(dig_all[a:b], dig), l
            exp, _ = oracle.dedup(dig, sub["length"], dd_h, us_h, bl_h, ix_h)
            for f in ("kind", "index", "blob_index", "uncompressed_offset"):
                assert np.array_equal(out[f][a:b], exp[f]), (l, f)
            # ref: a dict entry id for DICT, else a chunk id of the CALL (the layer's
            # own ids are offset by its first chunk)
            own = exp["kind"] != nydus_gpu.DICT
            assert np.array_equal(out["ref"][a:b][own] - a, exp["ref"][own]), l
            assert np.array_equal(out["ref"][a:b][~own], exp["ref"][~own]), l
    finally:
        del buf
        torch.cuda.empty_cache()


def test_streaming_pack_of_a_9gib_file(oracle):
    """One regular file larger than 8 GiB in a layer tar (its size needs the
    GNU base-256 encoding: tarfile's GNU header) streamed through
    converter.Pack's path (ngpu_pack_write in 64 MiB pieces): chunk k of the
    file has file_offset k * S past 2^32 and 2^33, the tail chunk is partial,
    a small file after it is chunked from the right stream offset, and the
    sampled digests (first, around 4 GiB and 8 GiB, last, the small file)
    equal the oracle's.  Pieces are a fixed random block xor its index, so
    every chunk is distinct (all NEW)."""
    import io
    import tarfile
    S, piece = MiB, 64 * MiB
    size = 9 * (1 << 30) + 12345
    base = np.random.default_rng(0x9B16).integers(0, 256, piece, dtype=np.uint8)

    def chunk_of(p):  # piece p of the file's bytes
        x = base.copy()
        x.view(np.uint64)[::4096] ^= np.uint64(p + 1)  # distinct in every 1 MiB chunk
        return x

    hi = tarfile.TarInfo("big.bin")
    hi.size, hi.mode, hi.mtime = size, 0o644, 1_700_000_000
    head = hi.tobuf(format=tarfile.GNU_FORMAT)
    assert head[124] & 0x80  # base-256 size field
    small = bytes(range(256)) * 40
    si = tarfile.TarInfo("after.txt")
    si.size = len(small)
    tail_tar = si.tobuf(format=tarfile.GNU_FORMAT) + small + bytes(-len(small) % 512) + bytes(1024)
    eng = nydus_gpu.Engine(chunk_size=S)
    want = {}
    sample = {0, 1, 4095, 4096, 4097, 8191, 8192, 8193, size // S}
    try:
        w = eng.pack()
        w.write(head)
        done = 0
        p = 0
        while done < size:
            data = chunk_of(p)[: min(piece, size - done)]
            for k in range(done // S, (done + len(data) + S - 1) // S):
                if k in sample:
                    a = k * S - done
                    want[k] = oracle.blake3(data[a:a + S].tobytes())
            w.write(data)
            done += len(data)
            p += 1
        w.write(bytes(-size % 512) + tail_tar)
        ch, res, st = w.close()
    finally:
        eng.close()
    n_big = -(-size // S)
    assert len(ch) == n_big + 1 and st["chunks"] == n_big + 1
    big = ch[:n_big]
    assert (big["file_index"] == 0).all() and (ch["file_index"][-1] == 1)
    assert np.array_equal(big["file_offset"], np.arange(n_big, dtype=np.uint64) * S)
    assert int(big["file_offset"][-1]) > (1 << 33) and int(big["length"][-1]) == size - (n_big - 1) * S
    assert np.array_equal(big["offset"], 512 + np.arange(n_big, dtype=np.uint64) * S)
    assert int(ch["offset"][-1]) == 512 + -(-size // 512) * 512 + 512
    for k, d in want.items():
        assert res["digest"][k].tobytes() == d, k
    assert res["digest"][-1].tobytes() == oracle.blake3(small)
    assert (res["kind"] == nydus_gpu.NEW).all() and st["new_chunks"] == n_big + 1


def test_c4_one_gpu_share_through_an_8_part_node(oracle):
    """configs[3] (C4) at one GPU's share of the 8-GPU node, through the C
    ABI's node as the driver's node would run it: device 0 listed 8 times, 8
    parts x 16 layers x 1 GiB (256 x 4 MiB files, 1 MiB chunks, 131,072
    chunks), 30 % of the chunks drawn from the 65,536-content pool, and the
    node dict = pool digests + 16M random filler + 1,000 later duplicates of
    pool rows, partitioned by digest prefix over the 8 parts (routed
    exchange).  Checked:
    * every pool chunk is DICT with the pool row's id (the FIRST table row of
      its digest, not the later duplicate) and that row's index / offset;
    * every other chunk is NEW, indices 0.. and 1 MiB-step v6 offsets per
      layer (prefix sums), per-layer stats equal to the decisions;
    * the replicated dict and the copy exchange give byte-identical results;
    * three sampled layers field by field against the oracle's dedup of that
      layer alone with the whole 16M-entry dict (digests by the oracle)."""
    import torch
    import bench
    from nydus_gpu import rafs
    wl = dict(bench.WORKLOADS["c4"])
    S, P, W, L = wl["chunk"], wl["pool"], 8, 16
    wl["n_files"] = wl["n_files"] * L
    _, stride, _, _ = bench.synthetic_layout(1, wl["file_size"], S)
    parts = []
    try:
        for i in range(W):
            buf, ch = bench.build_layer_on_gpu(torch, wl["n_files"], wl["file_size"], S,
                                               seed=0x6E79647573 + i)
            info, planted = bench.plant_pool(torch, buf, ch, stride, wl, seed=i)
            parts.append(dict(buf=buf, ch=ch, sel=info["chunks"], src=info["content"],
                              d_ch=torch.from_numpy(ch.view(np.uint8).copy()).cuda()))
        n = len(parts[0]["ch"])
        assert n == 16 * 1024 and int(parts[0]["buf"].numel()) > (16 << 30)
        per_layer = n // L
        first = np.arange(L + 1, dtype=np.int64) * per_layer
        d_first = torch.from_numpy(first).cuda()
        pool = bench.pool_digests(torch, nydus_gpu, wl, 0).cpu().numpy()
        rng = np.random.default_rng(0xC4)
        m = P + wl["dict_entries"] + 1000
        recs = np.zeros(m, rafs.CHUNK_INFO_DTYPE)
        recs["block_id"][:P] = pool
        recs["block_id"][P:m - 1000] = rng.integers(0, 256, (wl["dict_entries"], 32), dtype=np.uint8)
        dup = rng.choice(P, 1000, replace=False)
        recs["block_id"][m - 1000:] = pool[dup]
        recs["uncompressed_size"] = S
        recs["compressed_size"] = S
        recs["blob_index"] = rng.integers(0, 8, m)
        recs["index"] = rng.permutation(m).astype(np.uint32)
        recs["uncompressed_offset"] = np.arange(m, dtype=np.uint64) * S
        blobs = rafs.make_blob_table([f"{b:064x}" for b in range(8)], S)
        node = nydus_gpu.Node([0] * W, chunk_size=S)
        results = {}
        try:
            for name, mode in (("routed", nydus_gpu.NODE_DICT_PARTITION | nydus_gpu.NODE_EXCHANGE_ROUTED),
                               ("replicate", nydus_gpu.NODE_DICT_REPLICATE),
                               ("copy", nydus_gpu.NODE_DICT_PARTITION | nydus_gpu.NODE_EXCHANGE_COPY)):
                d = node.dict_create(recs, blobs, mode=mode)
                outs = []
                for i, p in enumerate(parts):
                    if name == "copy" and i >= 2:
                        break  # the copy exchange: two parts suffice for the equality
                    out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
                    st = torch.zeros(L * nydus_gpu.LAYER_STATS_DTYPE.itemsize, dtype=torch.uint8,
                                     device="cuda")
                    node.process_device(i, d, p["buf"].data_ptr(), p["buf"].numel(), p["d_ch"].data_ptr(),
                                        n, out.data_ptr(), d_first.data_ptr(), L, st.data_ptr(),
                                        stream=torch.cuda.current_stream().cuda_stream)
                    torch.cuda.synchronize()
                    outs.append((out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE).copy(),
                                 st.cpu().numpy().view(nydus_gpu.LAYER_STATS_DTYPE).copy()))
                for e in node.engines:
                    e.device_status()
                d.release()
                results[name] = outs
        finally:
            node.close()
        total_dict = 0
        for i, p in enumerate(parts):
            out, stats = results["routed"][i]
            sel, src = p["sel"], p["src"]
            assert (out["kind"][sel] == nydus_gpu.DICT).all(), i
            assert np.array_equal(out["ref"][sel], src), i  # pool row = content id: the first row
            assert np.array_equal(out["index"][sel], recs["index"][src]), i
            assert np.array_equal(out["uncompressed_offset"][sel], recs["uncompressed_offset"][src]), i
            rest = np.ones(n, bool)
            rest[sel] = False
            assert (out["kind"][rest] == nydus_gpu.NEW).all(), i
            for layer in range(L):
                a, b = first[layer], first[layer + 1]
                new = out["kind"][a:b] == nydus_gpu.NEW
                k = int(new.sum())
                assert np.array_equal(out["index"][a:b][new], np.arange(k)), (i, layer)
                assert np.array_equal(out["uncompressed_offset"][a:b][new],
                                      np.arange(k, dtype=np.uint64) * S), (i, layer)
                assert stats["new_chunks"][layer] == k and stats["dict_chunks"][layer] == per_layer - k
            total_dict += len(sel)
            for other in ("replicate", "copy"):
                if i < len(results[other]):
                    assert results[other][i][0].tobytes() == out.tobytes(), (other, i)
                    assert results[other][i][1].tobytes() == stats.tobytes(), (other, i)
        assert total_dict > 0.29 * W * n
        # three sampled layers against the oracle with the whole dict
        for i, layer in ((0, 0), (3, 7), (7, 15)):
            p = parts[i]
            out = results["routed"][i][0]
            a, b = first[layer], first[layer + 1]
            ch = p["ch"]
            lo = int(ch["offset"][a])
            hi = int(ch["offset"][b - 1] + ch["length"][b - 1])
            blob = p["buf"][lo:hi].cpu().numpy()
            sub = ch[a:b].copy()
            sub["offset"] -= lo
            dig = oracle.digest_chunks(blob, sub.view(oracle.CHUNK_DTYPE), "blake3")
            assert np.array_equal(out["digest"][a:b], dig), (i, layer)
            exp, _ = oracle.dedup(dig, sub["length"], recs["block_id"], recs["uncompressed_size"],
                                  recs["blob_index"], recs["index"], dict_uoff=recs["uncompressed_offset"])
            for f in ("kind", "index", "blob_index", "uncompressed_offset"):
                assert np.array_equal(out[f][a:b], exp[f]), (i, layer, f)
            own = exp["kind"] != nydus_gpu.DICT
            assert np.array_equal(out["ref"][a:b][own] - a, exp["ref"][own]), (i, layer)
            assert np.array_equal(out["ref"][a:b][~own], exp["ref"][~own]), (i, layer)
    finally:
        parts.clear()
        torch.cuda.empty_cache()
