"""GPU: PackOption.OCIRef -- `nydus-image create --type targz-ref`
(pkg/converter/tool/builder.go:180-218, convert_unix.go:346-351, 500-509).

The Pack writer takes the ORIGINAL gzip layer blob; the library inflates it on
the host while keeping deflate checkpoints (zran), the tar stream takes the
tar-rafs digest/dedup path on the GPU, and the output stream carries blob.meta
(chunk infos + checkpoint table + dictionaries), blob.digest, image.boot and
the TOC -- no image.blob: the chunks stay in the gzip blob, which is the
bootstrap's own blob.

Pinned:
* TestPackRef (tests/converter_test.go:530-605) restated: the TOC finds
  image.boot and blob.meta with their uncompressed digests, and Merge(OCIRef)
  of the layer (OriginalDigest = the gzip digest) returns [gzip digest];
* the chunk list and every chunk digest of the decompressed stream equal the
  oracle's over the same tar (tar-rafs chunking, BLAKE3).
Restated, not pinned (VERIFY): the blob.meta zran layout, the chunk records'
compressed ranges.  They are checked for self-consistency: every chunk comes
back out of the gzip blob through its checkpoint (ngpu_ref_chunk_read, the
reader side nydusd has) with the bytes and digest the bootstrap records."""
import gzip
import hashlib
import io
import tarfile
import zlib

import numpy as np
import pytest

import nydus_gpu

pytestmark = pytest.mark.gpu


def _gzip(data, level=6):
    return gzip.compress(data, compresslevel=level, mtime=0)


def _pack_ref(gz, piece=65536):
    from nydus_gpu import converter as cv
    out = io.BytesIO()
    w = cv.Pack(out, cv.PackOption(OCIRef=True))
    for a in range(0, len(gz), piece):
        w.write(gz[a:a + piece])
    res = w.close()
    return out.getvalue(), res


def _files_of(tar):
    """{path: bytes} of the tar's regular files with data, in tar order."""
    out = {}
    with tarfile.open(fileobj=io.BytesIO(tar)) as tf:
        for m in tf.getmembers():
            if m.isreg() and m.size:
                out["/" + m.name.lstrip("./")] = tf.extractfile(m).read()
    return out


def _check_layer(oracle, tar, gz, stream, S=0x100000):
    import blob_ref
    boot, e_boot = blob_ref.unpack_entry(stream, blob_ref.ENTRY_BOOTSTRAP)
    meta, e_meta = blob_ref.unpack_entry(stream, "blob.meta")
    header, e_hdr = blob_ref.unpack_entry(stream, "blob.meta.header")
    assert e_boot is not None and e_meta is not None and e_hdr is not None  # found through the TOC
    assert e_boot["uncompressed_digest"] == hashlib.sha256(boot).hexdigest()
    assert e_meta["uncompressed_digest"] == hashlib.sha256(meta).hexdigest()
    assert len(header) == 4096
    # the tar entry "blob.meta" is the (uncompressed) array + tables, then the header
    off, size = blob_ref.seek_file_by_tar_header(stream, "blob.meta")
    assert stream[off:off + size] == meta + header
    meta = meta + header
    with pytest.raises(blob_ref.NotFound):  # no image.blob: the data stays in the gzip blob
        blob_ref.unpack_entry(stream, blob_ref.ENTRY_BLOB)
    dump = nydus_gpu.rafs_dump(boot)
    assert dump["fs_version"] == 6 and dump["chunk_size"] == S
    assert len(dump["blobs"]) == 1 and dump["blobs"][0]["id"] == hashlib.sha256(gz).hexdigest()
    # chunk list + digests of every file == the oracle over the same tar
    files = _files_of(tar)
    got = {i["path"]: i["chunks"] for i in dump["inodes"] if "chunks" in i}
    assert set(got) == set(files)
    by_index = {}
    for path, body in files.items():
        chs = got[path]
        assert len(chs) == -(-len(body) // S), path
        for k, c in enumerate(chs):
            piece = body[k * S:(k + 1) * S]
            assert c[0] == oracle.blake3(piece).hex(), (path, k)
            assert c[6] == len(piece) and c[7] == k * S, (path, k)
            by_index.setdefault(c[8], piece)
    # every own-blob chunk back out of the gzip blob through its checkpoint
    for idx, piece in by_index.items():
        assert nydus_gpu.ref_chunk_read(gz, meta, idx) == piece, idx
    return dump, meta


def test_testpackref_restated(oracle):
    """converter_test.go:530-605 (TestPackRef) through the Python mirror."""
    from nydus_gpu import converter as cv
    import layers
    tar = layers.oci_lower_tar()
    gz = _gzip(tar)
    stream, res = _pack_ref(gz)
    assert res["digest"] == "sha256:" + hashlib.sha256(stream).hexdigest()
    _check_layer(oracle, tar, gz, stream)
    gz_digest = "sha256:" + hashlib.sha256(gz).hexdigest()
    merged = io.BytesIO()
    blobs = cv.Merge([cv.Layer(Digest=res["digest"], ReaderAt=stream, OriginalDigest=gz_digest)],
                     merged, cv.MergeOption(OCIRef=True))
    assert blobs == [gz_digest]
    # the layer's blob record carries Merge's --blob-digests / --blob-sizes /
    # --blob-toc-digests (convert_unix.go:579-587; restated offsets, VERIFY)
    from nydus_gpu import rafs
    toc = io.BytesIO()
    cv.UnpackEntry(stream, cv.EntryTOC, toc)
    rec = rafs.read_v6(merged.getvalue())["blobs"]
    assert rec["blob_id"][0].decode() == gz_digest.split(":")[1]
    meta = bytes(rec["reserved"][0])
    assert meta[32:64] == hashlib.sha256(toc.getvalue()).digest()
    assert meta[64:96].hex() == res["digest"].split(":")[1]
    assert int.from_bytes(meta[96:104], "little") == len(stream)


@pytest.mark.parametrize("level", [1, 9])
def test_ociref_large_layer_many_checkpoints(oracle, level):
    """A ~40 MiB layer (random and compressible files, duplicates, a file of
    several MiB): many deflate checkpoints, chunks that start far into a
    checkpoint's output, INTRA chunks; gzip written in odd-sized pieces."""
    rng = np.random.default_rng(level)
    out = io.BytesIO()
    with tarfile.open(fileobj=out, mode="w", format=tarfile.PAX_FORMAT) as tw:
        bodies = []
        for i in range(30):
            if i % 3 == 0:
                body = rng.integers(0, 256, int(rng.integers(1, 3 << 20)), dtype=np.uint8).tobytes()
            elif i % 3 == 1:
                words = [b"nydus", b"chunk", b"dict", b"rafs", b"blob", b"layer", b"gzip\n"]
                body = b" ".join(words[j] for j in rng.integers(0, len(words), 200_000))
            else:
                body = bodies[int(rng.integers(0, len(bodies)))]
            bodies.append(body)
            ti = tarfile.TarInfo(f"d/f{i:02d}")
            ti.size, ti.mtime = len(body), 1_700_000_000
            tw.addfile(ti, io.BytesIO(body))
    tar = out.getvalue()
    gz = _gzip(tar, level)
    stream, res = _pack_ref(gz, piece=123_457)
    dump, meta = _check_layer(oracle, tar, gz, stream)
    # checkpoint table: at least one per MiB of output, increasing offsets
    import struct
    h = meta[-4096:]
    zt_off, zt_size, zt_cnt = struct.unpack_from("<QQQ", h, 40)
    assert zt_cnt >= len(tar) // (2 << 20) and zt_size == 40 * zt_cnt
    outs = [struct.unpack_from("<Q", meta, zt_off + 40 * i + 8)[0] for i in range(zt_cnt)]
    assert outs == sorted(outs) and outs[0] == 0
    assert res["stats"]["intra_chunks"] > 0


def test_ociref_errors():
    """Truncated gzip: the close fails (ETAR); bytes after the gzip stream
    (a second member): EUNSUPP; not gzip at all: ETAR; fs version 5: the
    reference's own error."""
    from nydus_gpu import converter as cv
    import layers
    gz = _gzip(layers.oci_lower_tar())
    with pytest.raises((cv.ConverterError, nydus_gpu.NgpuError)) as e:
        _pack_ref(gz[: len(gz) // 2])
    assert "truncated" in str(e.value)
    with pytest.raises((cv.ConverterError, nydus_gpu.NgpuError)) as e:
        _pack_ref(gz + gz)
    assert "multi-member" in str(e.value)
    with pytest.raises((cv.ConverterError, nydus_gpu.NgpuError)):
        _pack_ref(layers.oci_lower_tar())  # a plain tar is not a gzip blob
    with pytest.raises(cv.ConverterError, match="oci ref can only be supported by fs version 6"):
        cv.Pack(io.BytesIO(), cv.PackOption(OCIRef=True, FsVersion="5"))


def test_ociref_needs_no_dict_and_takes_no_reserve():
    eng = nydus_gpu.Engine()
    try:
        w = eng.pack(ociref=True)
        with pytest.raises(nydus_gpu.NgpuError) as e:
            w.write_zero_copy(b"x" * 100)
        assert e.value.code == nydus_gpu.EINVAL
    finally:
        eng.close()
    assert zlib  # (zlib is what the library inflates with)
