"""RAFS v6 bootstrap chunk-table helpers (host side, no GPU).

Layout (pkg/layout/layout.go:18-27; record format decoded from the
reference fixture pkg/filesystem/testdata/v6-bootstrap-chunk-pos-438272.tar.gz,
SURVEY.md §8(c)):

* v6 super block at 1024 (magic 0xE0F5E1E2), extended super block at 1152:
  ``flags u64, blob_table_offset u64, blob_table_size u32, chunk_size u32,
  chunk_table_offset u64 (@1176 = RafsV6ChunkInfoOffset), chunk_table_size u64,
  prefetch_table_offset u64, prefetch_table_size u32``;
* chunk table = 80-byte records (CHUNK_INFO_DTYPE).

``canonical`` gives the inspect-equivalent comparison form: the table as a set
keyed by digest (nydus writes it in hash-map iteration order, so byte order is
meaningless).
"""
from __future__ import annotations

import struct
import tarfile

import numpy as np

RAFS_V6_MAGIC = 0xE0F5E1E2
RAFS_V5_MAGIC = 0x52414653
SUPER_OFFSET = 1024
EXT_OFFSET = 1024 + 128
CHUNK_INFO_OFFSET = 1024 + 128 + 24  # layout.go:27

CHUNK_INFO_DTYPE = np.dtype([("block_id", "u1", (32,)), ("blob_index", "<u4"), ("flags", "<u4"),
                             ("compressed_size", "<u4"), ("uncompressed_size", "<u4"),
                             ("compressed_offset", "<u8"), ("uncompressed_offset", "<u8"),
                             ("file_offset", "<u8"), ("index", "<u4"), ("reserved", "<u4")])
assert CHUNK_INFO_DTYPE.itemsize == 80

CHUNK_FLAG_COMPRESSED = 0x1

# RAFS v6 blob table entry (256 B), decoded from the same fixture: 64 ASCII hex
# chars of blob id, then blob_index, chunk_size, chunk_count,
# compression_algo, digest_algo, features (u32 each), compressed_size,
# uncompressed_size (u64), rest meta-info fields (zero here).
BLOB_DTYPE = np.dtype([("blob_id", "S64"), ("blob_index", "<u4"), ("chunk_size", "<u4"),
                       ("chunk_count", "<u4"), ("compression_algo", "<u4"), ("digest_algo", "<u4"),
                       ("features", "<u4"), ("compressed_size", "<u8"), ("uncompressed_size", "<u8"),
                       ("reserved", "u1", (152,))])
assert BLOB_DTYPE.itemsize == 256
DIGEST_ALGO = {"blake3": 0, "sha256": 1}
COMPRESSOR_NONE = 0


def detect_fs_version(header: bytes) -> str:
    """Port of DetectFsVersion (pkg/layout/layout.go:60-76)."""
    if len(header) < 8:
        raise ValueError("header buffer to DetectFsVersion is too small")
    magic, ver = struct.unpack_from("<II", header, 0)
    if magic == RAFS_V5_MAGIC and ver == 0x500:
        return "v5"
    if len(header) >= 1024 + 128 + 256 and struct.unpack_from("<I", header, SUPER_OFFSET)[0] == RAFS_V6_MAGIC:
        return "v6"
    raise ValueError("unknown file system header")


def read_v6(boot: bytes) -> dict:
    if detect_fs_version(boot) != "v6":
        raise ValueError("not a RAFS v6 bootstrap")
    flags, bto, bts, cs, cto, cts, pto, pts = struct.unpack_from("<QQIIQQQI", boot, EXT_OFFSET)
    if cts % 80:
        raise ValueError("chunk table size is not a multiple of 80")
    table = np.frombuffer(boot, dtype=CHUNK_INFO_DTYPE, count=cts // 80, offset=cto).copy()
    blobs = np.frombuffer(boot, dtype=BLOB_DTYPE, count=bts // 256, offset=bto).copy() if bts else \
        np.zeros(0, BLOB_DTYPE)
    return {"flags": flags, "blob_table_offset": bto, "blob_table_size": bts, "chunk_size": cs,
            "chunk_table_offset": cto, "chunk_table_size": cts, "chunks": table, "blobs": blobs,
            "blob_ids": [b.decode() for b in blobs["blob_id"]]}


def read_v6_from_targz(path: str) -> dict:
    """The reference fixtures ship image/image.boot inside a .tar.gz."""
    with tarfile.open(path, "r:gz") as tf:
        for m in tf.getmembers():
            if m.name.endswith("image.boot"):
                return read_v6(tf.extractfile(m).read())
    raise ValueError("no image.boot in archive")


def make_blob_table(blob_ids, chunk_size, counts=None, digester="blake3", sizes=None) -> np.ndarray:
    t = np.zeros(len(blob_ids), BLOB_DTYPE)
    for i, bid in enumerate(blob_ids):
        t[i]["blob_id"] = bid.encode() if isinstance(bid, str) else bid
        t[i]["blob_index"] = i
        t[i]["chunk_size"] = chunk_size
        t[i]["chunk_count"] = counts[i] if counts is not None else 0
        t[i]["compression_algo"] = COMPRESSOR_NONE
        t[i]["digest_algo"] = DIGEST_ALGO[digester]
        if sizes is not None:
            t[i]["compressed_size"] = t[i]["uncompressed_size"] = sizes[i]
    return t


def write_v6_bootstrap(records: np.ndarray, chunk_size: int, flags: int = 0x4,
                       blobs: np.ndarray = None) -> bytes:
    """Minimal RAFS v6 bootstrap: super blocks + blob table (at 0x1000, as in
    the reference fixture) + chunk table.  Enough for ChunkDictPath loading,
    Merge's blob bookkeeping and chunk-table comparison (no inodes)."""
    recs = np.ascontiguousarray(records).view(CHUNK_INFO_DTYPE)
    blobs = np.zeros(0, BLOB_DTYPE) if blobs is None else np.ascontiguousarray(blobs, BLOB_DTYPE)
    bto = 4096
    cto = bto + (blobs.nbytes + 4095) // 4096 * 4096
    buf = bytearray(cto + recs.nbytes)
    struct.pack_into("<I", buf, SUPER_OFFSET, RAFS_V6_MAGIC)
    struct.pack_into("<QQIIQQQI", buf, EXT_OFFSET, flags, bto if blobs.size else 0, blobs.nbytes,
                     chunk_size, cto, recs.nbytes, 0, 0)
    buf[bto:bto + blobs.nbytes] = blobs.tobytes()
    buf[cto:] = recs.tobytes()
    return bytes(buf)


def write_v6_dict_file(path: str, n_records: int, chunk_size: int, pieces, flags: int = 0x4,
                       blobs: np.ndarray = None) -> int:
    """The same minimal RAFS v6 bootstrap as write_v6_bootstrap, written to
    `path` with its chunk table streamed from `pieces` (an iterable of
    CHUNK_INFO_DTYPE arrays, n_records in all): a ChunkDictPath file of any
    size without holding its table in memory.  -> bytes written."""
    head = bytearray(write_v6_bootstrap(np.zeros(0, CHUNK_INFO_DTYPE), chunk_size, flags, blobs))
    cto = len(head)
    struct.pack_into("<Q", head, EXT_OFFSET + 32, n_records * 80)  # chunk_table_size
    done = 0
    with open(path, "wb") as f:
        f.write(head)
        for p in pieces:
            p = np.ascontiguousarray(p).view(CHUNK_INFO_DTYPE).reshape(-1)
            p.tofile(f)
            done += len(p)
    if done != n_records:
        raise ValueError(f"{done} records written, {n_records} declared")
    return cto + 80 * n_records


def canonical(records: np.ndarray):
    """inspect-equivalent canonical form: sorted by digest."""
    recs = np.asarray(records).view(CHUNK_INFO_DTYPE).reshape(-1)
    rows = [(bytes(r["block_id"]).hex(), int(r["blob_index"]), int(r["flags"]),
             int(r["compressed_size"]), int(r["uncompressed_size"]), int(r["compressed_offset"]),
             int(r["uncompressed_offset"]), int(r["file_offset"]), int(r["index"])) for r in recs]
    return sorted(rows)


def check_offset_rules(records: np.ndarray, align: int = 4096):
    """The layout rules the v6 fixture obeys (and our writer must): indices are a
    permutation of 0..n-1; in index order, uncompressed offsets advance by the
    align-rounded size and compressed offsets by the compressed size."""
    recs = np.asarray(records).view(CHUNK_INFO_DTYPE).reshape(-1)
    order = np.argsort(recs["index"], kind="stable")
    r = recs[order]
    if not np.array_equal(r["index"], np.arange(len(r))):
        return False
    uo = r["uncompressed_offset"].astype(np.int64)
    us = r["uncompressed_size"].astype(np.int64)
    co = r["compressed_offset"].astype(np.int64)
    cs = r["compressed_size"].astype(np.int64)
    exp_u = np.concatenate([[uo[0] if len(uo) else 0], (uo[:-1] + us[:-1] + align - 1) // align * align])
    exp_c = np.concatenate([[co[0] if len(co) else 0], co[:-1] + cs[:-1]])
    return bool(np.array_equal(uo, exp_u) and np.array_equal(co, exp_c))

