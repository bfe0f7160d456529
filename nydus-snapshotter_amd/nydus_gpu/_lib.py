"""ctypes binding of libnydusgpu.so (include/nydus_gpu.h).

The library is the product: it is loaded from the package directory (built
in-tree by ``make``); there is no fallback implementation — if the .so or a
gfx950 GPU is missing the calls raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# NYDUS_GPU_LIB: an alternative build of the same library (A/B benchmarking)
LIB_PATH = os.environ.get("NYDUS_GPU_LIB") or os.path.join(PKG_DIR, "libnydusgpu.so")

DIGESTERS = {"blake3": 0, "sha256": 1}
KIND_NAMES = {0: "NEW", 1: "INTRA", 2: "DICT", 3: "DIGESTED", 4: "UNHASHED"}
# DIGESTED: a digest-stage record (the dedup stage takes only these; callers
# supplying their own digests set it); UNHASHED: the dedup stage found no
# digest written for the chunk (the call fails with EDEVICE).
NEW, INTRA, DICT, DIGESTED, UNHASHED = 0, 1, 2, 3, 4

ERRORS = {-1: "EINVAL", -2: "EHIP", -3: "ENOMEM", -4: "ETAR", -5: "EUNSUPP",
          -6: "ENODEV", -7: "EIO", -8: "EFORMAT", -9: "ENOTFOUND", -10: "ECANCELED",
          -11: "EDEVICE"}
EINVAL, EUNSUPP, ENODEV, EFORMAT, ENOTFOUND, ECANCELED, EDEVICE = -1, -5, -6, -8, -9, -10, -11

# PackOption.Compressor -> TOCEntry flag values (pkg/converter/types.go:22-31);
# "" is nydus-image's default (zstd).
COMPRESSORS = {"": 0x2, "none": 0x1, "zstd": 0x2, "lz4_block": 0x4}
PACK_RETAIN = 0x1
PACK_OCIREF = 0x2  # ngpu_pack_write takes the original gzip layer (targz-ref)

WRITE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
READ_AT_FN = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                              ctypes.c_uint64)

TOC_ENTRY_DTYPE = np.dtype([("flags", "<u4"), ("reserved1", "<u4"), ("name", "S16"),
                            ("uncompressed_digest", "u1", (32,)), ("compressed_offset", "<u8"),
                            ("compressed_size", "<u8"), ("uncompressed_size", "<u8"),
                            ("reserved2", "u1", (48,))])
assert TOC_ENTRY_DTYPE.itemsize == 128

CHUNK_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u4"), ("file_index", "<u4"),
                        ("file_offset", "<u8")])
RESULT_DTYPE = np.dtype([("digest", "u1", (32,)), ("kind", "<u4"), ("index", "<u4"),
                         ("ref", "<u8"), ("blob_index", "<u4"), ("dict_blob", "<u4"),
                         ("uncompressed_offset", "<u8")])
assert CHUNK_DTYPE.itemsize == 24 and RESULT_DTYPE.itemsize == 64

# Every symbol include/nydus_gpu.h declares (checked by tests/test_host.py).
EXPORTS = ["ngpu_abi_version", "ngpu_create", "ngpu_destroy", "ngpu_last_error",
           "ngpu_device_count", "ngpu_alloc_pinned", "ngpu_free_pinned", "ngpu_dict_load",
           "ngpu_dict_load_bootstrap", "ngpu_dict_clear", "ngpu_dict_size", "ngpu_tar_chunks",
           "ngpu_process", "ngpu_process_device", "ngpu_pack_tar", "ngpu_free_host",
           "ngpu_chunk_table", "ngpu_last_timing", "ngpu_timing_at", "ngpu_digest_device",
           "ngpu_dict_probe_device", "ngpu_dedup_device", "ngpu_dict_load_device",
           "ngpu_pack_open", "ngpu_pack_write", "ngpu_pack_reserve", "ngpu_pack_commit",
           "ngpu_pack_close", "ngpu_pack_abort", "ngpu_dedup_layers_device",
           "ngpu_process_layers_device", "ngpu_host_error", "ngpu_blob_write",
           "ngpu_pack_open_ex", "ngpu_pack_finish", "ngpu_unpack_entry", "ngpu_merge", "ngpu_merge_ex", "ngpu_rafs_dump",
           "ngpu_write_fd", "ngpu_dict_open", "ngpu_dict_create", "ngpu_dict_create_device",
           "ngpu_dict_retain", "ngpu_dict_release", "ngpu_dict_entries", "ngpu_set_dict",
           "ngpu_dict_probe", "ngpu_process_dict", "ngpu_process_dict_device",
           "ngpu_pack_open_dict", "ngpu_pack_set_cancel", "ngpu_node_create", "ngpu_node_destroy",
           "ngpu_node_size", "ngpu_node_engine", "ngpu_node_dict_open", "ngpu_node_dict_create",
           "ngpu_node_owner", "ngpu_node_pack_open", "ngpu_node_process_device",
           "ngpu_device_status", "ngpu_unpack",
           # ABI 4
           "ngpu_dict_create_device_gid", "ngpu_route_digests", "ngpu_route_hits",
           "ngpu_pack_set_output", "ngpu_ref_chunk_read",
           # ABI 5
           "ngpu_node_process_step", "ngpu_batch_stats",
           # ABI 7
           "ngpu_pack_engine", "ngpu_engine_counters_get", "ngpu_merge_ex2"]

LAYER_STATS_DTYPE = np.dtype([("chunks", "<u8"), ("new_chunks", "<u8"), ("intra_chunks", "<u8"),
                              ("dict_chunks", "<u8"), ("new_bytes", "<u8"), ("own_blob_index", "<u4"),
                              ("blobs", "<u4"), ("uncompressed_size", "<u8")])

HIT_DTYPE = np.dtype([("entry", "<u4"), ("index", "<u4"), ("blob", "<u4"), ("usize", "<u4"),
                      ("uncompressed_offset", "<u8")])
assert HIT_DTYPE.itemsize == 24
MISS = 0xFFFFFFFF


class NgpuConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("digester", ctypes.c_uint32),
                ("chunk_size", ctypes.c_uint32), ("fs_version", ctypes.c_uint32),
                ("staging_bytes", ctypes.c_uint64), ("leaves_per_lane", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


FLAG_TIMING = 0x1
FLAG_ALIGNED_CHUNK = 0x2
FLAG_GRID_STAGES = 0x4  # no fused one-workgroup path for small calls (tests / tuning)
FLAG_NO_BATCH = 0x8  # every Pack close its own launches (no batched close of small packs)


class NgpuTiming(ctypes.Structure):
    _fields_ = [("digest_ms", ctypes.c_float), ("tree_ms", ctypes.c_float),
                ("dedup_ms", ctypes.c_float), ("total_ms", ctypes.c_float),
                ("group_log2", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


class NgpuLayerStats(ctypes.Structure):
    _fields_ = [("chunks", ctypes.c_uint64), ("new_chunks", ctypes.c_uint64),
                ("intra_chunks", ctypes.c_uint64), ("dict_chunks", ctypes.c_uint64),
                ("new_bytes", ctypes.c_uint64), ("own_blob_index", ctypes.c_uint32),
                ("blobs", ctypes.c_uint32), ("uncompressed_size", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class NgpuBlobOptions(ctypes.Structure):
    _fields_ = [("compressor", ctypes.c_uint32), ("level", ctypes.c_int32),
                ("threads", ctypes.c_uint32), ("digester", ctypes.c_uint32),
                ("chunk_size", ctypes.c_uint32), ("n_dict_blobs", ctypes.c_uint32),
                ("dict_blobs", ctypes.c_void_p), ("dict_chunks", ctypes.c_void_p),
                ("n_dict_chunks", ctypes.c_uint64), ("fs_version", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("prefetch_patterns", ctypes.c_char_p)]


class NgpuBlobInfo(ctypes.Structure):
    _fields_ = [("stream_bytes", ctypes.c_uint64), ("blob_bytes", ctypes.c_uint64),
                ("bootstrap_bytes", ctypes.c_uint64), ("blob_chunks", ctypes.c_uint64),
                ("compressed_chunks", ctypes.c_uint64), ("stream_digest", ctypes.c_uint8 * 32),
                ("blob_digest", ctypes.c_uint8 * 32), ("toc_digest", ctypes.c_uint8 * 32),
                ("dict_records", ctypes.c_uint64), ("meta_entries", ctypes.c_uint64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_[:5]}
        d["dict_records"] = self.dict_records
        d["meta_entries"] = self.meta_entries
        for k in ("stream_digest", "blob_digest", "toc_digest"):
            d[k] = bytes(getattr(self, k)).hex()
        return d


class NgpuError(RuntimeError):
    def __init__(self, code, msg=""):
        self.code = code
        super().__init__(f"{ERRORS.get(code, code)}: {msg}" if msg else ERRORS.get(code, str(code)))


_lib = None


def lib():
    """Load libnydusgpu.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `make -C {PKG_DIR}` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    pu64 = ctypes.POINTER(u64)
    L.ngpu_abi_version.restype = i32
    L.ngpu_create.argtypes = [ctypes.POINTER(NgpuConfig), ctypes.POINTER(vp)]
    L.ngpu_destroy.argtypes = [vp]
    L.ngpu_destroy.restype = None
    L.ngpu_last_error.argtypes = [vp]
    L.ngpu_last_error.restype = ctypes.c_char_p
    L.ngpu_device_status.argtypes = [vp]
    L.ngpu_device_count.restype = i32
    L.ngpu_alloc_pinned.argtypes = [vp, u64, ctypes.POINTER(vp)]
    L.ngpu_free_pinned.argtypes = [vp, vp]
    L.ngpu_dict_load.argtypes = [vp, vp, vp, vp, vp, u64]
    L.ngpu_dict_load_bootstrap.argtypes = [vp, ctypes.c_char_p]
    L.ngpu_dict_clear.argtypes = [vp]
    L.ngpu_dict_size.argtypes = [vp]
    L.ngpu_dict_size.restype = u64
    L.ngpu_tar_chunks.argtypes = [vp, u64, u32, vp, u64, pu64, pu64]
    L.ngpu_process.argtypes = [vp, vp, u64, vp, u64, vp, ctypes.POINTER(NgpuLayerStats)]
    L.ngpu_process_device.argtypes = [vp, vp, u64, vp, u64, vp, vp, ctypes.POINTER(NgpuLayerStats)]
    L.ngpu_pack_tar.argtypes = [vp, vp, u64, ctypes.POINTER(vp), ctypes.POINTER(vp), pu64,
                                ctypes.POINTER(NgpuLayerStats)]
    L.ngpu_free_host.argtypes = [vp]
    L.ngpu_free_host.restype = None
    L.ngpu_chunk_table.argtypes = [vp, vp, u64, vp, u64, pu64]
    L.ngpu_last_timing.argtypes = [vp, ctypes.POINTER(NgpuTiming)]
    L.ngpu_timing_at.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(NgpuTiming)]
    L.ngpu_batch_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    L.ngpu_digest_device.argtypes = [vp, vp, u64, vp, u64, vp, vp]
    L.ngpu_dict_probe_device.argtypes = [vp, vp, u64, u64, vp, vp]
    L.ngpu_dedup_device.argtypes = [vp, vp, u64, vp, vp, u32, vp, ctypes.POINTER(NgpuLayerStats)]
    L.ngpu_dict_load_device.argtypes = [vp, vp, vp, vp, vp, u64, u32]
    L.ngpu_dedup_layers_device.argtypes = [vp, vp, u64, vp, vp, u32, vp, u64, vp, vp]
    L.ngpu_process_layers_device.argtypes = [vp, vp, u64, vp, u64, vp, vp, u64, vp, vp]
    L.ngpu_pack_open.argtypes = [vp, ctypes.POINTER(vp)]
    L.ngpu_pack_write.argtypes = [vp, vp, u64]
    L.ngpu_pack_reserve.argtypes = [vp, ctypes.POINTER(vp), pu64]
    L.ngpu_pack_commit.argtypes = [vp, u64]
    L.ngpu_pack_close.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), pu64,
                                  ctypes.POINTER(NgpuLayerStats)]
    L.ngpu_pack_abort.argtypes = [vp]
    L.ngpu_pack_abort.restype = None
    L.ngpu_host_error.restype = ctypes.c_char_p
    L.ngpu_blob_write.argtypes = [vp, u64, vp, vp, u64, ctypes.POINTER(NgpuLayerStats),
                                  ctypes.POINTER(NgpuBlobOptions), WRITE_FN, vp,
                                  ctypes.POINTER(NgpuBlobInfo)]
    L.ngpu_pack_open_ex.argtypes = [vp, u32, ctypes.POINTER(vp)]
    L.ngpu_pack_finish.argtypes = [vp, ctypes.POINTER(NgpuBlobOptions), WRITE_FN, vp,
                                   ctypes.POINTER(vp), ctypes.POINTER(vp), pu64,
                                   ctypes.POINTER(NgpuLayerStats), ctypes.POINTER(NgpuBlobInfo)]
    L.ngpu_unpack_entry.argtypes = [READ_AT_FN, vp, u64, ctypes.c_char_p, WRITE_FN, vp, vp]
    L.ngpu_unpack.argtypes = [READ_AT_FN, vp, u64, WRITE_FN, vp]
    L.ngpu_rafs_dump.argtypes = [vp, u64, WRITE_FN, vp]
    L.ngpu_merge.argtypes = [ctypes.POINTER(vp), pu64, ctypes.POINTER(ctypes.c_char_p), u64, vp,
                             u64, WRITE_FN, vp, ctypes.POINTER(vp)]
    L.ngpu_merge_ex.argtypes = [ctypes.POINTER(vp), pu64, ctypes.POINTER(ctypes.c_char_p), u64, vp,
                                u64, ctypes.POINTER(NgpuMergeOptions), WRITE_FN, vp, ctypes.POINTER(vp)]
    L.ngpu_merge_ex2.argtypes = [ctypes.POINTER(vp), pu64, ctypes.POINTER(ctypes.c_char_p), u64, vp,
                                 u64, ctypes.POINTER(NgpuMergeOptions), vp, vp, vp, WRITE_FN, vp,
                                 ctypes.POINTER(vp)]
    L.ngpu_pack_engine.argtypes = [vp]
    L.ngpu_pack_engine.restype = vp
    L.ngpu_engine_counters_get.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    L.ngpu_dict_open.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.ngpu_dict_create.argtypes = [vp, vp, u64, vp, u32, ctypes.POINTER(vp)]
    L.ngpu_dict_create_device.argtypes = [vp, vp, vp, vp, vp, vp, u64, u32, ctypes.POINTER(vp)]
    L.ngpu_dict_create_device_gid.argtypes = [vp, vp, vp, vp, vp, vp, vp, u64, u32, ctypes.POINTER(vp)]
    L.ngpu_route_digests.argtypes = [vp, u64, u64, u32, u64, u32, vp, vp, vp, vp]
    L.ngpu_route_hits.argtypes = [vp, vp, u64, vp, vp]
    L.ngpu_pack_set_output.argtypes = [vp, ctypes.c_void_p, WRITE_FN, vp]
    L.ngpu_ref_chunk_read.argtypes = [vp, u64, vp, u64, u32, vp, u32, ctypes.POINTER(u32)]
    L.ngpu_dict_retain.argtypes = [vp]
    L.ngpu_dict_retain.restype = None
    L.ngpu_dict_release.argtypes = [vp]
    L.ngpu_dict_release.restype = None
    L.ngpu_dict_entries.argtypes = [vp]
    L.ngpu_dict_entries.restype = u64
    L.ngpu_set_dict.argtypes = [vp, vp]
    L.ngpu_dict_probe.argtypes = [vp, vp, u64, u64, vp, vp]
    L.ngpu_process_dict.argtypes = [vp, vp, vp, u64, vp, u64, vp, ctypes.POINTER(NgpuLayerStats)]
    L.ngpu_process_dict_device.argtypes = [vp, vp, vp, u64, vp, u64, vp, vp, u64, vp, vp,
                                           ctypes.POINTER(NgpuLayerStats)]
    L.ngpu_pack_open_dict.argtypes = [vp, vp, u32, ctypes.POINTER(vp)]
    L.ngpu_pack_set_cancel.argtypes = [vp, vp]
    L.ngpu_node_create.argtypes = [vp, u32, ctypes.POINTER(NgpuConfig), ctypes.POINTER(vp)]
    L.ngpu_node_destroy.argtypes = [vp]
    L.ngpu_node_destroy.restype = None
    L.ngpu_node_size.argtypes = [vp]
    L.ngpu_node_size.restype = u32
    L.ngpu_node_engine.argtypes = [vp, u32]
    L.ngpu_node_engine.restype = vp
    L.ngpu_node_dict_open.argtypes = [vp, ctypes.c_char_p, u32, ctypes.POINTER(vp)]
    L.ngpu_node_dict_create.argtypes = [vp, vp, u64, vp, u32, u32, ctypes.POINTER(vp)]
    L.ngpu_node_owner.argtypes = [vp, vp]
    L.ngpu_node_owner.restype = u32
    L.ngpu_node_pack_open.argtypes = [vp, vp, u32, ctypes.POINTER(vp)]
    L.ngpu_node_process_device.argtypes = [vp, u32, vp, vp, u64, vp, u64, vp, vp, u64, vp, vp]
    L.ngpu_node_process_step.argtypes = [vp, vp, ctypes.POINTER(NgpuNodePart), u32, u32]
    _lib = L
    return L


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else None


def _buf(data):
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return np.frombuffer(data, dtype=np.uint8)


def tar_chunks(tar, chunk_size: int = 0x100000):
    """Host tar front end: tar bytes -> CHUNK_DTYPE array (no GPU needed)."""
    L = lib()
    buf = _buf(tar)
    n, nf = ctypes.c_uint64(0), ctypes.c_uint64(0)
    # one walk: every chunk holds >= 1 of its file's 512-B data blocks, so
    # len / 512 + 1 bounds the count (capped; a second walk only if exceeded)
    cap = min(buf.size // 512 + 1, 1 << 20)
    out = np.zeros(cap, dtype=CHUNK_DTYPE)
    rc = L.ngpu_tar_chunks(_ptr(buf), buf.size, chunk_size, _ptr(out), cap, ctypes.byref(n),
                           ctypes.byref(nf))
    if rc:
        raise NgpuError(rc, "tar parse")
    if n.value > cap:
        out = np.zeros(n.value, dtype=CHUNK_DTYPE)
        rc = L.ngpu_tar_chunks(_ptr(buf), buf.size, chunk_size, _ptr(out), n.value, ctypes.byref(n),
                               ctypes.byref(nf))
        if rc:
            raise NgpuError(rc, "tar parse")
    return out[:n.value].copy() if n.value < cap else out


def chunk_table(chunks, results) -> np.ndarray:
    """RAFS v6 chunk-info records (n x 80 bytes) of the layer's NEW chunks."""
    L = lib()
    ch = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
    rs = np.ascontiguousarray(results, dtype=RESULT_DTYPE)
    n = ctypes.c_uint64(0)
    rc = L.ngpu_chunk_table(_ptr(ch), _ptr(rs), len(ch), None, 0, ctypes.byref(n))
    if rc:
        raise NgpuError(rc, "chunk table")
    out = np.zeros((n.value, 80), dtype=np.uint8)
    rc = L.ngpu_chunk_table(_ptr(ch), _ptr(rs), len(ch), _ptr(out), n.value, ctypes.byref(n))
    if rc:
        raise NgpuError(rc, "chunk table")
    return out


def _host_check(rc, what):
    if rc:
        msg = lib().ngpu_host_error()
        raise NgpuError(rc, f"{what}: {msg.decode() if msg else ''}")


class FdWriter:
    """dest for blob streams written straight from C (ngpu_write_fd) to a file
    descriptor, without a Python callback per batch."""

    def __init__(self, fd: int):
        self.fd = fd


class _Sink:
    """io.Writer -> ngpu_write_fn (exceptions are kept and re-raised)."""

    def __init__(self, dest):
        self.dest, self.exc = dest, None
        if isinstance(dest, FdWriter):
            self.fn = WRITE_FN(ctypes.cast(lib().ngpu_write_fd, ctypes.c_void_p).value)
            self.ctx = ctypes.c_void_p(dest.fd)
            return
        self.ctx = None

        def fn(_ctx, buf, n):
            try:
                self.dest.write(ctypes.string_at(buf, n))
                return 0
            except BaseException as e:  # noqa: BLE001 - re-raised by the caller
                self.exc = e
                return 1
        self.fn = WRITE_FN(fn)

    def reraise(self):
        if self.exc is not None:
            raise self.exc


def blob_options(compressor: str = "", level: int = 0, threads: int = 0, digester: str = "blake3",
                 chunk_size: int = 0x100000, dict_blobs: np.ndarray = None,
                 dict_chunks: np.ndarray = None, fs_version: int = 6, prefetch_patterns: str = ""):
    if compressor not in COMPRESSORS:
        raise ValueError(f"unsupported compressor {compressor!r}")
    pf = prefetch_patterns.encode() if prefetch_patterns else None
    o = NgpuBlobOptions(compressor=COMPRESSORS[compressor], level=level, threads=threads,
                        digester=DIGESTERS[digester], chunk_size=chunk_size, fs_version=fs_version,
                        prefetch_patterns=pf)
    keep = [pf]
    if dict_blobs is not None and len(dict_blobs):
        b = np.ascontiguousarray(dict_blobs).view(np.uint8).reshape(-1)
        o.n_dict_blobs = b.size // 256
        o.dict_blobs = b.ctypes.data
        keep.append(b)
    if dict_chunks is not None and len(dict_chunks):
        c = np.ascontiguousarray(dict_chunks).view(np.uint8).reshape(-1)
        o.n_dict_chunks = c.size // 80
        o.dict_chunks = c.ctypes.data
        keep.append(c)
    return o, keep


def blob_write(data, chunks, results, stats: dict, dest, compressor: str = "", level: int = 0,
               threads: int = 0, digester: str = "blake3", chunk_size: int = 0x100000,
               dict_blobs: np.ndarray = None, dict_chunks: np.ndarray = None, fs_version: int = 6,
               prefetch_patterns: str = "") -> dict:
    """Host: write the nydus blob stream of a packed layer to `dest` (a
    writable file-like); returns the ngpu_blob_info as a dict."""
    L = lib()
    buf = _buf(data)
    ch = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
    rs = np.ascontiguousarray(results, dtype=RESULT_DTYPE)
    st = NgpuLayerStats(**{k: stats[k] for k, _ in NgpuLayerStats._fields_})
    o, keep = blob_options(compressor, level, threads, digester, chunk_size, dict_blobs, dict_chunks,
                           fs_version, prefetch_patterns)
    sink = _Sink(dest)
    info = NgpuBlobInfo()
    rc = L.ngpu_blob_write(_ptr(buf), buf.size, _ptr(ch), _ptr(rs), len(ch), ctypes.byref(st),
                           ctypes.byref(o), sink.fn, sink.ctx, ctypes.byref(info))
    sink.reraise()
    _host_check(rc, "blob_write")
    del keep
    return info.as_dict()


def unpack_entry(blob, name: str):
    """UnpackEntry (convert_unix.go:284-320) over bytes / a numpy buffer:
    returns (entry data, TOC entry record or None when found by tar header).
    Raises NgpuError(ENOTFOUND) like ErrNotFound."""
    L = lib()
    src = _buf(blob)

    def ra(_ctx, buf, n, off):
        n = min(n, src.size - off)
        if n <= 0:
            return -1
        ctypes.memmove(buf, src.ctypes.data + off, n)
        return n
    rfn = READ_AT_FN(ra)
    out = []
    sink = _Sink(type("W", (), {"write": lambda _s, b: out.append(b)})())
    toc = np.zeros(1, TOC_ENTRY_DTYPE)
    rc = L.ngpu_unpack_entry(rfn, None, src.size, name.encode(), sink.fn, None, _ptr(toc))
    sink.reraise()
    _host_check(rc, f"unpack_entry {name}")
    return b"".join(out), (toc[0] if toc[0]["name"] else None)


def unpack(blob, dest=None):
    """Unpack (convert_unix.go:669-719): a packed layer's nydus stream (bytes /
    numpy buffer) back to an OCI tar, written to `dest` (file-like) or
    returned as bytes."""
    L = lib()
    src = _buf(blob)

    def ra(_ctx, buf, n, off):
        n = min(n, src.size - off)
        if n <= 0:
            return -1
        ctypes.memmove(buf, src.ctypes.data + off, n)
        return n
    rfn = READ_AT_FN(ra)
    out = []
    sink = _Sink(dest if dest is not None else type("W", (), {"write": lambda _s, b: out.append(b)})())
    rc = L.ngpu_unpack(rfn, None, src.size, sink.fn, None)
    sink.reraise()
    _host_check(rc, "unpack")
    return None if dest is not None else b"".join(out)


def rafs_dump(bootstrap: bytes) -> dict:
    """ngpu_rafs_dump: the canonical JSON view of a RAFS v5 / v6 bootstrap
    (the `nydus-image inspect` restatement), parsed."""
    import json
    L = lib()
    buf = _buf(bootstrap)
    out = []
    sink = _Sink(type("W", (), {"write": lambda _s, b: out.append(b)})())
    rc = L.ngpu_rafs_dump(_ptr(buf), buf.size, sink.fn, None)
    sink.reraise()
    _host_check(rc, "rafs_dump")
    return json.loads(b"".join(out).decode("ascii"))


def ref_chunk_read(gz, blob_meta, index: int, cap: int = 1 << 24) -> bytes:
    """ngpu_ref_chunk_read: chunk `index` of an OCIRef layer's own blob, out of
    the original gzip blob through the checkpoints in its blob.meta entry."""
    g, m = _buf(gz), _buf(blob_meta)
    out = np.empty(cap, np.uint8)
    n = ctypes.c_uint32(0)
    _host_check(lib().ngpu_ref_chunk_read(_ptr(g), g.size, _ptr(m), m.size, index, _ptr(out), cap,
                                          ctypes.byref(n)), "ref_chunk_read")
    return out[: n.value].tobytes()


def route_digests(d_digests: int, stride: int, n: int, world: int, d_out: int, d_rows: int,
                  d_counts: int, seg_cap: int = 0, rounds: int = 0, stream: int = 0):
    """ngpu_route_digests (device pointers, async on `stream`): each digest to
    its owner's segment of d_out with its row id in d_rows; d_counts (128 u32)
    receives the per-owner counts.  seg_cap > 0: padded [rounds][world][seg_cap]."""
    rc = lib().ngpu_route_digests(ctypes.c_void_p(d_digests) if d_digests else None, stride, n, world,
                                  seg_cap, rounds, ctypes.c_void_p(d_out) if d_out else None,
                                  ctypes.c_void_p(d_rows) if d_rows else None,
                                  ctypes.c_void_p(d_counts), ctypes.c_void_p(stream) if stream else None)
    if rc:
        raise NgpuError(rc, "route_digests")


def route_hits(d_routed: int, d_rows: int, m: int, d_hits: int, stream: int = 0):
    """ngpu_route_hits: d_hits[d_rows[i]] = d_routed[i] (padding rows skipped)."""
    rc = lib().ngpu_route_hits(ctypes.c_void_p(d_routed) if d_routed else None,
                               ctypes.c_void_p(d_rows) if d_rows else None, m,
                               ctypes.c_void_p(d_hits) if d_hits else None,
                               ctypes.c_void_p(stream) if stream else None)
    if rc:
        raise NgpuError(rc, "route_hits")


class NgpuMergeOptions(ctypes.Structure):
    _fields_ = [("parent_bootstrap", ctypes.c_void_p), ("parent_size", ctypes.c_uint64),
                ("prefetch_patterns", ctypes.c_char_p)]


def merge(bootstraps, layer_digests, dict_bootstrap: bytes = None, parent_bootstrap: bytes = None,
          prefetch_patterns: str = "", rafs_blobs=None):
    """ngpu_merge_ex2: per-layer bootstraps (bytes, lowest first) + layer digest
    hex strings -> (merged bootstrap bytes, [blob ids in first-appearance
    order]).  The merged bootstrap holds the overlaid inode tree.
    rafs_blobs: per layer None, or (RAFS blob digest hex, size, TOC digest
    hex) for a targz-ref layer (Merge's --blob-digests / --blob-sizes /
    --blob-toc-digests, builder.go:242-253)."""
    L = lib()
    bufs = [_buf(b) for b in bootstraps]
    n = len(bufs)
    ptrs = (ctypes.c_void_p * max(1, n))(*[b.ctypes.data for b in bufs])
    sizes = (ctypes.c_uint64 * max(1, n))(*[b.size for b in bufs])
    digs = (ctypes.c_char_p * max(1, n))(*[(d or "").encode() for d in layer_digests])
    dbuf = _buf(dict_bootstrap) if dict_bootstrap is not None else None
    out = []
    sink = _Sink(type("W", (), {"write": lambda _s, b: out.append(b)})())
    ids = ctypes.c_void_p()
    pbuf = _buf(parent_bootstrap) if parent_bootstrap is not None else None
    opt = NgpuMergeOptions(_ptr(pbuf) if pbuf is not None else None, pbuf.size if pbuf is not None else 0,
                           (prefetch_patterns or "").encode())
    rd = rs = rt = None
    if rafs_blobs is not None and any(r is not None for r in rafs_blobs):
        rd = (ctypes.c_char_p * max(1, n))(*[r[0].encode() if r else None for r in rafs_blobs])
        rs = (ctypes.c_uint64 * max(1, n))(*[int(r[1]) if r else 0 for r in rafs_blobs])
        rt = (ctypes.c_char_p * max(1, n))(*[r[2].encode() if r else None for r in rafs_blobs])
    rc = L.ngpu_merge_ex2(ptrs, sizes, digs, n, _ptr(dbuf) if dbuf is not None else None,
                          dbuf.size if dbuf is not None else 0, ctypes.byref(opt), rd, rs, rt,
                          sink.fn, None, ctypes.byref(ids))
    sink.reraise()
    _host_check(rc, "merge")
    try:
        s = ctypes.string_at(ids).decode()
    finally:
        L.ngpu_free_host(ids)
    return b"".join(out), (s.split(",") if s else [])


DEFAULT_DICT = object()  # "the engine's default dict" (the calls without a dict argument)


class ChunkDict:
    """A chunk dict handle (ngpu_dict*): the HBM-resident HashChunkDict of one
    ChunkDictPath (or of arrays), reference counted.  A pack opened with it
    keeps its own reference, so releasing the handle never disturbs a pack."""

    def __init__(self, handle):
        self._h = handle

    @property
    def handle(self) -> int:
        return self._h.value if self._h else 0

    @property
    def entries(self) -> int:
        return lib().ngpu_dict_entries(self._h)

    def release(self):
        if getattr(self, "_h", None):
            lib().ngpu_dict_release(self._h)
            self._h = None

    __del__ = release

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.release()

    def probe_device(self, d_digests: int, stride: int, n: int, d_hits: int, stream: int = 0):
        rc = lib().ngpu_dict_probe(self._h, ctypes.c_void_p(d_digests), stride, n,
                                   ctypes.c_void_p(d_hits), ctypes.c_void_p(stream) if stream else None)
        if rc:
            raise NgpuError(rc, "dict_probe")


def _dict_arg(d):
    return None if d is None else d._h


class Engine:
    """One GPU engine (ngpu_engine*).  Mirrors the PackOption fields the
    digest/dedup stage consumes (pkg/converter/types.go:58-90)."""

    @classmethod
    def _borrow(cls, handle, owner, digester, chunk_size, fs_version):
        """A view of an engine owned by something else (a Node): close() is a no-op."""
        e = cls.__new__(cls)
        e._h, e._owner = handle, owner
        e.digester, e.chunk_size, e.fs_version = digester, chunk_size, fs_version
        return e

    def __init__(self, device: int = 0, digester: str = "blake3", chunk_size: int = 0x100000,
                 fs_version: int = 6, leaves_per_lane: int = 0, staging_bytes: int = 0,
                 timing: bool = False, flags: int = 0, aligned_chunk: bool = False):
        self._owner = None
        L = lib()
        if digester not in DIGESTERS:
            raise ValueError(f"unsupported digester {digester!r}")
        cfg = NgpuConfig(device=device, digester=DIGESTERS[digester], chunk_size=chunk_size,
                         fs_version=fs_version, staging_bytes=staging_bytes,
                         leaves_per_lane=leaves_per_lane,
                         flags=flags | (FLAG_TIMING if timing else 0) |
                         (FLAG_ALIGNED_CHUNK if aligned_chunk else 0))
        h = ctypes.c_void_p()
        rc = L.ngpu_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc:
            raise NgpuError(rc, "ngpu_create")
        self._h = h
        self.digester = digester
        self.chunk_size = chunk_size
        self.fs_version = fs_version

    def close(self):
        if getattr(self, "_h", None) and getattr(self, "_owner", None) is None:
            lib().ngpu_destroy(self._h)
        self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what):
        if rc:
            msg = lib().ngpu_last_error(self._h)
            raise NgpuError(rc, f"{what}: {msg.decode() if msg else ''}")

    def device_status(self):
        """ngpu_device_status: raise the first error a device-pointer stage
        recorded since the last check (waits for the engine's streams)."""
        self._check(lib().ngpu_device_status(self._h), "device_status")

    def dict_load(self, digests, usize, blob_index, chunk_index=None):
        d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1, 32)
        us = np.ascontiguousarray(usize, dtype=np.uint32)
        bl = np.ascontiguousarray(blob_index, dtype=np.uint32)
        ci = None if chunk_index is None else np.ascontiguousarray(chunk_index, dtype=np.uint32)
        self._check(lib().ngpu_dict_load(self._h, _ptr(d), _ptr(us), _ptr(bl), _ptr(ci), len(us)),
                    "dict_load")

    def dict_load_bootstrap(self, path: str):
        self._check(lib().ngpu_dict_load_bootstrap(self._h, path.encode()), "dict_load_bootstrap")

    def dict_clear(self):
        self._check(lib().ngpu_dict_clear(self._h), "dict_clear")

    def dict_open(self, path: str) -> ChunkDict:
        """ngpu_dict_open: load (or reuse, if unchanged) a RAFS v6 chunk-dict bootstrap."""
        h = ctypes.c_void_p()
        self._check(lib().ngpu_dict_open(self._h, path.encode(), ctypes.byref(h)), "dict_open")
        return ChunkDict(h)

    def dict_create(self, records, blobs=None) -> ChunkDict:
        """From 80-B RAFS v6 chunk records (table order) + 256-B blob records."""
        r = np.ascontiguousarray(records).view(np.uint8).reshape(-1)
        b = None if blobs is None or not len(blobs) else np.ascontiguousarray(blobs).view(np.uint8).reshape(-1)
        h = ctypes.c_void_p()
        self._check(lib().ngpu_dict_create(self._h, _ptr(r), r.size // 80, _ptr(b),
                                           0 if b is None else b.size // 256, ctypes.byref(h)),
                    "dict_create")
        return ChunkDict(h)

    def dict_create_device(self, d_digests: int, d_usize: int, d_blob: int, d_index: int, n: int,
                           n_blobs: int, d_uoff: int = 0, d_gid: int = 0) -> ChunkDict:
        """d_gid: device u32 global entry ids (0 = positions), so a shard of a
        partitioned dict answers with global ids (ngpu_dict_create_device_gid)."""
        h = ctypes.c_void_p()
        self._check(lib().ngpu_dict_create_device_gid(
            self._h, self._vp(d_digests), self._vp(d_usize), self._vp(d_blob), self._vp(d_index),
            self._vp(d_uoff), self._vp(d_gid), n, n_blobs, ctypes.byref(h)), "dict_create_device")
        return ChunkDict(h)

    def set_dict(self, d):
        self._check(lib().ngpu_set_dict(self._h, _dict_arg(d)), "set_dict")

    @property
    def dict_size(self) -> int:
        return lib().ngpu_dict_size(self._h)

    def process(self, data, chunks, dict=DEFAULT_DICT):
        """Host data + chunk descriptors -> (RESULT_DTYPE array, stats dict).
        dict: a ChunkDict, None (no dict) or the engine's default."""
        buf = _buf(data)
        ch = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
        out = np.zeros(len(ch), dtype=RESULT_DTYPE)
        st = NgpuLayerStats()
        if dict is DEFAULT_DICT:
            rc = lib().ngpu_process(self._h, _ptr(buf), buf.size, _ptr(ch), len(ch), _ptr(out),
                                    ctypes.byref(st))
        else:
            rc = lib().ngpu_process_dict(self._h, _dict_arg(dict), _ptr(buf), buf.size, _ptr(ch),
                                         len(ch), _ptr(out), ctypes.byref(st))
        self._check(rc, "process")
        return out, st.as_dict()

    def process_dict_device(self, dict, d_data: int, length: int, d_chunks: int, n: int, d_out: int,
                            d_layer_first: int = 0, n_layers: int = 1, d_stats: int = 0,
                            stream: int = 0, want_stats: bool = False):
        st = NgpuLayerStats()
        self._check(lib().ngpu_process_dict_device(
            self._h, _dict_arg(dict), self._vp(d_data), length, self._vp(d_chunks), n, self._vp(d_out),
            self._vp(d_layer_first), n_layers, self._vp(d_stats), self._vp(stream),
            ctypes.byref(st) if want_stats else None), "process_dict_device")
        return st.as_dict() if want_stats else None

    def process_device(self, d_data: int, length: int, d_chunks: int, n: int, d_out: int,
                       stream: int = 0, want_stats: bool = False):
        """Device pointers in (ints), enqueue on `stream`; returns stats if asked
        (which synchronises)."""
        st = NgpuLayerStats()
        self._check(lib().ngpu_process_device(self._h, ctypes.c_void_p(d_data), length,
                                              ctypes.c_void_p(d_chunks), n, ctypes.c_void_p(d_out),
                                              ctypes.c_void_p(stream) if stream else None,
                                              ctypes.byref(st) if want_stats else None),
                    "process_device")
        return st.as_dict() if want_stats else None

    # ---- split stages, device pointers (ints) ---------------------------------
    @staticmethod
    def _vp(x):
        return ctypes.c_void_p(x) if x else None

    def digest_device(self, d_data: int, length: int, d_chunks: int, n: int, d_out: int,
                      stream: int = 0):
        self._check(lib().ngpu_digest_device(self._h, self._vp(d_data), length, self._vp(d_chunks),
                                             n, self._vp(d_out), self._vp(stream)), "digest_device")

    def dict_probe_device(self, d_digests: int, stride: int, n: int, d_hits: int, stream: int = 0):
        self._check(lib().ngpu_dict_probe_device(self._h, self._vp(d_digests), stride, n,
                                                 self._vp(d_hits), self._vp(stream)), "dict_probe_device")

    def dedup_device(self, d_chunks: int, n: int, d_out: int, d_hits: int = 0, n_dict_blobs: int = 0,
                     stream: int = 0, want_stats: bool = False):
        st = NgpuLayerStats()
        self._check(lib().ngpu_dedup_device(self._h, self._vp(d_chunks), n, self._vp(d_out),
                                            self._vp(d_hits), n_dict_blobs, self._vp(stream),
                                            ctypes.byref(st) if want_stats else None), "dedup_device")
        return st.as_dict() if want_stats else None

    def dedup_layers_device(self, d_chunks: int, n: int, d_out: int, d_layer_first: int,
                            n_layers: int, d_stats: int = 0, d_hits: int = 0, n_dict_blobs: int = 0,
                            stream: int = 0):
        self._check(lib().ngpu_dedup_layers_device(self._h, self._vp(d_chunks), n, self._vp(d_out),
                                                   self._vp(d_hits), n_dict_blobs,
                                                   self._vp(d_layer_first), n_layers, self._vp(d_stats),
                                                   self._vp(stream)), "dedup_layers_device")

    def process_layers_device(self, d_data: int, length: int, d_chunks: int, n: int, d_out: int,
                              d_layer_first: int, n_layers: int, d_stats: int = 0, stream: int = 0):
        self._check(lib().ngpu_process_layers_device(self._h, self._vp(d_data), length,
                                                     self._vp(d_chunks), n, self._vp(d_out),
                                                     self._vp(d_layer_first), n_layers,
                                                     self._vp(d_stats), self._vp(stream)),
                    "process_layers_device")

    def dict_load_device(self, d_digests: int, d_usize: int, d_blob: int, d_index: int, n: int,
                         n_blobs: int):
        self._check(lib().ngpu_dict_load_device(self._h, self._vp(d_digests), self._vp(d_usize),
                                                self._vp(d_blob), self._vp(d_index), n, n_blobs),
                    "dict_load_device")

    def last_timing(self) -> dict:
        t = NgpuTiming()
        self._check(lib().ngpu_last_timing(self._h, ctypes.byref(t)), "last_timing")
        return t.as_dict()

    def batch_stats(self) -> dict:
        """Batched Pack closes (batch.hip): launch sets, packs in them, most in one."""
        out = (ctypes.c_uint64 * 3)()
        self._check(lib().ngpu_batch_stats(self._h, out), "batch_stats")
        return {"batches": out[0], "packs": out[1], "max_packs": out[2]}

    def counters(self) -> dict:
        """ngpu_engine_counters_get: what the engine holds now (open packs,
        pooled staging / stream sets) -- the leak check of abort paths."""
        out = (ctypes.c_uint64 * 8)()
        self._check(lib().ngpu_engine_counters_get(self._h, out), "engine_counters")
        keys = ("open_packs", "staging_pool_bufs", "staging_pool_bytes", "pack_pool", "land_pool",
                "batch_waitable")
        return {k: int(out[i]) for i, k in enumerate(keys)}

    def timing_at(self, back: int) -> dict:
        """Stage timings of the call `back` calls before the last one (the
        engine keeps its last 64); lets a caller time back-to-back calls
        without synchronising between them."""
        t = NgpuTiming()
        self._check(lib().ngpu_timing_at(self._h, back, ctypes.byref(t)), "timing_at")
        return t.as_dict()

    def pack(self, retain: bool = False, dict=DEFAULT_DICT, ociref: bool = False) -> "PackWriter":
        """Streaming Pack (converter.Pack mirror): returns a writer.  retain=True
        keeps the layer in HBM so finish() can write the nydus blob stream.
        dict: a ChunkDict, None, or the engine's default at open time.
        ociref=True (PackOption.OCIRef, targz-ref): write() takes the original
        gzip layer blob; no chunk dict."""
        return PackWriter(self, retain, None if ociref else dict, ociref)

    def pack_tar(self, tar):
        """Whole tar layer -> (chunks, results, stats)."""
        L = lib()
        buf = _buf(tar)
        pc, pr = ctypes.c_void_p(), ctypes.c_void_p()
        n = ctypes.c_uint64(0)
        st = NgpuLayerStats()
        self._check(L.ngpu_pack_tar(self._h, _ptr(buf), buf.size, ctypes.byref(pc), ctypes.byref(pr),
                                    ctypes.byref(n), ctypes.byref(st)), "pack_tar")
        try:
            nn = n.value
            ch = np.empty(nn, dtype=CHUNK_DTYPE)
            rs = np.empty(nn, dtype=RESULT_DTYPE)
            if nn:
                ctypes.memmove(ch.ctypes.data, pc, nn * CHUNK_DTYPE.itemsize)
                ctypes.memmove(rs.ctypes.data, pr, nn * RESULT_DTYPE.itemsize)
        finally:
            L.ngpu_free_host(pc)
            L.ngpu_free_host(pr)
        return ch, rs, st.as_dict()


class PackWriter:
    """Mirror of the io.WriteCloser returned by converter.Pack
    (pkg/converter/convert_unix.go:325): write() the uncompressed layer tar in
    any split, close() -> (chunks, results, stats).  Errors raise NgpuError;
    a failed writer is released (like Close() reporting the builder error)."""

    _out = None  # set_output: (options, keep-alive arrays, sink)

    def __init__(self, engine: Engine, retain: bool = False, dict=DEFAULT_DICT, ociref: bool = False):
        self._eng = engine
        h = ctypes.c_void_p()
        fl = (PACK_RETAIN if retain else 0) | (PACK_OCIREF if ociref else 0)
        if dict is DEFAULT_DICT:
            rc = lib().ngpu_pack_open_ex(engine._h, fl, ctypes.byref(h))
        else:
            rc = lib().ngpu_pack_open_dict(engine._h, _dict_arg(dict), fl, ctypes.byref(h))
        engine._check(rc, "pack_open")
        self._p = h
        self._out = None  # set_output: (options, keep-alive arrays, sink)
        # cancel flag (ngpu_pack_set_cancel): caller-owned, outlives the pack
        self._cancel = ctypes.c_int32(0)
        lib().ngpu_pack_set_cancel(self._p, ctypes.byref(self._cancel))

    def set_output(self, dest, compressor: str = "", level: int = 0, threads: int = 0,
                   dict_blobs: np.ndarray = None, prefetch_patterns: str = ""):
        """ngpu_pack_set_output (needs retain=True, before the first write): the
        blob stream goes to `dest` while the tar is written; finish() then
        completes it (call finish() with no dest)."""
        o, keep = blob_options(compressor, level, threads, self._eng.digester, self._eng.chunk_size,
                               dict_blobs, fs_version=self._eng.fs_version,
                               prefetch_patterns=prefetch_patterns)
        sink = _Sink(dest)
        rc = lib().ngpu_pack_set_output(self._p, ctypes.byref(o), sink.fn, sink.ctx)
        if rc:
            self.abort()
            self._eng._check(rc, "pack_set_output")
        self._out = (o, keep, sink)

    def cancel(self):
        """ctx.Done(): the running or next write / close fails with ECANCELED.
        Safe to call from another thread."""
        self._cancel.value = 1

    def write(self, data) -> int:
        buf = _buf(data)
        rc = lib().ngpu_pack_write(self._p, _ptr(buf), buf.size)
        if rc:
            self.abort()
            if self._out is not None:
                self._out[2].reraise()  # dest failed under the emitter
            self._eng._check(rc, "pack_write")
        return buf.size

    def write_zero_copy(self, data) -> int:
        """Copy into the engine's pinned staging via reserve/commit."""
        L = lib()
        buf = _buf(data)
        off = 0
        while off < buf.size:
            ptr, avail = ctypes.c_void_p(), ctypes.c_uint64(0)
            rc = L.ngpu_pack_reserve(self._p, ctypes.byref(ptr), ctypes.byref(avail))
            if rc:
                self.abort()
                self._eng._check(rc, "pack_reserve")
            take = min(avail.value, buf.size - off)
            ctypes.memmove(ptr.value, buf.ctypes.data + off, take)
            rc = L.ngpu_pack_commit(self._p, take)
            if rc:
                self.abort()
                self._eng._check(rc, "pack_commit")
            off += take
        return buf.size

    def abort(self):
        if self._p:
            lib().ngpu_pack_abort(self._p)
            self._p = None

    def close(self):
        ch, rs, st, _ = self._finish(None)
        return ch, rs, st

    def finish(self, dest, compressor: str = "", level: int = 0, threads: int = 0,
               dict_blobs: np.ndarray = None, prefetch_patterns: str = ""):
        """close() + write the nydus blob stream to `dest` (needs retain=True).
        Returns (chunks, results, stats, blob info dict)."""
        return self._finish(dest, compressor, level, threads, dict_blobs, prefetch_patterns)

    def _finish(self, dest, compressor="", level=0, threads=0, dict_blobs=None, prefetch_patterns=""):
        L = lib()
        pc, pr = ctypes.c_void_p(), ctypes.c_void_p()
        n = ctypes.c_uint64(0)
        st = NgpuLayerStats()
        info = NgpuBlobInfo()
        p, self._p = self._p, None
        if dest is None and self._out is not None:  # the stream already flows (set_output)
            sink = self._out[2]
            rc = L.ngpu_pack_finish(p, None, WRITE_FN(), None, ctypes.byref(pc), ctypes.byref(pr),
                                    ctypes.byref(n), ctypes.byref(st), ctypes.byref(info))
            sink.reraise()
            dest = sink.dest
        elif dest is None:
            rc = L.ngpu_pack_finish(p, None, WRITE_FN(), None, ctypes.byref(pc), ctypes.byref(pr),
                                    ctypes.byref(n), ctypes.byref(st), None)
            sink = None
        else:
            o, keep = blob_options(compressor, level, threads, self._eng.digester,
                                   self._eng.chunk_size, dict_blobs, fs_version=self._eng.fs_version,
                                   prefetch_patterns=prefetch_patterns)
            sink = _Sink(dest)
            rc = L.ngpu_pack_finish(p, ctypes.byref(o), sink.fn, sink.ctx, ctypes.byref(pc),
                                    ctypes.byref(pr), ctypes.byref(n), ctypes.byref(st),
                                    ctypes.byref(info))
            sink.reraise()
        self._eng._check(rc, "pack_finish")
        try:
            nn = n.value
            ch = np.empty(nn, dtype=CHUNK_DTYPE)
            rs = np.empty(nn, dtype=RESULT_DTYPE)
            if nn:
                ctypes.memmove(ch.ctypes.data, pc, nn * CHUNK_DTYPE.itemsize)
                ctypes.memmove(rs.ctypes.data, pr, nn * RESULT_DTYPE.itemsize)
        finally:
            L.ngpu_free_host(pc)
            L.ngpu_free_host(pr)
        return ch, rs, st.as_dict(), (info.as_dict() if dest is not None else None)


class NgpuNodePart(ctypes.Structure):
    """ngpu_node_part: one device's share of a node step (device pointers)."""
    _fields_ = [("d_data", ctypes.c_void_p), ("len", ctypes.c_uint64), ("d_chunks", ctypes.c_void_p),
                ("n", ctypes.c_uint64), ("d_out", ctypes.c_void_p), ("d_layer_first", ctypes.c_void_p),
                ("n_layers", ctypes.c_uint64), ("d_stats", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


NODE_STEP_RCCL = 1  # ngpu_node_process_step: the all-to-alls are RCCL ncclAllToAllv
NODE_DICT_PARTITION, NODE_DICT_REPLICATE = 0, 1
NODE_EXCHANGE_COPY = 0x100  # | PARTITION: the broadcast + DMA exchange (the default since ABI 7)
NODE_EXCHANGE_ROUTED = 0x200  # | PARTITION: the peer-kernel exchange (opt-in since ABI 7)


class Node:
    """One process driving several GPUs (ngpu_node*): one
    engine per listed device (a device may repeat, to rehearse a multi-GPU
    node on one GPU); node chunk dicts are partitioned by digest prefix (the
    probe exchange runs over xGMI) or replicated."""

    def __init__(self, devices, digester: str = "blake3", chunk_size: int = 0x100000,
                 fs_version: int = 6, staging_bytes: int = 0, timing: bool = False, flags: int = 0):
        L = lib()
        cfg = NgpuConfig(device=0, digester=DIGESTERS[digester], chunk_size=chunk_size,
                         fs_version=fs_version, staging_bytes=staging_bytes,
                         flags=flags | (FLAG_TIMING if timing else 0))
        devs = (ctypes.c_int32 * len(devices))(*devices)
        h = ctypes.c_void_p()
        rc = L.ngpu_node_create(devs, len(devices), ctypes.byref(cfg), ctypes.byref(h))
        if rc:
            raise NgpuError(rc, "ngpu_node_create")
        self._h = h
        self.devices = list(devices)
        self.digester, self.chunk_size = digester, chunk_size
        self.engines = [Engine._borrow(ctypes.c_void_p(L.ngpu_node_engine(h, i)), self, digester,
                                       chunk_size, fs_version) for i in range(len(devices))]

    def close(self):
        if getattr(self, "_h", None):
            for e in self.engines:
                e._h = None
            lib().ngpu_node_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __len__(self):
        return lib().ngpu_node_size(self._h)

    def owner(self, digest: bytes) -> int:
        b = np.frombuffer(bytes(digest), np.uint8)
        return lib().ngpu_node_owner(self._h, _ptr(b))

    def _err(self, rc, what):
        if rc:
            msg = lib().ngpu_last_error(self.engines[0]._h)
            raise NgpuError(rc, f"{what}: {msg.decode() if msg else ''}")

    def dict_open(self, path: str, mode: int = NODE_DICT_PARTITION) -> ChunkDict:
        h = ctypes.c_void_p()
        self._err(lib().ngpu_node_dict_open(self._h, path.encode(), mode, ctypes.byref(h)),
                  "node_dict_open")
        return ChunkDict(h)

    def dict_create(self, records, blobs=None, mode: int = NODE_DICT_PARTITION) -> ChunkDict:
        r = np.ascontiguousarray(records).view(np.uint8).reshape(-1)
        b = None if blobs is None or not len(blobs) else np.ascontiguousarray(blobs).view(np.uint8).reshape(-1)
        h = ctypes.c_void_p()
        self._err(lib().ngpu_node_dict_create(self._h, _ptr(r), r.size // 80, _ptr(b),
                                              0 if b is None else b.size // 256, mode, ctypes.byref(h)),
                  "node_dict_create")
        return ChunkDict(h)

    def pack(self, dict=None, retain: bool = False) -> "PackWriter":
        """A streaming Pack on the least-loaded engine (fewest open packs);
        its `part` attribute is the node index it was placed on."""
        h = ctypes.c_void_p()
        self._err(lib().ngpu_node_pack_open(self._h, _dict_arg(dict), PACK_RETAIN if retain else 0,
                                            ctypes.byref(h)), "node_pack_open")
        w = PackWriter.__new__(PackWriter)
        # the pack's engine, for error messages and finish() options
        eh = lib().ngpu_pack_engine(h)
        w.part = next(i for i, e in enumerate(self.engines) if e._h.value == eh)
        w._eng = self.engines[w.part]
        w._p = h
        w._cancel = ctypes.c_int32(0)
        lib().ngpu_pack_set_cancel(w._p, ctypes.byref(w._cancel))
        return w

    def process_step(self, dict, parts, rccl: bool = False):
        """ngpu_node_process_step: every device's part at once, one all-to-all-v
        each way (RCCL with rccl=True, peer copies otherwise).  parts: one dict
        per node device with keys d_data, len, d_chunks, n, d_out and optionally
        d_layer_first, n_layers, d_stats, stream (ints: device pointers)."""
        arr = (NgpuNodePart * len(parts))()
        for i, p in enumerate(parts):
            arr[i] = NgpuNodePart(p.get("d_data", 0) or None, p.get("len", 0),
                                  p.get("d_chunks", 0) or None, p.get("n", 0), p.get("d_out", 0) or None,
                                  p.get("d_layer_first", 0) or None, p.get("n_layers", 1 if p.get("d_layer_first") else 0),
                                  p.get("d_stats", 0) or None, p.get("stream", 0) or None)
        self._err(lib().ngpu_node_process_step(self._h, _dict_arg(dict), arr, len(parts),
                                               NODE_STEP_RCCL if rccl else 0), "node_process_step")

    def process_device(self, i: int, dict, d_data: int, length: int, d_chunks: int, n: int,
                       d_out: int, d_layer_first: int = 0, n_layers: int = 1, d_stats: int = 0,
                       stream: int = 0):
        vp = Engine._vp
        self.engines[i]._check(lib().ngpu_node_process_device(
            self._h, i, _dict_arg(dict), vp(d_data), length, vp(d_chunks), n, vp(d_out),
            vp(d_layer_first), n_layers, vp(d_stats), vp(stream)), "node_process_device")
