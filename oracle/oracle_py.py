"""ctypes loader for liboracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product package.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

CHUNK_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u4"), ("file_index", "<u4"),
                        ("file_offset", "<u8")])
DECISION_DTYPE = np.dtype([("kind", "<u4"), ("index", "<u4"), ("ref", "<u8"),
                           ("blob_index", "<u4"), ("pad", "<u4"), ("uncompressed_offset", "<u8")])
KINDS = {0: "NEW", 1: "INTRA", 2: "DICT"}

_lib = None


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        L.oracle_blake3.argtypes = [vp, ctypes.c_size_t, vp]
        L.oracle_sha256.argtypes = [vp, ctypes.c_size_t, vp]
        L.oracle_tar_chunks.argtypes = [vp, u64, u32, vp, u64, ctypes.POINTER(u64)]
        L.oracle_tar_chunks.restype = ctypes.c_int64
        L.oracle_dedup.argtypes = [vp, vp, u64, vp, vp, vp, vp, vp, u64, u32, vp, ctypes.POINTER(u32)]
        L.oracle_dedup.restype = u64
        L.oracle_digest_chunks.argtypes = [vp, vp, u64, ctypes.c_int, vp]
        L.oracle_cpu_digest_dedup.argtypes = [vp, vp, u64, ctypes.c_int, ctypes.c_int, vp, vp, vp]
        L.oracle_cpu_digest_dedup.restype = u64
        L.oracle_cpu_pack_pipeline.argtypes = [vp, vp, u64, ctypes.c_int, vp, vp, vp, vp,
                                               ctypes.POINTER(ctypes.c_int)]
        L.oracle_cpu_pack_pipeline.restype = u64
        L.oracle_cpu_impl.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def blake3(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_blake3(data, len(data), out)
    return out.raw


def sha256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_sha256(data, len(data), out)
    return out.raw


def digest(data: bytes, digester: str) -> bytes:
    return sha256(data) if digester == "sha256" else blake3(data)


def tar_chunks(tar, chunk_size: int):
    """tar bytes/ndarray -> structured array of CHUNK_DTYPE (restated a3)."""
    buf = np.frombuffer(tar, dtype=np.uint8) if not isinstance(tar, np.ndarray) else tar
    nf = ctypes.c_uint64(0)
    n = lib().oracle_tar_chunks(_ptr(buf), buf.size, chunk_size, None, 0, ctypes.byref(nf))
    if n < 0:
        raise ValueError(f"oracle_tar_chunks failed: {n}")
    out = np.zeros(n, dtype=CHUNK_DTYPE)
    lib().oracle_tar_chunks(_ptr(buf), buf.size, chunk_size, _ptr(out), n, ctypes.byref(nf))
    return out


def digest_chunks(data, chunks, digester: str) -> np.ndarray:
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    ch = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
    out = np.zeros((len(ch), 32), dtype=np.uint8)
    lib().oracle_digest_chunks(_ptr(buf), _ptr(ch), len(ch), 1 if digester == "sha256" else 0, _ptr(out))
    return out


def dedup(digests, sizes, dict_digests=None, dict_sizes=None, dict_blob=None, dict_index=None,
          align=4096, dict_uoff=None):
    """Restated dedup decisions.  DICT decisions copy the dict entry's chunk
    index and uncompressed offset (dict_uoff; 0 when not given)."""
    digests = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1, 32)
    sizes = np.ascontiguousarray(sizes, dtype=np.uint32)
    n = len(sizes)
    m = 0 if dict_digests is None else len(dict_sizes)
    if m:
        dict_digests = np.ascontiguousarray(dict_digests, dtype=np.uint8).reshape(-1, 32)
        dict_sizes = np.ascontiguousarray(dict_sizes, dtype=np.uint32)
        dict_blob = np.ascontiguousarray(dict_blob, dtype=np.uint32)
        dict_index = np.ascontiguousarray(dict_index, dtype=np.uint32)
        if dict_uoff is not None:
            dict_uoff = np.ascontiguousarray(dict_uoff, dtype=np.uint64)
    out = np.zeros(n, dtype=DECISION_DTYPE)
    own = ctypes.c_uint32(0)
    lib().oracle_dedup(_ptr(digests), _ptr(sizes), n, _ptr(dict_digests) if m else None,
                       _ptr(dict_sizes) if m else None, _ptr(dict_blob) if m else None,
                       _ptr(dict_index) if m else None,
                       _ptr(dict_uoff) if m and dict_uoff is not None else None, m, align,
                       _ptr(out), ctypes.byref(own))
    return out, (None if own.value == 0xFFFFFFFF else own.value)


def cpu_digest_dedup(data, chunks, digester: str, threads: int):
    """Timed CPU baseline: SIMD/SHA-NI digests over `threads` + stream dedup."""
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    ch = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
    dig = np.zeros((len(ch), 32), dtype=np.uint8)
    sizes = np.ascontiguousarray(ch["length"], dtype=np.uint32)
    dec = np.zeros(len(ch), dtype=DECISION_DTYPE)
    lib().oracle_cpu_digest_dedup(_ptr(buf), _ptr(ch), len(ch), 1 if digester == "sha256" else 0,
                                  threads, _ptr(dig), _ptr(sizes), _ptr(dec))
    return dig, dec


def cpu_pack_pipeline(data, chunks, digester: str):
    """Timed CPU baseline of one layer's converter pipeline, single-threaded:
    digests + stream dedup + zstd (level 1) of the NEW chunks in blob order +
    SHA-256 of the compressed stream.  -> (compressed bytes, stream digest),
    or None when libzstd / OpenSSL are absent."""
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    ch = np.ascontiguousarray(chunks, dtype=CHUNK_DTYPE)
    dig = np.zeros((len(ch), 32), dtype=np.uint8)
    sizes = np.ascontiguousarray(ch["length"], dtype=np.uint32)
    dec = np.zeros(len(ch), dtype=DECISION_DTYPE)
    sd = np.zeros(32, dtype=np.uint8)
    ok = ctypes.c_int(0)
    total = lib().oracle_cpu_pack_pipeline(_ptr(buf), _ptr(ch), len(ch),
                                           1 if digester == "sha256" else 0, _ptr(dig), _ptr(sizes),
                                           _ptr(dec), _ptr(sd), ctypes.byref(ok))
    return (int(total), sd.tobytes()) if ok.value else None


def cpu_impl() -> str:
    f = lib().oracle_cpu_impl()
    return ("blake3=official-C-SIMD(llvm_blake3)" if f & 1 else "blake3=scalar-oracle") + "," + \
           ("sha256=OpenSSL" if f & 2 else "sha256=scalar-oracle")
