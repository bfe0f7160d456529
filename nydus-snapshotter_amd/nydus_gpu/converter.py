"""Host-side mirror of the reference's converter API for the digest/dedup path.

Mirrors pkg/converter (Go) names, argument meaning and error behaviour for the
part this engine replaces:

* ``PackOption`` / ``MergeOption`` — pkg/converter/types.go:58-133 (fields the
  path consumes; ``Digester`` is the API extension);
* ``Pack(dest, opt)`` — convert_unix.go:325: returns a write-closer; the caller
  streams the uncompressed layer tar into it; ``close()`` must be checked (it
  raises the builder error, convert_unix.go:323-324).  The GPU engine does the
  chunking/digest/dedup (libnydusgpu.so ``ngpu_pack_*``); ``close()`` writes a
  RAFS v6 bootstrap with the layer's blob table and chunk table to ``dest``;
* ``Merge(layers, dest, opt)`` — convert_unix.go:560 + tool.Merge
  (builder.go:220-294): blob bookkeeping only (merge does not
  re-hash).  Returns the referenced blob digests in first-appearance order,
  e.g. ``[dict, upper]`` for TestPack (tests/converter_test.go:513-519).

Out of scope here: compression and the blob data /
TOC stream.  The layer's own blob ID is therefore derived from its content
identity — SHA-256 over the NEW chunks' digests in index order — instead of
the SHA-256 of the compressed blob nydus-image would write.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import BinaryIO, List, Optional, Sequence

import numpy as np

from . import rafs
from ._lib import DICT, NEW, Engine, NgpuError, chunk_table

_ENGINES = {}


class ConverterError(RuntimeError):
    pass


@dataclass
class PackOption:
    """pkg/converter/types.go:58-90 (fields used by the digest/dedup stage)."""
    WorkDir: str = ""
    BuilderPath: str = ""
    FsVersion: str = ""          # "5" | "6" (default "6", builder.go:79-81)
    ChunkDictPath: str = ""      # bootstrap of the chunk dict image
    PrefetchPatterns: str = ""
    Compressor: str = ""
    OCIRef: bool = False
    AlignedChunk: bool = False
    ChunkSize: str = ""          # power of two in [0x1000, 0x1000000] (types.go:76)
    BatchSize: str = ""
    Timeout: Optional[float] = None
    Encrypt: bool = False
    Digester: str = ""           # API extension: "blake3" (default) | "sha256"
    Device: int = 0              # GPU ordinal


@dataclass
class MergeOption:
    """pkg/converter/types.go:92-133 (fields used by the blob bookkeeping)."""
    WorkDir: str = ""
    BuilderPath: str = ""
    FsVersion: str = ""
    ChunkDictPath: str = ""
    ParentBootstrapPath: str = ""
    PrefetchPatterns: str = ""
    WithTar: bool = False
    OCI: bool = False
    OCIRef: bool = False
    Timeout: Optional[float] = None
    AppendFiles: list = field(default_factory=list)


def parse_chunk_size(s: str) -> int:
    if not s:
        return 0x100000
    v = int(s, 0)
    if v & (v - 1) or v < 0x1000 or v > 0x1000000:
        raise ConverterError(f"invalid chunk size {s}: must be power of two in [0x1000, 0x1000000]")
    return v


def _engine(opt: PackOption) -> Engine:
    fs = int(opt.FsVersion or "6")
    if fs not in (5, 6):
        raise ConverterError(f"invalid fs version {opt.FsVersion}")
    dg = opt.Digester or "blake3"
    key = (opt.Device, dg, parse_chunk_size(opt.ChunkSize), fs)
    if key not in _ENGINES:
        _ENGINES[key] = Engine(device=opt.Device, digester=dg, chunk_size=key[2], fs_version=fs)
    return _ENGINES[key]


def _own_blob_id(chunks: np.ndarray, results: np.ndarray) -> str:
    new = results[results["kind"] == NEW]
    return hashlib.sha256(new["digest"].tobytes()).hexdigest()


class _PackWriteCloser:
    def __init__(self, dest: BinaryIO, opt: PackOption):
        self._dest, self._opt = dest, opt
        self._eng = _engine(opt)
        self._dict_ids: List[str] = []
        self._dict_blob: Optional[np.ndarray] = None
        if opt.ChunkDictPath:
            with open(opt.ChunkDictPath, "rb") as f:
                boot = rafs.read_v6(f.read())
            self._dict_ids = boot["blob_ids"]
            self._dict_blob = boot["chunks"]["blob_index"].astype(np.int64)
            self._eng.dict_load_bootstrap(opt.ChunkDictPath)
        else:
            self._eng.dict_clear()
        self._w = self._eng.pack()
        self.result = None

    def write(self, data) -> int:
        return self._w.write(data)

    def close(self):
        ch, res, st = self._w.close()
        # blob table in real-index order (first-hit allocation, VERIFY semantics)
        nblobs = int(st["blobs"])
        ids: List[Optional[str]] = [None] * nblobs
        own = st["own_blob_index"]
        own_id = _own_blob_id(ch, res) if own != 0xFFFFFFFF else None
        if own != 0xFFFFFFFF:
            ids[own] = own_id
        d = res[res["kind"] == DICT]
        for r in d:
            inner = int(self._dict_blob[int(r["ref"])])
            ids[int(r["blob_index"])] = self._dict_ids[inner] if inner < len(self._dict_ids) else \
                f"{inner:064x}"
        if any(i is None for i in ids):
            raise ConverterError("inconsistent blob table")
        cs = parse_chunk_size(self._opt.ChunkSize)
        counts = [int((res["kind"] == NEW).sum()) if i == own else 0 for i in range(nblobs)]
        blobs = rafs.make_blob_table(ids, cs, counts, self._opt.Digester or "blake3")
        recs = chunk_table(ch, res).view(rafs.CHUNK_INFO_DTYPE).reshape(-1)
        flags = 0x4 if (self._opt.Digester or "blake3") == "blake3" else 0x0
        self._dest.write(rafs.write_v6_bootstrap(recs, cs, flags=flags, blobs=blobs))
        self.result = {"chunks": ch, "results": res, "stats": st, "blob_ids": ids, "own_blob_id": own_id}
        return self.result


def Pack(dest: BinaryIO, opt: PackOption) -> _PackWriteCloser:
    """convert_unix.go:325 — returns a writer; stream the layer tar into it and
    check close()."""
    if opt.OCIRef:
        raise ConverterError("OCIRef packing has no chunk digest stage (not accelerated)")
    return _PackWriteCloser(dest, opt)


def Merge(layers: Sequence[bytes], dest: BinaryIO, opt: MergeOption) -> List[str]:
    """convert_unix.go:560 — merge per-layer bootstraps; returns the referenced
    blob digests (sha256:<id>) in first-appearance order.  Each layer may hold
    dict blobs plus at most one blob of its own ([nydus v2.3.0] merge.rs)."""
    blob_ids: List[str] = []
    chunks = []
    cs = 0
    for boot_bytes in layers:
        boot = rafs.read_v6(boot_bytes)
        cs = cs or boot["chunk_size"]
        local = []
        for bid in boot["blob_ids"]:
            if bid not in blob_ids:
                blob_ids.append(bid)
            local.append(blob_ids.index(bid))
        recs = boot["chunks"].copy()
        if len(recs):
            recs["blob_index"] = np.asarray(local, np.uint32)[recs["blob_index"]]
        chunks.append(recs)
    allrecs = np.concatenate(chunks) if chunks else np.zeros(0, rafs.CHUNK_INFO_DTYPE)
    counts = [int((allrecs["blob_index"] == i).sum()) for i in range(len(blob_ids))]
    dest.write(rafs.write_v6_bootstrap(allrecs, cs or 0x100000,
                                       blobs=rafs.make_blob_table(blob_ids, cs or 0x100000, counts)))
    return ["sha256:" + b for b in blob_ids]


__all__ = ["PackOption", "MergeOption", "Pack", "Merge", "ConverterError", "NgpuError", "parse_chunk_size"]
