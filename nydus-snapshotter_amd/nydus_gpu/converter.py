"""Host-side mirror of the reference's converter API for the digest/dedup path.

Mirrors pkg/converter (Go) names, argument meaning and error behaviour for the
part this engine replaces; the work itself happens in libnydusgpu.so (GPU
digest/dedup, host C++ blob writer, reader and merge):

* ``PackOption`` / ``MergeOption`` / ``Layer`` — pkg/converter/types.go:37-133
  (fields the path consumes; ``Digester`` is the API extension);
* ``Pack(dest, opt)`` — convert_unix.go:325: returns a write-closer; the caller
  streams the uncompressed layer tar into it; ``close()`` must be checked (it
  raises the builder error, convert_unix.go:323-324).  The GPU engine does the
  chunking/digest/dedup (``ngpu_pack_*``) with the layer kept in HBM;
  ``close()`` writes the nydus formatted stream `data | tar_header | ... |
  toc | tar_header` to ``dest`` (``ngpu_pack_finish``: NEW chunks gathered on
  the GPU, compressed on the host per ``Compressor``, image.boot, TOC);
* ``UnpackEntry(ra, name, target)`` — convert_unix.go:284-320 (TOC first,
  tar-header walk as fallback);
* ``Merge(layers, dest, opt)`` — convert_unix.go:560-666 + tool.Merge
  (builder.go:220-294): unpacks each layer's image.boot, merges the blob and
  chunk tables (no re-hashing) and returns the referenced blob
  digests in first-appearance order; a layer's own blob is named after
  ``Layer.Digest`` (the sha256 of its whole Pack output), so TestPack's
  ``[dict blob, upper blob]`` (tests/converter_test.go:513-519) holds exactly.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import BinaryIO, List, Optional, Sequence

import numpy as np

import hashlib
import io
import tarfile

import threading

import logging

from ._lib import (COMPRESSORS, DICT, ECANCELED, ENOTFOUND, EUNSUPP, NEW, Engine, NgpuError, merge, unpack,
                   unpack_entry)

_log = logging.getLogger("nydus_gpu.converter")

EntryBlob = "image.blob"            # convert_unix.go:45
EntryBootstrap = "image.boot"       # :46
EntryBlobMeta = "blob.meta"         # :47
EntryBlobMetaHeader = "blob.meta.header"  # :48
EntryTOC = "rafs.blob.toc"          # :49

_ENGINES = {}


class ConverterError(RuntimeError):
    """A Go `error` of pkg/converter; `code` is the NGPU_E* code when the
    library refused the request (EUNSUPP: an option the builder does not
    implement)."""

    def __init__(self, msg="", code=None):
        super().__init__(msg)
        self.code = code


class ErrNotFound(ConverterError):
    """types.go:33-35."""


@dataclass
class UnpackOption:
    """pkg/converter/types.go:135-145."""
    WorkDir: str = ""
    BuilderPath: str = ""
    Timeout: Optional[float] = None
    Stream: bool = False


@dataclass
class File:
    """utils.go:24-28: an extra file packToTar puts beside image.boot."""
    Name: str
    Reader: BinaryIO
    Size: int


@dataclass
class Layer:
    """types.go:37-44: Digest of the whole nydus tar blob ("sha256:<hex>") and
    its bytes (ReaderAt)."""
    Digest: str
    ReaderAt: bytes
    OriginalDigest: Optional[str] = None


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


_ENGINES_MU = threading.Lock()


def _engine(opt: PackOption) -> Engine:
    fs = int(opt.FsVersion or "6")
    if fs not in (5, 6):
        raise ConverterError(f"invalid fs version {opt.FsVersion}")
    dg = opt.Digester or "blake3"
    # AlignedChunk only matters for RAFS v5 (types.go:73-74): v6 always aligns
    aligned = bool(opt.AlignedChunk) and fs == 5
    key = (opt.Device, dg, parse_chunk_size(opt.ChunkSize), fs, aligned)
    with _ENGINES_MU:
        if key not in _ENGINES:
            _ENGINES[key] = Engine(device=opt.Device, digester=dg, chunk_size=key[2], fs_version=fs,
                                   aligned_chunk=aligned)
        return _ENGINES[key]


class _PackWriteCloser:
    """One Pack: its own chunk dict handle (ngpu_dict_open: loaded once per
    unchanged ChunkDictPath, shared by every Pack that names it) and its own
    cancel flag, so concurrent Packs on one cached engine never see each
    other's dict (the reference runs one nydus-image per Pack)."""

    def __init__(self, dest: BinaryIO, opt: PackOption, ociref: bool = False):
        self._dest, self._opt = dest, opt
        if (opt.Compressor or "") not in COMPRESSORS:
            raise ConverterError(f"unsupported compressor {opt.Compressor!r}")
        # OCIRef: packRef (builder.go:180-218) passes none of the options but
        # the blob and the source, so nydus-image's defaults apply (v6, 1 MiB
        # chunks, blake3, no chunk dict)
        self._eng = _engine(PackOption(Device=opt.Device) if ociref else opt)
        cd = None
        if opt.ChunkDictPath and not ociref:
            try:
                cd = self._eng.dict_open(opt.ChunkDictPath)
            except NgpuError as e:
                raise ConverterError(f"load chunk dict {opt.ChunkDictPath}: {e}") from e
        try:
            self._w = self._eng.pack(retain=not ociref, dict=cd, ociref=ociref)
        finally:
            if cd is not None:
                cd.release()  # the pack holds its own reference
        # `dest` is known now (convert_unix.go:325): the blob stream leaves while
        # the tar arrives (ngpu_pack_set_output, early emission).
        # PrefetchPatterns: the builder's stdin, "/" by default (builder.go:125-127, 166)
        try:
            self._w.set_output(dest, compressor="" if ociref else (opt.Compressor or ""),
                               prefetch_patterns="" if ociref else opt.PrefetchPatterns)
        except NgpuError as e:
            raise ConverterError(f"pack output: {e}") from e
        self._timer = None
        if opt.Timeout:
            # builder.go:153-158: exec.CommandContext(ctx with Timeout) kills the
            # builder; here the pack's cancel flag stops it
            self._timer = threading.Timer(opt.Timeout, self._w.cancel)
            self._timer.daemon = True
            self._timer.start()
        self.result = None

    def _killed(self, e: NgpuError):
        if e.code == ECANCELED:
            why = f", possibly due to timeout {self._opt.Timeout}s" if self._opt.Timeout else ""
            return ConverterError(f"signal: killed{why}: {e}")
        return e

    def cancel(self):
        """ctx.Done(): the running write/close fails (safe from any thread)."""
        self._w.cancel()

    def write(self, data) -> int:
        try:
            return self._w.write(data)
        except NgpuError as e:
            self._stop_timer()
            raise self._killed(e) from e

    def _stop_timer(self):
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None

    def close(self):
        try:
            ch, res, st, info = self._w.finish(None)  # the rest of the stream (set_output)
        except NgpuError as e:
            raise self._killed(e) from e
        finally:
            self._stop_timer()
        self.result = {"chunks": ch, "results": res, "stats": st, "info": info,
                       "digest": "sha256:" + info["stream_digest"]}
        return self.result


# tool.DetectFeatures (pkg/converter/tool/feature.go:114-146): a Pack's
# required features are checked once per process against the builder's.  The
# builder emulated is the pinned nydus-image v2.3.0 (misc/snapshotter/
# Dockerfile:5), whose `create -h` lists all three (feature_test.go:255, 379),
# so every feature is detected.  Pack() then refuses the two this builder does
# not implement (batch chunks, encryption) with EUNSUPP: the reference hands
# both flags to the builder unconditionally (builder.go:137-142) and never
# returns a blob without them.  A later Pack requiring another set fails
# ("features changed").
FeatureTar2Rafs, FeatureBatchSize, FeatureEncrypt = "--type tar-rafs", "--batch-size", "--encrypt"
_BUILDER_FEATURES = {FeatureTar2Rafs, FeatureBatchSize, FeatureEncrypt}
_FEATURES = {"required": None, "detected": None}
_FEATURES_MU = threading.Lock()


def DetectFeatures(required) -> set:
    required = frozenset(required)
    with _FEATURES_MU:
        if _FEATURES["required"] is None:
            _FEATURES["required"] = required
            det = set()
            for f in sorted(required):
                if f in _BUILDER_FEATURES:
                    det.add(f)
                else:
                    _log.warning("the feature '%s' is ignored, it requires higher version of "
                                 "nydus-image (the GPU builder does not implement it)", f)
            _FEATURES["detected"] = det
        if _FEATURES["required"] != required:
            raise ConverterError(f"features changed: {sorted(_FEATURES['required'])} -> {sorted(required)}")
        return set(_FEATURES["detected"])


def _reset_feature_detection():
    """Tests only: forget the once-per-process detection."""
    with _FEATURES_MU:
        _FEATURES["required"] = _FEATURES["detected"] = None


def Pack(dest: BinaryIO, opt: PackOption) -> _PackWriteCloser:
    """convert_unix.go:325 — returns a writer; stream the layer tar into it and
    check close()."""
    fs = opt.FsVersion or "6"
    required = {FeatureTar2Rafs}
    if opt.BatchSize not in ("", "0"):
        required.add(FeatureBatchSize)
    if opt.Encrypt:
        required.add(FeatureEncrypt)
    detected = DetectFeatures(required)
    if opt.OCIRef:
        if fs != "6":
            raise ConverterError("oci ref can only be supported by fs version 6")
        # packRef (builder.go:180-218): `nydus-image create --type targz-ref`.
        # The writer takes the ORIGINAL gzip layer (LayerConvertFunc passes it
        # undecompressed, convert_unix.go:857-859): inflated and indexed on the
        # host (gzip checkpoints), digested and deduped on the GPU; the stream
        # holds blob.meta (chunk infos + checkpoints), image.boot and the TOC,
        # and the bootstrap's own blob is the gzip blob.
        return _PackWriteCloser(dest, opt, ociref=True)
    if FeatureBatchSize in detected and fs != "6":
        raise ConverterError("'--batch-size' can only be supported by fs version 6")
    # v2.3.0 would write batch chunks (small chunks compressed as one, another
    # blob.meta) or an encrypted blob: refused, never silently dropped
    if FeatureBatchSize in detected:
        raise ConverterError(f"batch chunks (--batch-size {opt.BatchSize}) not implemented by the "
                             "GPU builder", code=EUNSUPP)
    if FeatureEncrypt in detected:
        raise ConverterError("blob encryption (--encrypt) not implemented by the GPU builder",
                             code=EUNSUPP)
    return _PackWriteCloser(dest, opt)


def Unpack(ra: bytes, dest: BinaryIO, opt: Optional[UnpackOption] = None):
    """convert_unix.go:669-719 — the nydus layer stream back to an OCI tar
    (ngpu_unpack: image.boot's inode tree, chunks from image.blob)."""
    try:
        unpack(ra, dest)
    except NgpuError as e:
        raise ConverterError(f"unpack nydus tar: {e}") from e


def UnpackEntry(ra: bytes, targetName: str, target: BinaryIO):
    """convert_unix.go:284-293: copy entry data to target; returns the TOC
    entry (None when found by tar header).  Raises ErrNotFound."""
    try:
        data, toc = unpack_entry(ra, targetName)
    except NgpuError as e:
        if e.code == ENOTFOUND:
            raise ErrNotFound(str(e)) from e
        raise
    target.write(data)
    return toc


def Merge(layers: Sequence[Layer], dest: BinaryIO, opt: MergeOption) -> List[str]:
    """convert_unix.go:560-666 — merge per-layer bootstraps; returns the
    referenced blob digests (sha256:<id>) in first-appearance order."""
    boots, digests, refs = [], [], []
    for layer in layers:
        b = io.BytesIO()
        try:
            UnpackEntry(layer.ReaderAt, EntryBootstrap, b)
        except ConverterError as e:
            raise ConverterError(f"unpack all bootstraps: unpack nydus tar: {e}") from e
        boots.append(b.getvalue())
        # an OCIRef layer's blob is its original gzip blob, named by its
        # OriginalDigest (getBootstrapPath, convert_unix.go:567-573)
        digests.append((layer.OriginalDigest or layer.Digest).split(":", 1)[-1])
        if layer.OriginalDigest:
            # --blob-digests / --blob-sizes / --blob-toc-digests
            # (convert_unix.go:579-587): the nydus stream's digest and size,
            # and calcBlobTOCDigest (:541-554): sha256 of the TOC entry data
            toc = io.BytesIO()
            try:
                UnpackEntry(layer.ReaderAt, EntryTOC, toc)
            except ConverterError as e:
                raise ConverterError(f"calc blob toc digest for layer {layer.Digest}: {e}") from e
            refs.append((layer.Digest.split(":", 1)[-1], len(layer.ReaderAt),
                         hashlib.sha256(toc.getvalue()).hexdigest()))
        else:
            refs.append(None)
    dict_boot = parent = None
    if opt.ChunkDictPath:
        with open(opt.ChunkDictPath, "rb") as f:
            dict_boot = f.read()
    if opt.ParentBootstrapPath:  # --parent-bootstrap (builder.go:235-237)
        with open(opt.ParentBootstrapPath, "rb") as f:
            parent = f.read()
    try:
        merged, ids = merge(boots, digests, dict_boot, parent_bootstrap=parent,
                            prefetch_patterns=opt.PrefetchPatterns, rafs_blobs=refs)
    except NgpuError as e:
        raise ConverterError(f"merge bootstrap: {e}") from e
    if opt.WithTar:  # packToTar (utils.go:92-160): image/ + image/image.boot
        out = io.BytesIO()
        with tarfile.open(fileobj=out, mode="w", format=tarfile.PAX_FORMAT) as tw:
            d = tarfile.TarInfo("image")
            d.type, d.mode = tarfile.DIRTYPE, 0o755
            tw.addfile(d)
            h = tarfile.TarInfo("image/" + EntryBootstrap)
            h.mode, h.size = 0o444, len(merged)
            tw.addfile(h, io.BytesIO(merged))
            for f in opt.AppendFiles:  # File{Name, Reader, Size} (utils.go:24-28)
                h = tarfile.TarInfo("image/" + f.Name)
                h.mode, h.size = 0o444, f.Size
                tw.addfile(h, f.Reader)
        dest.write(out.getvalue())
    else:
        dest.write(merged)
    return ["sha256:" + i for i in ids]


__all__ = ["PackOption", "MergeOption", "UnpackOption", "Layer", "File", "Pack", "Merge", "Unpack",
           "UnpackEntry", "DetectFeatures", "ConverterError",
           "ErrNotFound", "NgpuError", "parse_chunk_size", "EntryBlob", "EntryBootstrap", "EntryTOC"]
