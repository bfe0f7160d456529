"""nydus_gpu — MI355X chunk digest + dedup engine for the nydus conversion path.

Python view of libnydusgpu.so (C ABI in include/nydus_gpu.h).  The engine
replaces the digest/dedup stage that pkg/converter hands to
`nydus-image create` (pkg/converter/tool/builder.go:148-178).
"""
from ._lib import (CHUNK_DTYPE, COMPRESSORS, DEFAULT_DICT, DICT, DIGESTED, DIGESTERS,  # noqa: F401
                   ECANCELED, EDEVICE, EFORMAT, EINVAL, ENODEV, EUNSUPP, UNHASHED,
                   ENOTFOUND, EXPORTS, FLAG_GRID_STAGES, FLAG_NO_BATCH, HIT_DTYPE, FdWriter, INTRA, KIND_NAMES, LAYER_STATS_DTYPE, MISS, NEW,
                   RESULT_DTYPE, TOC_ENTRY_DTYPE, ChunkDict, Engine, Node, NODE_DICT_PARTITION,
                   NODE_DICT_REPLICATE, NODE_EXCHANGE_COPY, NODE_EXCHANGE_ROUTED, NODE_STEP_RCCL, NgpuError, blob_write, chunk_table,
                   lib, merge, rafs_dump, ref_chunk_read, route_digests, route_hits, tar_chunks, unpack,
                   unpack_entry)

__all__ = ["Engine", "Node", "NODE_DICT_PARTITION", "NODE_DICT_REPLICATE", "NODE_EXCHANGE_COPY", "NODE_EXCHANGE_ROUTED", "NODE_STEP_RCCL",
           "route_digests", "route_hits", "ref_chunk_read", "ChunkDict", "DEFAULT_DICT", "NgpuError", "tar_chunks", "chunk_table", "lib", "CHUNK_DTYPE",
           "RESULT_DTYPE", "HIT_DTYPE", "MISS", "NEW", "INTRA", "DICT", "DIGESTED", "UNHASHED", "KIND_NAMES", "DIGESTERS", "EXPORTS",
           "COMPRESSORS", "TOC_ENTRY_DTYPE", "FdWriter", "blob_write", "unpack_entry", "unpack", "merge", "rafs_dump",
           "FLAG_GRID_STAGES", "FLAG_NO_BATCH", "EINVAL", "EFORMAT", "ENODEV", "EUNSUPP", "ENOTFOUND", "ECANCELED", "EDEVICE"]
