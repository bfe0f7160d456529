"""nydus_gpu — MI355X chunk digest + dedup engine for the nydus conversion path.

Python view of libnydusgpu.so (C ABI in include/nydus_gpu.h).  The engine
replaces the digest/dedup stage that pkg/converter hands to
`nydus-image create` (pkg/converter/tool/builder.go:148-178).
"""
from ._lib import (CHUNK_DTYPE, DICT, DIGESTERS, EXPORTS, HIT_DTYPE, INTRA, KIND_NAMES, MISS,  # noqa: F401
                   LAYER_STATS_DTYPE, NEW, RESULT_DTYPE, Engine, NgpuError, chunk_table, lib, tar_chunks)

__all__ = ["Engine", "NgpuError", "tar_chunks", "chunk_table", "lib", "CHUNK_DTYPE",
           "RESULT_DTYPE", "HIT_DTYPE", "MISS", "NEW", "INTRA", "DICT", "KIND_NAMES", "DIGESTERS", "EXPORTS"]
