"""Canonical chunk-table dump of a RAFS v6 bootstrap or a nydus blob stream —
the comparison form SURVEY.md §8(f) next-2 asks for in place of
`nydus-image inspect` (unavailable here; the reference reads blob ids the same
way, `nydus-image inspect -R blobs`, pkg/tarfs/tarfs.go:284-306).

Chunk tables are written in hash-map iteration order by nydus-image, so two
converters' tables can only be compared as sets keyed by digest: records are
emitted sorted by (digest, blob id, index) with the blob index replaced by the
blob id.

usage:
  python -m nydus_gpu.inspect FILE            # JSON dump
  python -m nydus_gpu.inspect --diff A B      # exit 0 iff the chunk sets match
FILE may be a bootstrap (image.boot) or a whole Pack output stream.
"""
from __future__ import annotations

import argparse
import json
import sys

from . import rafs
from ._lib import NgpuError, unpack_entry


def load_bootstrap(data: bytes) -> dict:
    """A bootstrap, or the image.boot entry of a nydus blob stream."""
    try:
        rafs.detect_fs_version(data)
        return rafs.read_v6(data)
    except ValueError:
        pass
    try:
        boot, _ = unpack_entry(data, "image.boot")
    except NgpuError as e:
        raise ValueError(f"neither a RAFS v6 bootstrap nor a nydus blob stream: {e}") from e
    return rafs.read_v6(boot)


def canonical(b: dict) -> dict:
    ids = b["blob_ids"]
    recs = []
    for r in b["chunks"]:
        bi = int(r["blob_index"])
        recs.append({"digest": bytes(r["block_id"]).hex(),
                     "blob_id": ids[bi] if bi < len(ids) else f"#{bi}",
                     "flags": int(r["flags"]), "compressed_size": int(r["compressed_size"]),
                     "uncompressed_size": int(r["uncompressed_size"]),
                     "compressed_offset": int(r["compressed_offset"]),
                     "uncompressed_offset": int(r["uncompressed_offset"]),
                     "file_offset": int(r["file_offset"]), "index": int(r["index"])})
    recs.sort(key=lambda x: (x["digest"], x["blob_id"], x["index"]))
    return {"flags": int(b["flags"]), "chunk_size": int(b["chunk_size"]),
            "blobs": sorted(set(ids)), "chunks": recs}


def diff(a: dict, b: dict, fields=("digest", "blob_id", "uncompressed_size")) -> list:
    """Records present in one dump and not the other, compared on `fields`."""
    ka = {tuple(r[f] for f in fields) for r in a["chunks"]}
    kb = {tuple(r[f] for f in fields) for r in b["chunks"]}
    return [("-", k) for k in sorted(ka - kb)] + [("+", k) for k in sorted(kb - ka)]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m nydus_gpu.inspect")
    ap.add_argument("files", nargs="+")
    ap.add_argument("--diff", action="store_true", help="compare the chunk sets of two files")
    args = ap.parse_args(argv)
    dumps = [canonical(load_bootstrap(open(f, "rb").read())) for f in args.files]
    if args.diff:
        if len(dumps) != 2:
            ap.error("--diff takes two files")
        d = diff(*dumps)
        for sign, k in d:
            print(sign, *k)
        return 1 if d else 0
    for dmp in dumps:
        json.dump(dmp, sys.stdout, indent=1)
        print()
    return 0


if __name__ == "__main__":
    sys.exit(main())
