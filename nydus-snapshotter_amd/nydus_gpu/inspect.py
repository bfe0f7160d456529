"""Canonical chunk-table dump of a RAFS v5 / v6 bootstrap or a nydus blob stream —
the comparison form SURVEY.md §8(f) next-2 asks for in place of
`nydus-image inspect` (unavailable here; the reference reads blob ids the same
way, `nydus-image inspect -R blobs`, pkg/tarfs/tarfs.go:284-306).

Chunk tables are written in hash-map iteration order by nydus-image, so two
converters' tables can only be compared as sets keyed by digest: records are
emitted sorted by (digest, blob id, index) with the blob index replaced by the
blob id.

A v5 bootstrap has no chunk table: its records are the chunk infos of every
file's inode, one per distinct (digest, blob, index).  `--tree` dumps the inode
tree instead (ngpu_rafs_dump: every inode depth first with its metadata and
chunk records), and `--diff --tree` compares two trees path by path.

usage:
  python -m nydus_gpu.inspect FILE            # JSON dump of the chunk set
  python -m nydus_gpu.inspect --tree FILE     # JSON dump of the inode tree
  python -m nydus_gpu.inspect --diff A B      # exit 0 iff the chunk sets match
  python -m nydus_gpu.inspect --diff --tree A B  # exit 0 iff the trees match
FILE may be a bootstrap (image.boot) or a whole Pack output stream.
"""
from __future__ import annotations

import argparse
import json
import sys

import numpy as np

from . import rafs
from ._lib import NgpuError, rafs_dump, unpack_entry


def bootstrap_bytes(data: bytes) -> bytes:
    """A bootstrap as is, or the image.boot entry of a nydus blob stream."""
    try:
        rafs.detect_fs_version(data)
        return data
    except ValueError:
        pass
    try:
        return unpack_entry(data, "image.boot")[0]
    except NgpuError as e:
        raise ValueError(f"neither a RAFS bootstrap nor a nydus blob stream: {e}") from e


def load_bootstrap(data: bytes) -> dict:
    """{"blob_ids", "chunks" (CHUNK_INFO_DTYPE), "flags", "chunk_size"} of a
    bootstrap or of the image.boot entry of a nydus blob stream."""
    boot = bootstrap_bytes(data)
    if rafs.detect_fs_version(boot) == "v6":
        return rafs.read_v6(boot)
    d = rafs_dump(boot)
    rows = {}
    for ino in d["inodes"]:
        for c in ino.get("chunks", []):
            rows.setdefault((c[0], c[1], c[8]), c)
    recs = np.zeros(len(rows), rafs.CHUNK_INFO_DTYPE)
    for i, c in enumerate(rows.values()):
        recs[i]["block_id"] = np.frombuffer(bytes.fromhex(c[0]), np.uint8)
        (recs[i]["blob_index"], recs[i]["flags"], recs[i]["compressed_offset"], recs[i]["compressed_size"],
         recs[i]["uncompressed_offset"], recs[i]["uncompressed_size"], recs[i]["file_offset"],
         recs[i]["index"]) = c[1:9]
    return {"blob_ids": [b["id"] for b in d["blobs"]], "chunks": recs, "flags": d["flags"],
            "chunk_size": d["chunk_size"]}


def tree(data: bytes) -> dict:
    """The inode tree (ngpu_rafs_dump) with blob indices replaced by blob ids."""
    d = rafs_dump(bootstrap_bytes(data))
    ids = [b["id"] for b in d["blobs"]]
    for ino in d["inodes"]:
        for c in ino.get("chunks", []):
            c[1] = ids[c[1]] if c[1] < len(ids) else f"#{c[1]}"
    return d


def tree_diff(a: dict, b: dict) -> list:
    """Paths missing on one side (-/+) or whose inode differs (~); inode
    numbers aside, as they depend on the tree's numbering, not the content."""
    def key(i):
        return {k: v for k, v in i.items() if k != "ino"}
    pa = {i["path"]: key(i) for i in a["inodes"]}
    pb = {i["path"]: key(i) for i in b["inodes"]}
    out = [("-", p) for p in sorted(pa.keys() - pb.keys())] + [("+", p) for p in sorted(pb.keys() - pa.keys())]
    out += [("~", p) for p in sorted(pa.keys() & pb.keys()) if pa[p] != pb[p]]
    return out


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
    ap.add_argument("--tree", action="store_true", help="the inode tree instead of the chunk set")
    args = ap.parse_args(argv)
    if args.tree:
        dumps = [tree(open(f, "rb").read()) for f in args.files]
    else:
        dumps = [canonical(load_bootstrap(open(f, "rb").read())) for f in args.files]
    if args.diff:
        if len(dumps) != 2:
            ap.error("--diff takes two files")
        d = tree_diff(*dumps) if args.tree else diff(*dumps)
        for sign, k in d:
            print(sign, *(k if isinstance(k, tuple) else (k,)))
        return 1 if d else 0
    for dmp in dumps:
        json.dump(dmp, sys.stdout, indent=1)
        print()
    return 0


if __name__ == "__main__":
    sys.exit(main())
