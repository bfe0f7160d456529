#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run in the BUILD container only (it needs ROCm LLVM's libclang-cpp.so, which
vendors the official BLAKE3 C implementation v1.8.2 as ``llvm_blake3_*``).
The outputs are plain JSON data; the GPU box never runs this script.

Independent implementations used here (none of them is oracle/ code):
  * BLAKE3  — ctypes -> /opt/rocm/lib/llvm/lib/libclang-cpp.so llvm_blake3_*
  * SHA-256 — Python hashlib (OpenSSL)
  * tar     — Python tarfile (independent of oracle/tar_ref.c)
  * dedup   — the small restatement ``dedup_py`` below (independent of
              oracle/dedup_ref.c), following SURVEY.md §8(a) a5/a6.

Fixtures:
  kat.json    — digests of input ``i % 251`` for many lengths x {blake3, sha256}
                plus the BLAKE3 spec vectors ("" and "abc").
  layers.json — per layer tar (tests/golden/layers.py) x chunk size x digester:
                chunk list, digests, dedup decisions; plus the TestPack scenario
                (tests/converter_test.go:459-528) with a chunk dict.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import sys
import tarfile
import io

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import layers  # noqa: E402

LIBS = ["/opt/rocm/lib/llvm/lib/libclang-cpp.so", "/usr/lib/x86_64-linux-gnu/libLLVM-15.so.1"]


class LLVMBlake3:
    def __init__(self):
        last = None
        for p in LIBS:
            try:
                self.lib = ctypes.CDLL(p)
                self.lib.llvm_blake3_hasher_init
                break
            except (OSError, AttributeError) as e:  # pragma: no cover
                last = e
        else:  # pragma: no cover
            raise RuntimeError(f"no llvm_blake3 available: {last}")
        self.lib.llvm_blake3_hasher_update.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        self.lib.llvm_blake3_hasher_finalize.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        self.lib.llvm_blake3_hasher_init.argtypes = [ctypes.c_void_p]
        self.state = ctypes.create_string_buffer(8192)

    def __call__(self, data: bytes) -> bytes:
        self.lib.llvm_blake3_hasher_init(self.state)
        self.lib.llvm_blake3_hasher_update(self.state, data, len(data))
        out = ctypes.create_string_buffer(32)
        self.lib.llvm_blake3_hasher_finalize(self.state, out, 32)
        return out.raw


def pattern(n: int) -> bytes:
    return bytes(i % 251 for i in range(n))


KAT_LENGTHS = [0, 1, 2, 3, 4, 5, 6, 7, 8, 55, 56, 63, 64, 65, 119, 127, 128, 129,
               1023, 1024, 1025, 2047, 2048, 2049, 3072, 3073, 4096, 4097, 5120,
               5121, 6144, 6145, 7168, 7169, 8192, 8193, 16383, 16384, 16385,
               31744, 65535, 65536, 65537, 102400, 131072 + 777, (1 << 20) - 1,
               1 << 20, (1 << 20) + 1, 3 * (1 << 20) + 5]

CHUNK_SIZES = {"oci_upper": [0x100000, 0x10000],
               "alpine_like": [0x100000, 0x10000],
               "chunk_dict": [0x100000, 0x1000],
               "oci_lower": [0x100000, 0x1000],
               "edge_pax": [0x100000, 0x10000, 0x1000],
               "edge_gnu": [0x10000]}


def chunks_py(tar_bytes: bytes, chunk_size: int):
    """tar -> [(offset, length, file_index, file_offset)] via Python tarfile."""
    out = []
    tf = tarfile.open(fileobj=io.BytesIO(tar_bytes), mode="r:")
    fi = 0
    for m in tf.getmembers():
        if m.isreg():
            for off in range(0, m.size, chunk_size):
                out.append((m.offset_data + off, min(chunk_size, m.size - off), fi, off))
            fi += 1
    return out


def dedup_py(digests, sizes, dict_entries=(), align=4096):
    """Independent restatement of SURVEY.md §8(a) a5/a6.

    dict_entries: [(digest, usize, inner_blob, index)] in chunk-table order.
    Returns (decisions, own_blob) with decision = (kind, index, ref, blob, uoff).
    """
    gd = {}
    for e, (d, sz, blob, idx) in enumerate(dict_entries):
        gd.setdefault(d, e)
    layered = {}
    real = {}
    nxt = 0
    own = None
    cur = 0
    new_count = 0
    out = []
    for i, (d, sz) in enumerate(zip(digests, sizes)):
        e = gd.get(d)
        if e is not None and dict_entries[e][1] in (0, sz):
            inner = dict_entries[e][2]
            if inner not in real:
                real[inner] = nxt
                nxt += 1
            out.append(("DICT", dict_entries[e][3], e, real[inner], 0))
            continue
        l = layered.get(d)
        if l is not None and sizes[l] in (0, sz):
            k, idx, _, blob, uoff = out[l]
            out.append(("INTRA", idx, l, blob, uoff))
            continue
        if own is None:
            own = nxt
            nxt += 1
        out.append(("NEW", new_count, i, own, cur))
        new_count += 1
        cur = (cur + sz + align - 1) // align * align
        layered.setdefault(d, i)
    return out, own


def main():
    b3 = LLVMBlake3()
    sha = lambda b: hashlib.sha256(b).digest()  # noqa: E731
    # spec sanity, before anything is written
    assert b3(b"").hex() == "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"
    assert b3(b"abc").hex() == "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"

    kat = {"source": {"blake3": "ROCm LLVM libclang-cpp.so llvm_blake3 (official BLAKE3 C v1.8.2)",
                      "sha256": "Python hashlib / OpenSSL"},
           "input": "byte i = i % 251", "vectors": []}
    for n in KAT_LENGTHS:
        p = pattern(n)
        kat["vectors"].append({"len": n, "blake3": b3(p).hex(), "sha256": sha(p).hex()})
    kat["spec"] = [{"input_hex": "", "blake3": b3(b"").hex()},
                   {"input_hex": b"abc".hex(), "blake3": b3(b"abc").hex()}]
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)

    doc = {"generator": "tests/golden/make_golden.py", "cases": []}
    tars = {k: fn() for k, fn in layers.LAYERS.items()}
    for name, tb in tars.items():
        for cs in CHUNK_SIZES[name]:
            ch = chunks_py(tb, cs)
            for dg, fn in (("blake3", b3), ("sha256", sha)):
                if dg == "sha256" and cs != 0x100000:
                    continue
                digs = [fn(tb[o:o + l]) for (o, l, _, _) in ch]
                dec, own = dedup_py(digs, [c[1] for c in ch])
                doc["cases"].append({
                    "layer": name, "chunk_size": cs, "digester": dg,
                    "tar_sha256": hashlib.sha256(tb).hexdigest(),
                    "chunks": ch, "digests": [d.hex() for d in digs],
                    "decisions": dec, "own_blob": own})

    # TestPack scenario (tests/converter_test.go:459-528): dict from the
    # chunk-dict layer (blob 0 of the dict), then lower & upper packed with it.
    cs = 0x100000
    dch = chunks_py(tars["chunk_dict"], cs)
    ddig = [b3(tars["chunk_dict"][o:o + l]) for (o, l, _, _) in dch]
    ddec, _ = dedup_py(ddig, [c[1] for c in dch])
    dict_entries = [(d, c[1], 0, dec[1]) for d, c, dec in zip(ddig, dch, ddec) if dec[0] == "NEW"]
    scen = {"dict": [[d.hex(), sz, blob, idx] for (d, sz, blob, idx) in dict_entries], "layers": {}}
    blobs_used = []
    for name in ("oci_lower", "oci_upper"):
        tb = tars[name]
        ch = chunks_py(tb, cs)
        digs = [b3(tb[o:o + l]) for (o, l, _, _) in ch]
        dec, own = dedup_py(digs, [c[1] for c in ch], dict_entries)
        scen["layers"][name] = {"chunks": ch, "digests": [d.hex() for d in digs],
                                "decisions": dec, "own_blob": own}
        # Merge bookkeeping: a layer references dict blobs it hit and at most one own blob.
        for k in dec:
            tag = "dict" if k[0] == "DICT" else name
            if tag not in blobs_used:
                blobs_used.append(tag)
    scen["expected_blobs"] = blobs_used  # converter_test.go:517-519: [dict, upper]
    assert blobs_used == ["dict", "oci_upper"], blobs_used
    doc["testpack"] = scen
    with open(os.path.join(HERE, "layers.json"), "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    print("wrote kat.json, layers.json:", len(doc["cases"]), "cases")


if __name__ == "__main__":
    main()
