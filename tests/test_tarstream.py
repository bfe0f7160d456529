"""The incremental tar scanner (csrc/tarstream.hpp) fed in random splits
(1..9000-byte pieces) gives the same chunks as the oracle and each chunk
receives exactly its own bytes.  Built with g++ on the host (no GPU)."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def scanner_bin(tmp_path_factory):
    d = tmp_path_factory.mktemp("tarstream")
    exe = str(d / "tarstream_split")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "nydus-snapshotter_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "tarstream_split.cpp"), "-o", exe])
    return exe


def _fnv(b):
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.mark.parametrize("layer,cs", [("edge_pax", 0x10000), ("edge_gnu", 0x10000), ("edge_pax", 0x1000),
                                      ("alpine_like", 0x100000), ("oci_lower", 0x1000)])
def test_split_feed_matches_oracle(scanner_bin, tars, oracle, layer, cs):
    tb = tars[layer]
    ref = oracle.tar_chunks(tb, cs)
    with tempfile.NamedTemporaryFile(suffix=".tar") as f:
        f.write(tb)
        f.flush()
        for seed in (1, 2, 3):
            out = subprocess.check_output([scanner_bin, f.name, str(cs), str(seed)], text=True).splitlines()
            assert out[-1] == f"FILES {ref.size and int(ref['file_index'].max()) + 1 or 0} BAD 0" or \
                out[-1].endswith("BAD 0")
            rows = [list(map(int, line.split(","))) for line in out[:-1]]
            assert len(rows) == len(ref)
            for r, c in zip(rows, ref):
                assert r[:4] == [int(c["offset"]), int(c["length"]), int(c["file_index"]), int(c["file_offset"])]
                o, ln = int(c["offset"]), int(c["length"])
                if ln <= 65536:
                    assert r[4] == _fnv(tb[o:o + ln])


def test_truncated_stream_is_error(scanner_bin, tars):
    tb = tars["oci_upper"][: len(tars["oci_upper"]) // 2]
    with tempfile.NamedTemporaryFile(suffix=".tar") as f:
        f.write(tb)
        f.flush()
        out = subprocess.check_output([scanner_bin, f.name, str(0x100000), "5"], text=True)
    assert "ERR -4" in out


def test_scanner_under_asan_ubsan(tmp_path, tars, oracle):
    """Host code under AddressSanitizer + UBSan (GPU sanitizers are not
    available; the scanner is pure host C++)."""
    exe = str(tmp_path / "tarstream_asan")
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "nydus-snapshotter_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "tarstream_split.cpp"), "-o", exe])
    for layer in ("edge_pax", "edge_gnu", "oci_upper"):
        p = tmp_path / f"{layer}.tar"
        p.write_bytes(tars[layer])
        out = subprocess.check_output([exe, str(p), str(0x10000), "7"], text=True,
                                      env={**os.environ, "ASAN_OPTIONS": "detect_leaks=1"})
        assert out.strip().endswith("BAD 0")
    # truncated and garbage inputs must fail cleanly, not crash
    for bad in (tars["oci_upper"][:1500], b"\x00" * 10 + b"garbage" * 100):
        p = tmp_path / "bad.tar"
        p.write_bytes(bad)
        subprocess.check_output([exe, str(p), str(0x1000), "3"], text=True)
