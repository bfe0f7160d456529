"""The gzip checkpoint index behind PackOption.OCIRef (csrc/zran.cpp), on the
CPU under ASan + UBSan (tests/cpp/zran_test.cpp): inflating through the
indexer equals zlib's output, and random ranges read back through the
checkpoints (zran_extract: inflatePrime + dictionary + raw inflate) equal the
stream -- for text, random and mixed data, gzip levels 1 / 6 / 9."""
import gzip
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def zran_exe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("zran") / "zran_test")
    csrc = os.path.join(ROOT, "nydus-snapshotter_amd", "csrc")
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "include"),
                           "-I", csrc, os.path.join(ROOT, "tests", "cpp", "zran_test.cpp"),
                           os.path.join(csrc, "zran.cpp"), os.path.join(csrc, "blob.cpp"),
                           os.path.join(csrc, "rafs.cpp"), "-o", exe, "-lz", "-lcrypto", "-ldl",
                           "-lpthread"])
    return exe


@pytest.mark.parametrize("kind", ["text", "random", "mixed"])
@pytest.mark.parametrize("level", [1, 6, 9])
def test_zran_index_and_random_reads(zran_exe, tmp_path, kind, level):
    rng = np.random.default_rng(level * 10 + len(kind))
    if kind == "text":
        words = np.array([b"chunk ", b"dict ", b"nydus ", b"layer\n", b"rafs ", b"blob "], dtype=object)
        data = b"".join(words[rng.integers(0, len(words), 1_500_000)])
    elif kind == "random":
        data = rng.integers(0, 256, 6 << 20, dtype=np.uint8).tobytes()
    else:
        parts = []
        for i in range(40):
            if i % 2:
                parts.append(rng.integers(0, 256, int(rng.integers(1, 300_000)), dtype=np.uint8).tobytes())
            else:
                parts.append(bytes(int(rng.integers(1, 200_000))) + b"x" * int(rng.integers(1, 50_000)))
        data = b"".join(parts)
    f = tmp_path / "l.gz"
    f.write_bytes(gzip.compress(data, compresslevel=level, mtime=0))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([zran_exe, str(f), str(1 << 20), str(level)], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, (r.stdout, r.stderr[-2000:])
    assert r.stdout.strip().endswith("ok")
    pts = int(r.stdout.split()[0].split("=")[1])
    assert pts >= max(1, len(data) // (2 << 20))
