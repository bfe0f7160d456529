"""Deterministic layer-tar builders shared by make_golden.py and the tests.

These restate the reference's test fixtures with a *seeded* payload so the
expected chunk digests can be committed:

* ``chunk_dict_tar``  — buildChunkDictTar   (tests/converter_test.go:177-194)
* ``oci_lower_tar``   — buildOCILowerTar    (tests/converter_test.go:196-223)
* ``oci_upper_tar``   — buildOCIUpperTar    (tests/converter_test.go:225-274)
* ``huge_string``     — hugeString          (tests/converter_test.go:91-111):
  alternating 512 KiB random / 512 KiB zero segments; the reference draws the
  random half from crypto/rand, here it is SHA-256 counter mode keyed by a seed.

plus edge-case tars for the chunker (PAX/GNU long names, hardlinks, symlinks,
zero-size files, whiteouts, exact chunk-size multiples, repeated content).

Only the Python standard library is used, so the same bytes are produced
here and on the GPU box.
"""
from __future__ import annotations

import hashlib
import io
import tarfile

MiB = 1 << 20


def prng_bytes(seed: int, n: int) -> bytes:
    """SHA-256 counter-mode byte stream (deterministic, seedable)."""
    out = bytearray()
    s = seed.to_bytes(8, "little")
    i = 0
    while len(out) < n:
        out += hashlib.sha256(s + i.to_bytes(8, "little")).digest()
        i += 1
    return bytes(out[:n])


def huge_string(mb: int, seed: int = 0x6875676553) -> bytes:
    seq = 512 * 1024
    parts = []
    for i in range((mb * MiB) // seq):
        parts.append(prng_bytes(seed + i, seq) if i % 2 == 0 else bytes(seq))
    return b"".join(parts)


class _TarBuilder:
    def __init__(self, fmt=tarfile.PAX_FORMAT):
        self.buf = io.BytesIO()
        self.tf = tarfile.open(fileobj=self.buf, mode="w", format=fmt)

    def _info(self, name, **kw):
        ti = tarfile.TarInfo(name)
        ti.mtime = 0
        ti.uid = ti.gid = 1000
        ti.uname = ti.gname = "nydus"
        ti.mode = kw.pop("mode", 0o444)
        for k, v in kw.items():
            setattr(ti, k, v)
        return ti

    def file(self, name, data: bytes):
        ti = self._info(name, size=len(data))
        self.tf.addfile(ti, io.BytesIO(data))

    def dir(self, name):
        self.tf.addfile(self._info(name, type=tarfile.DIRTYPE, mode=0o755))

    def symlink(self, name, target):
        self.tf.addfile(self._info(name, type=tarfile.SYMTYPE, linkname=target))

    def hardlink(self, name, target):
        self.tf.addfile(self._info(name, type=tarfile.LNKTYPE, linkname=target))

    def fifo(self, name):
        self.tf.addfile(self._info(name, type=tarfile.FIFOTYPE))

    def bytes(self) -> bytes:
        self.tf.close()
        return self.buf.getvalue()


def chunk_dict_tar(n: int = 100) -> bytes:
    t = _TarBuilder()
    t.dir("dir-1")
    for i in range(1, n):
        t.file(f"dir-1/file-{i}", f"lower-file-{i}".encode())
    return t.bytes()


def oci_lower_tar(n: int = 100) -> bytes:
    t = _TarBuilder()
    t.dir("dir-1")
    for i in range(1, n):
        t.file(f"dir-1/file-{i}", f"lower-file-{i}".encode())
    t.dir("dir-2")
    t.file("dir-2/file-1", b"lower-file-1")
    return t.bytes()


def oci_upper_tar(mb: int = 3) -> bytes:
    t = _TarBuilder()
    t.dir("dir-1")
    t.file("dir-1/.wh.file-1", b"")
    t.dir("dir-2")
    t.file("dir-2/.wh..wh..opq", b"")
    t.file("dir-2/file-1", huge_string(mb))
    t.file("dir-2/file-2", b"upper-file-2")
    t.file("dir-2/file-3", b"upper-file-3")
    return t.bytes()


# ---- Go archive/tar's encoding (the reference tests write their tars with it) ----
# tar.Writer.WriteHeader of a Header that fits USTAR (writeUSTARHeader /
# templateV7Plus / setFormat in Go's archive/tar): numbers as zero-padded octal
# with a NUL (width - 1 digits), a zero ModTime written as 0, magic "ustar\0" +
# "00", the checksum as 6 octal digits + NUL + space; directories keep the name
# they were given (no "/" appended, unlike Python's tarfile); Close() ends the
# archive with two zero blocks and no record padding.
def _go_octal(n: int, width: int) -> bytes:
    s = format(n, "o")
    return ("0" * max(0, width - 1 - len(s)) + s).encode() + b"\0"


def go_header(name: str, mode: int, size: int, typeflag: bytes, uid: int = 0, gid: int = 0,
              uname: str = "root", gname: str = "root", mtime: int = 0, linkname: str = "") -> bytes:
    h = bytearray(512)
    nb = name.encode()
    assert len(nb) <= 100
    h[0:len(nb)] = nb
    h[100:108] = _go_octal(mode, 8)
    h[108:116] = _go_octal(uid, 8)
    h[116:124] = _go_octal(gid, 8)
    h[124:136] = _go_octal(size, 12)
    h[136:148] = _go_octal(mtime, 12)
    h[156:157] = typeflag
    lb = linkname.encode()
    h[157:157 + len(lb)] = lb
    h[257:265] = b"ustar\x0000"
    h[265:265 + len(uname)] = uname.encode()
    h[297:297 + len(gname)] = gname.encode()
    h[329:337] = _go_octal(0, 8)
    h[337:345] = _go_octal(0, 8)
    h[148:156] = b" " * 8
    h[148:155] = _go_octal(sum(h), 7)
    h[155] = ord(" ")
    return bytes(h)


class GoTar:
    """The reference tests' writeFileToTar / writeDirToTar (tests/converter_test.go:
    129-167): mode 0444, the current user's uid / gid / names (root here)."""

    def __init__(self, uid: int = 0, gid: int = 0, uname: str = "root", gname: str = "root"):
        self.out = bytearray()
        self.ids = dict(uid=uid, gid=gid, uname=uname, gname=gname)

    def file(self, name: str, data: bytes):
        self.out += go_header(name, 0o444, len(data), b"0", **self.ids)
        self.out += data + bytes((-len(data)) % 512)

    def dir(self, name: str):
        self.out += go_header(name, 0o444, 0, b"5", **self.ids)

    def bytes(self) -> bytes:
        return bytes(self.out) + bytes(1024)


def oci_upper_tar_go(mb: int = 3) -> bytes:
    """buildOCIUpperTar (tests/converter_test.go:225-274) in Go's encoding,
    as TestUnpack (:607-635) packs it and compares the Unpack output's sha256
    with it."""
    t = GoTar()
    t.dir("dir-1")
    t.file("dir-1/.wh.file-1", b"")
    t.dir("dir-2")
    t.file("dir-2/.wh..wh..opq", b"")
    t.file("dir-2/file-1", huge_string(mb))
    t.file("dir-2/file-2", b"upper-file-2")
    t.file("dir-2/file-3", b"upper-file-3")
    return t.bytes()


def edge_tar(fmt=tarfile.PAX_FORMAT, chunk: int = 64 * 1024) -> bytes:
    """Chunker edge cases around a given chunk size."""
    t = _TarBuilder(fmt)
    t.dir("etc")
    t.file("etc/empty", b"")
    t.file("etc/one", b"x")
    t.file("a" * 150 + "/long-name-file", prng_bytes(1, 3000))  # long name
    t.file("exact", prng_bytes(2, chunk))
    t.file("exact-plus-1", prng_bytes(3, chunk + 1))
    t.file("two-minus-1", prng_bytes(4, 2 * chunk - 1))
    t.symlink("etc/link", "/etc/one")
    t.hardlink("etc/hard", "exact")
    t.fifo("etc/fifo")
    t.file("zeros", bytes(3 * chunk + 100))  # repeated all-zero chunks
    t.file("dup-of-exact", prng_bytes(2, chunk))  # whole-file duplicate
    t.file("odd-1023", prng_bytes(5, 1023))
    t.file("odd-1025", prng_bytes(6, 1025))
    t.file("odd-4097", prng_bytes(7, 4097))
    return t.bytes()


def alpine_like_tar(seed: int = 0xA1F1E) -> bytes:
    """C1 stand-in: ~8 MiB, a few hundred entries, mostly
    symlinks + small files + one ~1 MiB busybox-like binary."""
    import random

    rng = random.Random(seed)
    t = _TarBuilder()
    for d in ("bin", "etc", "lib", "usr", "usr/bin", "usr/lib", "var", "sbin"):
        t.dir(d)
    t.file("bin/busybox", prng_bytes(seed, 1_000_000 + 123))
    for i in range(220):
        t.symlink(f"bin/applet{i}", "/bin/busybox")
    for i in range(90):
        n = rng.choice([0, 17, 300, 1500, 4096, 9000, 40000, 70000])
        t.file(f"etc/conf{i}", prng_bytes(seed * 31 + i, n))
    libs = []
    for i in range(24):
        n = rng.randint(50_000, 600_000)
        libs.append(prng_bytes(seed * 77 + i, n))
        t.file(f"lib/lib{i}.so", libs[-1])
    t.file("usr/lib/libdup.so", libs[3])  # whole-file duplicates -> INTRA
    t.file("usr/lib/libcopy.so", libs[5])
    return t.bytes()


LAYERS = {
    "chunk_dict": chunk_dict_tar,
    "oci_lower": oci_lower_tar,
    "oci_upper": oci_upper_tar,
    "edge_pax": lambda: edge_tar(tarfile.PAX_FORMAT),
    "edge_gnu": lambda: edge_tar(tarfile.GNU_FORMAT),
    "alpine_like": alpine_like_tar,
}
