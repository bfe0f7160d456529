"""GPU soak: many random layer tars through ngpu_pack_tar and the streaming
Pack, every digest and decision checked against the CPU oracle (test
infrastructure: the oracle is the checker).  Random file-size mixes (empty,
a few bytes, around the 64-B block / 1 KiB leaf / chunk edges, multi-chunk),
chunk sizes 4 KiB .. 4 MiB, both digesters, every BLAKE3 lanes setting and
the grid-stage flag, engines reused across cases (as a converter's cached
engine is).  A failure names the case, the engine and the first bad chunk;
the digest guard turns an unwritten digest into NGPU_EDEVICE.

usage: python scripts/gpu_soak.py [cases] [seed]
       python scripts/gpu_soak.py --threads T [cases] [seed]
  --threads: T host threads share four cached engines and convert at once --
  pack_tar (engine stream), streaming Packs (per-Pack streams), device calls on
  each thread's own stream, Packs against a chunk dict -- every result checked
  (the workspace slots, Pack pools and lazy stage-end events under load).
"""
import threading
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "nydus-snapshotter_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: F401,E402  (one HIP runtime per process: torch's, loaded first)
import numpy as np  # noqa: E402

import layers  # noqa: E402
import nydus_gpu  # noqa: E402
import oracle_py as oracle  # noqa: E402

EDGES = [0, 1, 12, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 4095, 4096, 4097, 65535, 65536,
         65537, 1 << 20, (1 << 20) + 1]


def random_tar(rng, chunk, files=None, first=()):
    """A random layer tar; `files` (a list) collects (name, bytes) of its
    regular files; `first`: files written before the random ones."""
    t = layers._TarBuilder()
    t.dir("d")
    for name, data in first:
        t.file(name, data)
    n = int(rng.integers(1, 60))
    total = 0
    for i in range(n):
        r = rng.random()
        if r < 0.35:
            size = int(rng.choice(EDGES))
        elif r < 0.55:
            size = int(chunk * rng.integers(1, 4) + rng.integers(-2, 3))
        elif r < 0.9:
            size = int(rng.integers(0, 200_000))
        else:
            size = int(rng.integers(0, 6 << 20))
        size = max(0, min(size, (24 << 20) - total))
        total += size
        data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        if i and rng.random() < 0.1:  # a whole-file duplicate (INTRA)
            t.file(f"d/dup{i}", data)
        t.file(f"d/f{i}", data)
        if files is not None:
            files.append((f"base/f{i}", data))
        if rng.random() < 0.05:
            t.symlink(f"d/l{i}", f"f{i}")
    return t.bytes()


def check(tag, ch, out, tar, chunk, digester, recs=None):
    ech = oracle.tar_chunks(tar, chunk)
    if ch.tobytes() != ech.tobytes():
        raise AssertionError(f"{tag}: chunk table differs ({len(ch)} vs {len(ech)})")
    dig = oracle.digest_chunks(tar, ech, digester)
    kw = {}
    if recs is not None:
        kw = dict(dict_digests=recs["block_id"], dict_sizes=recs["uncompressed_size"],
                  dict_blob=recs["blob_index"], dict_index=recs["index"],
                  dict_uoff=recs["uncompressed_offset"])
    dec, _ = oracle.dedup(dig, ech["length"], **kw)
    bad = np.nonzero((out["digest"] != dig).any(axis=1))[0]
    if len(bad):
        i = int(bad[0])
        raise AssertionError(f"{tag}: {len(bad)} digest(s) differ, first chunk {i} "
                             f"(len {int(ech['length'][i])}, kind {int(out['kind'][i])}, "
                             f"got {out['digest'][i].tobytes().hex()})")
    for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
        if not np.array_equal(out[f], dec[f]):
            raise AssertionError(f"{tag}: decision field {f} differs")


def concurrent(threads, cases, seed):
    """T threads, shared engines, every call checked (see the module doc)."""
    import torch
    from nydus_gpu import rafs
    rng0 = np.random.default_rng(seed)
    configs = [(0x10000, "blake3", 0), (0x100000, "blake3", 0), (0x100000, "blake3", 8),
               (0x10000, "sha256", 0)]
    shared = []
    for chunk, dg, lanes in configs:
        eng = nydus_gpu.Engine(digester=dg, chunk_size=chunk, leaves_per_lane=lanes)
        base = []  # the dict: a layer's own records; its files are planted in later layers
        ch, out, _ = eng.pack_tar(random_tar(rng0, chunk, files=base))
        recs = nydus_gpu.chunk_table(ch, out).view(rafs.CHUNK_INFO_DTYPE).reshape(-1).copy()
        d = eng.dict_create(recs)
        shared.append((eng, chunk, dg, lanes, base, recs, d))
    # a one-process node of 4 parts on device 0 with a digest-prefix partitioned
    # dict: concurrent requesters exchange through their own (owner, requester)
    # channels (ngpu_node_*, node.hip)
    node = nydus_gpu.Node([0, 0, 0, 0], chunk_size=0x10000)
    nbase = []
    nch, nout, _ = node.engines[0].pack_tar(random_tar(rng0, 0x10000, files=nbase))
    nrecs = nydus_gpu.chunk_table(nch, nout).view(rafs.CHUNK_INFO_DTYPE).reshape(-1).copy()
    nd = node.dict_create(nrecs)
    counts = {"calls": 0, "chunks": 0, "node_calls": 0}
    mu = threading.Lock()
    errors = []

    def worker(tid):
        rng = np.random.default_rng(seed * 1000 + tid)
        stream = torch.cuda.Stream()
        try:
            for case in range(cases):
                eng, chunk, dg, lanes, base, recs, d = shared[int(rng.integers(0, len(shared)))]
                plant = base if rng.random() < 0.3 else ()  # the dict layer's files: DICT hits
                tar = random_tar(rng, chunk, first=plant)
                op = int(rng.integers(0, 6))
                tag = f"thread {tid} case {case} op {op} (chunk {chunk:#x}, {dg}, lanes {lanes})"
                if op == 4:  # node Pack against the partitioned dict
                    plant = nbase if rng.random() < 0.5 else ()
                    tar = random_tar(rng, 0x10000, first=plant)
                    w = node.pack(dict=nd)
                    w.write(tar)
                    ch, out, _ = w.close()
                    check(tag + " node", ch, out, tar, 0x10000, "blake3", nrecs)
                    with mu:
                        counts["node_calls"] += 1
                elif op == 5:  # early emission (ngpu_pack_set_output, the mirrors' Pack)
                    import hashlib
                    import io
                    sink = io.BytesIO()
                    use = d if rng.random() < 0.5 else None
                    w = eng.pack(dict=use, retain=True)
                    w.set_output(sink, compressor=str(rng.choice(["none", "zstd"])))
                    pos = 0
                    while pos < len(tar):
                        k = int(rng.integers(1, 3 << 20))
                        w.write(tar[pos:pos + k])
                        pos += k
                    ch, out, _, info = w.finish(None)
                    check(tag + " early", ch, out, tar, chunk, dg, recs if use is not None else None)
                    if hashlib.sha256(sink.getvalue()).hexdigest() != info["stream_digest"]:
                        raise AssertionError(f"{tag}: early stream digest differs from its bytes")
                elif op == 0:
                    ch, out, _ = eng.pack_tar(tar)
                    check(tag, ch, out, tar, chunk, dg)
                elif op in (1, 2):
                    use = d if op == 2 else None
                    w = eng.pack(dict=use)
                    pos = 0
                    while pos < len(tar):
                        k = int(rng.integers(1, 3 << 20))
                        w.write(tar[pos:pos + k])
                        pos += k
                    ch, out, _ = w.close()
                    check(tag, ch, out, tar, chunk, dg, recs if op == 2 else None)
                else:
                    ch = nydus_gpu.tar_chunks(tar, chunk)
                    n = len(ch)
                    with torch.cuda.stream(stream):
                        dbuf = torch.frombuffer(bytearray(tar), dtype=torch.uint8).to("cuda", non_blocking=False)
                        dch = torch.from_numpy(ch.view(np.uint8).copy()).to("cuda")
                        dout = torch.empty(max(n, 1) * 64, dtype=torch.uint8, device="cuda")
                        eng.process_dict_device(None, dbuf.data_ptr(), dbuf.numel(), dch.data_ptr(), n,
                                                dout.data_ptr(), stream=stream.cuda_stream)
                        host = dout.cpu()
                    stream.synchronize()
                    st = eng.device_status()
                    if st:
                        raise AssertionError(f"{tag}: device status {st}")
                    out = host.numpy()[: n * 64].view(nydus_gpu.RESULT_DTYPE)
                    check(tag, ch, out, tar, chunk, dg)
                with mu:
                    counts["calls"] += 1
                    counts["chunks"] += len(ch)
        except Exception as ex:  # reported by main
            errors.append(f"{type(ex).__name__}: {ex}")

    t0 = time.time()
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for eng, *_rest, d in shared:
        d.release()
        eng.close()
    nd.release()
    node.close()
    if errors:
        print(json.dumps({"soak": "FAILED", "errors": errors[:5]}), flush=True)
        sys.exit(1)
    print(json.dumps({"soak": "ok", "threads": threads, "cases_per_thread": cases, **counts,
                      "engines": len(shared), "seconds": round(time.time() - t0, 1)}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--threads":
        threads = int(sys.argv[2])
        rest = sys.argv[3:]
        return concurrent(threads, int(rest[0]) if rest else 50, int(rest[1]) if len(rest) > 1 else 0x50A5)
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0x50A4
    rng = np.random.default_rng(seed)
    engines = {}
    t0 = time.time()
    stats = {"cases": 0, "calls": 0, "chunks": 0, "bytes": 0}
    for case in range(cases):
        chunk = int(rng.choice([0x1000, 0x4000, 0x10000, 0x100000, 0x400000]))
        digester = "sha256" if rng.random() < 0.25 else "blake3"
        lanes = 0 if digester == "sha256" else int(rng.choice([0, 1, 2, 4, 8, 16]))
        flags = nydus_gpu.FLAG_GRID_STAGES if rng.random() < 0.2 else 0
        key = (chunk, digester, lanes, flags)
        if key not in engines:
            engines[key] = nydus_gpu.Engine(digester=digester, chunk_size=chunk,
                                            leaves_per_lane=lanes, flags=flags,
                                            staging_bytes=int(rng.choice([0, 4 * chunk])))
        eng = engines[key]
        tar = random_tar(rng, chunk)
        tag = f"case {case} (chunk {chunk:#x}, {digester}, lanes {lanes}, flags {flags:#x}, {len(tar)} B)"
        ch, out, st = eng.pack_tar(tar)
        check(tag + " pack_tar", ch, out, tar, chunk, digester)
        w = eng.pack()
        pos = 0
        while pos < len(tar):
            k = int(rng.integers(1, 3 << 20))
            w.write(tar[pos:pos + k])
            pos += k
        ch2, out2, st2 = w.close()
        check(tag + " stream", ch2, out2, tar, chunk, digester)
        stats["cases"] += 1
        stats["calls"] += 2
        stats["chunks"] += 2 * len(ch)
        stats["bytes"] += 2 * len(tar)
        if case % 20 == 0:
            print(f"case {case}: ok ({time.time() - t0:.0f} s)", flush=True)
    for e in engines.values():
        e.close()
    stats["engines"] = len(engines)
    stats["seconds"] = round(time.time() - t0, 1)
    print(json.dumps({"soak": "ok", **stats}), flush=True)


if __name__ == "__main__":
    main()
