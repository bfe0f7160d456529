#!/usr/bin/env python3
"""bench.py — GB/s of layer data chunk-hashed + deduped on MI355X.

Workload (BASELINE.json configs[1]): one synthetic 16 GiB
layer tar = 4096 regular files x 4 MiB of random bytes (real ustar/PAX
headers in between), PackOption.ChunkSize 1 MiB, blake3, no chunk dict.
The layer is resident in HBM before timing; one "step" = one pass of the hot
path over the layer through the C ABI (ngpu_process_device: BLAKE3 digests of
all 16384 chunks + intra-layer dedup decisions + stats readback) plus the D2H
copy of the 1 MiB result table.

Multi-GPU (torchrun, one process per GPU): every rank converts its own layer
(weak scaling, layers are independent — SURVEY.md §8(e)); no collective is in
the data path.  value = bytes of file data all ranks digested / max-over-ranks
time.

The JSON line also carries:
  roofline     — the dominant kernel (b3_groups) against the integer-VALU
                 peak: algorithmic ops (680 per BLAKE3 compression) per launch
                 / its HIP-event duration;
  cpu_baseline — the CPU digest+dedup stage (oracle/cpu_baseline.c: official
                 BLAKE3 C with AVX-512 dispatch, pthreads, stream-order dedup)
                 on a bounded sample of the same layer, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tarfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nydus-snapshotter_amd"))

MiB = 1 << 20
# gfx950 integer VALU peak: 256 CU x 4 SIMD x 16 lane-ops/clk x 2.4 GHz =
# 39.3 T int32 ops/s.  Measured, not assumed: a wave64 v_add3/v_xor/v_alignbit
# takes 4 SIMD cycles (rocprofv3: SQ_INSTS_VALU x 4 / 1024 SIMDs = the whole
# b3_groups duration at the GRBM clock; DESIGN.md §Roofline, profiles/).
SHA_MODES = {"auto": 0, "split": 1, "pair": 2, "lane": 3}
SHA_PAIR_MAX_CHUNKS = 256 * 128  # launch_sha256's auto rule (sha256.hip)
CLOCK_HZ = 2.4e9
PEAK_INT_OPS = 256 * 4 * 16 * 2.4e9
PEAK_HBM = 8.0e12
OPS_PER_COMPRESSION = 680  # 7 rounds x 8 G x 12 ops + 8 output xors
QUAD_COMPRESS_DEP_OPS = 190  # compress_quad: VALU ops per lane, one dependent chain
DEP_OP_CYCLES = 8.5          # a lone wave's dependent VALU op (tools/valu_exec.hip, profiles/r1/valu_exec_issue.jsonl)
KERNEL_BOUNDARY_S = 4.65e-6  # an empty kernel in a small call's trace (profiles/r2/c1_trace_diag_r2dg.txt)


def synthetic_layout(n_files: int, file_size: int, chunk_size: int):
    """Tar layout of the synthetic layer: header bytes per file, data offsets,
    and the chunk descriptors ngpu_tar_chunks would produce for it (checked by
    tests/test_bench.py against the real parser on a small instance)."""
    import nydus_gpu
    headers = np.zeros((n_files, 512), np.uint8)
    for i in range(n_files):
        ti = tarfile.TarInfo(f"usr/lib/file-{i:05d}.bin")
        ti.size = file_size
        ti.mtime = 0
        ti.uid = ti.gid = 0
        ti.uname = ti.gname = "root"
        ti.mode = 0o644
        hb = ti.tobuf(format=tarfile.GNU_FORMAT)
        assert len(hb) == 512
        headers[i] = np.frombuffer(hb, np.uint8)
    stride = 512 + (file_size + 511) // 512 * 512
    total = n_files * stride + 1024
    per_file = (file_size + chunk_size - 1) // chunk_size
    ch = np.zeros(n_files * per_file, nydus_gpu.CHUNK_DTYPE)
    k = np.arange(per_file, dtype=np.uint64)
    for i in range(n_files):
        s = slice(i * per_file, (i + 1) * per_file)
        ch["offset"][s] = i * stride + 512 + k * chunk_size
        ch["length"][s] = np.minimum(chunk_size, file_size - k * chunk_size)
        ch["file_index"][s] = i
        ch["file_offset"][s] = k * chunk_size
    return headers, stride, total, ch


def build_layer_on_gpu(torch, n_files, file_size, chunk_size, seed, dup_every=0):
    headers, stride, total, ch = synthetic_layout(n_files, file_size, chunk_size)
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(seed)
    step = 1 << 30
    for s in range(0, total, step):
        buf[s:min(total, s + step)].random_(0, 256, generator=g)
    body = buf[: n_files * stride].view(n_files, stride)
    body[:, :512].copy_(torch.from_numpy(headers).cuda())
    buf[n_files * stride:].zero_()
    if dup_every:  # plant duplicate files (whole-file copies)
        for i in range(dup_every, n_files, dup_every):
            body[i, 512:].copy_(body[i - 1, 512:])
    torch.cuda.synchronize()
    return buf, ch


_B3 = None


def ref_digest(data: bytes, digester: str) -> bytes:
    """An independent host digest for the post-run spot checks: OpenSSL SHA-256
    (hashlib) or the official BLAKE3 C that ROCm's LLVM vendors
    (llvm_blake3_* in libclang-cpp.so, ctypes) -- not the repo's oracle."""
    global _B3
    if digester == "sha256":
        import hashlib
        return hashlib.sha256(data).digest()
    if _B3 is None:
        import ctypes
        for path in ("/opt/rocm/lib/llvm/lib/libclang-cpp.so",
                     "/usr/lib/x86_64-linux-gnu/libLLVM-15.so.1"):
            try:
                lib = ctypes.CDLL(path)
                lib.llvm_blake3_hasher_init.argtypes = [ctypes.c_void_p]
                break
            except (OSError, AttributeError):
                lib = None
        if lib is None:
            raise RuntimeError("no llvm_blake3_* library for the BLAKE3 spot check")
        lib.llvm_blake3_hasher_update.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        lib.llvm_blake3_hasher_finalize.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        _B3 = (lib, ctypes.create_string_buffer(8192), ctypes)
    lib, st, ct = _B3
    lib.llvm_blake3_hasher_init(st)
    lib.llvm_blake3_hasher_update(st, data, len(data))
    out = ct.create_string_buffer(32)
    lib.llvm_blake3_hasher_finalize(st, out, 32)
    return out.raw


def high_offset_sample(ch: np.ndarray, k: int = 4, seed: int = 5) -> np.ndarray:
    """Chunk ids past 2^32 worth checking: every chunk that crosses a 4 GiB
    boundary, the last chunk, and k random chunks above 4 GiB."""
    off = ch["offset"].astype(np.uint64)
    end = off + ch["length"].astype(np.uint64) - np.uint64(1)
    cross = np.nonzero((off >> np.uint64(32)) != (end >> np.uint64(32)))[0]
    above = np.nonzero(off >= np.uint64(1 << 32))[0]
    rng = np.random.default_rng(seed)
    pick = rng.choice(above, min(k, len(above)), replace=False) if len(above) else above
    return np.unique(np.concatenate([cross, pick, [len(ch) - 1]]).astype(np.int64))


def check_high_digests(buf, ch, res, digester) -> dict:
    """Post-run check: C2/C3 layers reach offset 2^34, so
    verify the digests of high_offset_sample against ref_digest."""
    ids = high_offset_sample(ch)
    bad = []
    for i in ids:
        o, ln = int(ch["offset"][i]), int(ch["length"][i])
        want = ref_digest(buf[o:o + ln].cpu().numpy().tobytes(), digester)
        if res["digest"][i].tobytes() != want:
            bad.append(int(i))
    assert not bad, f"digest mismatch past 4 GiB at chunks {bad}"
    return {"chunks": len(ids), "max_offset": int(ch["offset"][ids].max()),
            "crossing_4gib": int(((ch["offset"][ids] >> 32) !=
                                  ((ch["offset"][ids] + ch["length"][ids] - 1) >> 32)).sum()),
            "ok": True}


def host_cpus():
    """CPUs this process may run on (sched affinity = what `nproc` prints) and
    the cgroup CPU quota in cores, if one is set."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return aff, quota


def cpu_baseline(host_sample: np.ndarray, ch: np.ndarray, digester: str, threads: int,
                 what: str = ""):
    """The CPU digest+dedup stage on all host cores and single-stream, each
    repeated for ~3 s (bounded sample)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    chs = ch.view(oracle_py.CHUNK_DTYPE)
    nbytes = int(chs["length"].sum())
    oracle_py.cpu_digest_dedup(host_sample, chs[:16], digester, 1)  # load libs

    def timed(t):
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle_py.cpu_digest_dedup(host_sample, chs, digester, t)
            reps += 1
            if time.perf_counter() - t0 > 3.0 or reps >= 200:
                return (time.perf_counter() - t0) / reps, reps
    t_single, r1 = timed(1)
    t_multi, reps = timed(threads)
    aff, quota = host_cpus()
    return {"value": round(nbytes / t_multi / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "sample": f"{what or 'first'} {nbytes / MiB:.1f} MiB of file data of the same layer "
                      f"({len(chs)} chunks), digest+dedup, {oracle_py.cpu_impl()}; "
                      f"{reps} reps on {threads} threads ({aff} CPUs in the process affinity, "
                      f"cgroup quota {quota} cores), {r1} single-stream",
            "single_stream_gbs": round(nbytes / t_single / 1e9, 3),
            "affinity_cpus": aff, "cgroup_cpu_quota": quota}


WORKLOADS = {
    "c1": dict(desc="C1: alpine-like OCI layer tar (~8 MiB: one ~1 MiB busybox-like binary, 24 "
                    "libraries, 90 small files, 220 symlinks; seed 0xA1F1E), RAFS v6, 1 MiB "
                    "chunks, blake3, no chunk dict -- the reference's CPU-runnable case",
               tar="alpine_like", chunk=MiB, digester="blake3", layers=1),
    "c1-sha256": dict(desc="C1 layer with the sha256 digester (a few chunks: the per-chunk "
                           "SHA-256 chain latency bounds it)",
                      tar="alpine_like", chunk=MiB, digester="sha256", layers=1),
    "c2": dict(desc="C2: 16 GiB layer tar, 4096 x 4 MiB files, 1 MiB chunks, blake3, no chunk dict",
               n_files=4096, file_size=4 * MiB, chunk=MiB, digester="blake3", layers=1),
    "c3": dict(desc="C3: 16 GiB layer, 1 MiB chunks, sha256, vs 200M-entry chunk dict in HBM "
                    "(30% of the layer's chunks planted)",
               n_files=4096, file_size=4 * MiB, chunk=MiB, digester="sha256", layers=1,
               dict_entries=200_000_000, plant=0.3, dict_file=True),
    "c3-64k": dict(desc="C3 layer with 64 KiB chunks: 16 GiB, sha256, 200M-entry chunk dict "
                        "(262144 chunks: one lane per chunk fills the chip)",
                   n_files=4096, file_size=4 * MiB, chunk=64 * 1024, digester="sha256", layers=1,
                   dict_entries=200_000_000, plant=0.3),
    "c3-blake3": dict(desc="C3 with blake3: 16 GiB layer, 1 MiB chunks, 200M-entry chunk dict",
                      n_files=4096, file_size=4 * MiB, chunk=MiB, digester="blake3", layers=1,
                      dict_entries=200_000_000, plant=0.3),
    "c4": dict(desc="C4: 1 TiB registry corpus = 1024 layers x 1 GiB (256 x 4 MiB files), 1 MiB "
                    "chunks, blake3, 30% of chunks drawn from a shared pool of 65536 contents "
                    "(counter-hash PRNG keyed by content id); chunk dict = pool digests + 16M "
                    "filler, partitioned by digest prefix over the GPUs, probes routed by "
                    "all-to-all; layers round-robin over the GPUs (at most 128 per GPU: one "
                    "GPU's share of the 8-GPU run)",
               n_files=256, file_size=4 * MiB, chunk=MiB, digester="blake3",
               layers_total=1024, max_layers_per_gpu=128, pool=65536,
               dict_entries=16_000_000, sharded=True),
    "c4-16": dict(desc="C4-shape per GPU: 16 x 1 GiB layers, 1 MiB chunks, blake3, 30% of chunks "
                       "from a shared pool of 65536 contents; chunk dict (pool + 16M filler) "
                       "partitioned by digest prefix over the GPUs, probes routed by all-to-all",
                  n_files=4096, file_size=4 * MiB, chunk=MiB, digester="blake3", layers=16,
                  pool=65536, dict_entries=16_000_000, sharded=True),
    "c5-1000": dict(desc="C5: 1000 layers x 64 MiB (16 x 4 MiB files), 64 KiB chunks, blake3, 30% of "
                         "chunks from a shared pool of 1024 contents; chunk dict (pool + 1M filler) "
                         "partitioned by digest prefix; layers split over the GPUs; one multi-layer "
                         "dedup launch set per step; then one host Merge of the layers' bootstraps",
                    n_files=16, file_size=4 * MiB, chunk=64 * 1024, digester="blake3",
                    layers_total=1000, pool=1024, dict_entries=1_000_000, sharded=True, merge=True),
    "c5": dict(desc="C5-shape: 16 GiB layer, 64 KiB chunks, blake3, no dict",
               n_files=1024, file_size=16 * MiB, chunk=64 * 1024, digester="blake3", layers=1),
    "small": dict(desc="1 GiB layer, 1 MiB chunks, blake3", n_files=256, file_size=4 * MiB,
                  chunk=MiB, digester="blake3", layers=1),
    # mid-size layers (the auto rule hashes them one leaf per lane or per lane quad)
    **{f"l{m}m": dict(desc=f"{m} MiB layer, 4 MiB files, 1 MiB chunks, blake3", n_files=m // 4,
                      file_size=4 * MiB, chunk=MiB, digester="blake3", layers=1)
       for m in (8, 16, 24, 32, 48, 64, 128, 256, 512, 1024, 2048)},
}


def pool_content(torch, ids, S, device="cuda"):
    """Pool contents for C4/C5: content i is a pure function of i (a splitmix64-
    style counter hash of (i, word index)), so every rank regenerates the same
    pool without holding it (65536 x 1 MiB would be 64 GiB)."""
    w = torch.arange(S // 8, dtype=torch.int64, device=device)
    z = (ids.to(torch.int64)[:, None] << 20) | w[None, :]
    z = z * -7046029254386353131 + 0x632BE59BD9B4E019  # 0x9E3779B97F4A7C15 as int64
    z = (z ^ ((z >> 30) & 0x3FFFFFFFF)) * -4658895280553007687  # 0xBF58476D1CE4E5B9
    z = (z ^ ((z >> 27) & 0x1FFFFFFFFF)) * -7723592293110705685  # 0x94D049BB133111EB
    z = z ^ ((z >> 31) & 0x1FFFFFFFF)
    return z.view(torch.uint8).view(len(ids), S)


def plant_pool(torch, buf, ch, stride, wl, seed):
    """C4/C5: overwrite ~30% of the chunks with pool contents (rank-seeded
    choice of chunks and of content ids).  -> ({"chunks": planted chunk ids,
    "content": their pool content ids}, count)."""
    S = wl["chunk"]
    per_file = wl["file_size"] // S
    n = len(ch)
    rows = buf[: wl["n_files"] * stride].view(wl["n_files"], stride)[:, 512:].view(wl["n_files"], per_file, S)
    rng = np.random.default_rng(seed)
    sel = np.nonzero(rng.random(n) < 0.3)[0]
    src = rng.integers(0, wl["pool"], len(sel))
    step = max(1, (256 * MiB) // S)
    for a in range(0, len(sel), step):
        f = torch.from_numpy(sel[a:a + step] // per_file).cuda()
        k = torch.from_numpy(sel[a:a + step] % per_file).cuda()
        rows[f, k] = pool_content(torch, torch.from_numpy(src[a:a + step]).cuda(), S)
    torch.cuda.synchronize()
    return {"chunks": sel, "content": src}, len(sel)


def pool_digests(torch, nydus_gpu, wl, device):
    """Digests of all pool contents (they go into the chunk dict)."""
    S, P = wl["chunk"], wl["pool"]
    eng = nydus_gpu.Engine(device=device, digester=wl["digester"], chunk_size=S)
    step = max(1, (512 * MiB) // S)
    out = torch.empty((P, 32), dtype=torch.uint8, device="cuda")
    pch = np.zeros(step, nydus_gpu.CHUNK_DTYPE)
    pch["offset"] = np.arange(step, dtype=np.uint64) * S
    pch["length"] = S
    d_pch = torch.from_numpy(pch.view(np.uint8).copy()).cuda()
    pout = torch.empty(step * 64, dtype=torch.uint8, device="cuda")
    try:
        for a in range(0, P, step):
            b = min(P, a + step)
            raw = pool_content(torch, torch.arange(a, b, device="cuda"), S).contiguous()
            # stream-ordered after pool_content's kernels
            eng.digest_device(raw.data_ptr(), raw.numel(), d_pch.data_ptr(), b - a, pout.data_ptr(),
                              stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            out[a:b] = pout.view(-1, 64)[: b - a, :32]
            del raw
    finally:
        eng.close()
    return out


def probe_bench(torch, nydus_gpu, eng, dd, Q, build_s, reps=5):
    """The chunk-dict probe alone (dict_probe_records through
    ngpu_dict_probe_device) over Q queries against the HBM-resident dict,
    30% of them planted dict digests: HIP-event time per launch on the
    launching stream, against the HBM roofline.  Algorithmic bytes per probe
    (for this layout): 32 B query + 8 B hash slot + 24 B hit
    record written, + 64 B dict record (key verify + hit fields) on a hit."""
    m = dd.shape[0]
    g = torch.Generator(device="cuda").manual_seed(0x9B0B)
    q = torch.empty((Q, 32), dtype=torch.uint8, device="cuda")
    q.random_(0, 256, generator=g)
    k = int(Q * 0.3)
    q[:k] = dd[torch.randint(0, m, (k,), device="cuda", generator=g)]
    q = q[torch.randperm(Q, device="cuda", generator=g)].contiguous()
    hits = torch.empty((Q, 6), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    eng.dict_probe_device(q.data_ptr(), 32, Q, hits.data_ptr(), stream=s.cuda_stream)  # warm
    ev[0].record(s)
    for r in range(reps):
        eng.dict_probe_device(q.data_ptr(), 32, Q, hits.data_ptr(), stream=s.cuda_stream)
        ev[r + 1].record(s)
    torch.cuda.synchronize()
    ms = [ev[r].elapsed_time(ev[r + 1]) for r in range(reps)]
    t = float(np.median(ms)) / 1e3
    nhit = int((hits[:, 0] != -1).sum())
    assert nhit >= k * 0.99, (nhit, k)
    alg = Q * (32 + 8 + 24) + nhit * 64
    del q, hits
    traffic, src = pmc_traffic("", "probe", "dict_probe_records")
    tr = {}
    if traffic:  # PMC request bytes of the same launches (scripts/gpu_pmc_probe.sh)
        tr = {"traffic": traffic, "traffic_source": src,
              "traffic_gbs": round(traffic / t / 1e9, 1),
              "traffic_frac": round(traffic / t / PEAK_HBM, 4),
              "lines_per_probe": round(traffic / 128 / Q, 2)}
        # the measured ceiling of random 128-B line reads on this chip
        # (tools/random_calib.hip: one random 8-B read, or a slot read and a
        # dependent 64-B record read, per thread over a table >= 4 GiB; the
        # request counters read exactly 1.000 / 2.000 lines per thread there)
        cal, csrc = newest_profile("random_calib.json")
        pm, _ = newest_profile("pmc_req_probe.json")
        if cal and pm and "read_request_bytes" in pm:
            big = [c for c in cal if c["table_bytes"] >= 4 << 30 and c["mode"] in (0, 3)]
            if big:
                ceil = max(c["reads"] * c["lines_per_read"] / (c["best_ms"] / 1e3) for c in big)
                lines_s = pm["read_request_bytes"] / 128 / t
                tr["random_line_ceiling"] = {
                    "glines_s": round(ceil / 1e9, 2), "probe_glines_s": round(lines_s / 1e9, 2),
                    "frac": round(lines_s / ceil, 4), "source": csrc,
                    "read_lines_per_probe": round(pm["read_request_bytes"] / 128 / Q, 3)}
    return {"kernel": "dict_probe_records", "queries": Q, "hits": nhit, "dict_entries": m, **tr,
            "ms": round(t * 1e3, 4), "gprobes_s": round(Q / t / 1e9, 2),
            "bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": round(PEAK_HBM / 1e9, 1),
            "unit": "GB/s", "frac": round(alg / t / PEAK_HBM, 4), "algorithmic_bytes": alg,
            # SURVEY.md §8(d)'s per-probe model: 32-B query + one 128-B bucket
            # line + 8-B result, + 32-B digest verify on a hit (~200 B)
            "line_model": {"bytes": Q * (32 + 128 + 8) + nhit * 32,
                           "frac": round((Q * (32 + 128 + 8) + nhit * 32) / t / PEAK_HBM, 4)},
            "build": {"kernel": "dict_insert", "entries": m, "s": round(build_s, 4),
                      "gentries_s": round(m / build_s / 1e9, 2)}}


def sharded_dict_extra(torch, dist, eng, buf, d_ch, n, stream, rank, world, backend,
                       entries=4 << 20, plant=0.3, steps=10, warmup=3):
    """N > 1 only: the C4 exchange on this run's layers, so the driver's
    multi-GPU run puts RCCL on xGMI under the product's dict path
    (nydus_gpu/dist.py).  Every rank plants 30 % of its own
    layer's chunk digests; one all_gather_into_tensor assembles the global
    dict (planted rows of every rank + random filler, same table on every
    rank), each rank keeps its digest-prefix partition
    (ShardedChunkDict.load -> ngpu_dict_create_device), and a step is
    digest -> all_to_all_single probe routing (counts, queries, hits back) ->
    dedup with the returned hits.  Checked: every rank's DICT count equals
    its planted count, summed over ranks.  Reported beside the headline
    line, never as `value`."""
    from nydus_gpu.dist import ShardedChunkDict, engine_load_fn, engine_probe_fn
    cdev = None if backend == "nccl" else "cpu"
    d_out = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    eng.digest_device(buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n, d_out.data_ptr())
    torch.cuda.synchronize()
    k = int(n * plant)
    g = torch.Generator(device="cuda").manual_seed(0xC4 + rank)
    sel = torch.randperm(n, device="cuda", generator=g)[:k]
    mine = d_out.view(n, 64)[sel, :32].contiguous()
    every = torch.empty((world * k, 32), dtype=torch.uint8, device="cuda")
    if cdev:
        parts = [torch.empty((k, 32), dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, mine.cpu())
        every.copy_(torch.cat(parts))
    else:
        dist.all_gather_into_tensor(every, mine)
    # the DICT decisions this rank must see: every chunk of its layer whose
    # digest any rank planted (a layer's duplicate chunks, and identical
    # layers on several ranks -- the c1 rehearsal -- hit more than once)
    planted = set(bytes(r) for r in every.cpu().numpy())
    expect = sum(bytes(r) in planted for r in d_out.view(n, 64)[:, :32].cpu().numpy())
    m = max(entries, world * k)
    gd = torch.Generator(device="cuda").manual_seed(0xD1C7)  # same filler on every rank
    dd = torch.empty((m, 32), dtype=torch.uint8, device="cuda")
    dd.random_(0, 256, generator=gd)
    dd[: world * k] = every
    us = torch.zeros((m,), dtype=torch.int32, device="cuda")  # usize 0: wildcard, any size hits
    bl = torch.randint(0, 8, (m,), dtype=torch.int32, device="cuda", generator=gd)
    ix = torch.arange(m, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    # equal splits (cap = this layer's chunk count, the same on every rank):
    # the probe never syncs with the host, so steps pipeline like the headline
    sdict = ShardedChunkDict(rank, world, comm_device=cdev, cap=n)
    local_m = sdict.load(dd, us, bl, ix, 8, engine_load_fn(eng, 8))
    sdict.probe_fn = engine_probe_fn(eng, stream_fn=lambda: stream.cuda_stream)
    del dd, us, bl, ix, every
    d_first = torch.tensor([0, n], dtype=torch.int64, device="cuda")
    d_lst = torch.zeros(256, dtype=torch.uint8, device="cuda")
    probe_s = []

    def step():
        with torch.cuda.stream(stream):
            s = stream.cuda_stream
            eng.digest_device(buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n, d_out.data_ptr(),
                              stream=s)
            t0 = time.perf_counter()
            hits = sdict.probe(d_out.view(n, 64)[:, :32])  # equal splits: no host sync
            probe_s.append(time.perf_counter() - t0)
            eng.dedup_layers_device(d_ch.data_ptr(), n, d_out.data_ptr(), d_first.data_ptr(), 1,
                                    d_lst.data_ptr(), d_hits=hits.data_ptr(), n_dict_blobs=8,
                                    stream=s)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    probe_s.clear()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    kinds = torch.bincount(d_out.view(n, 64)[:, 32].to(torch.int64), minlength=3).cpu()  # kind u32 @32
    agg = torch.tensor([el, float(kinds[2]), float(k), float(np.median(probe_s)), float(expect)],
                       dtype=torch.float64)
    red = [agg.clone() for _ in range(world)]
    if cdev:
        dist.all_gather(red, agg)
    else:
        redc = [r.cuda() for r in red]
        dist.all_gather(redc, agg.cuda())
        red = [r.cpu() for r in redc]
    red = torch.stack(red)
    el_max = float(red[:, 0].max())
    hits_all, planted_all, expect_all = int(red[:, 1].sum()), int(red[:, 2].sum()), int(red[:, 4].sum())
    return {"what": "C4 exchange on this run's layers: digest -> all_to_all_single dict probe "
                    "(digest-prefix partition; RCCL over xGMI when backend is nccl) -> dedup",
            "backend": backend, "collectives": ["all_gather_into_tensor (dict build)",
                                                "all_to_all_single x2 per step (queries, hits; "
                                                "equal padded splits, no host sync)"],
            "dict_entries": m, "entries_this_gpu": local_m, "steps": steps,
            "ms_per_step": round(el_max / steps * 1e3, 3),
            "probe_enqueue_ms_median_max_rank": round(float(red[:, 3].max()) * 1e3, 3),
            "dict_hits_all_ranks": hits_all, "planted_all_ranks": planted_all,
            "expected_hits_all_ranks": expect_all,
            "hits_ok": hits_all == expect_all, "_elapsed": el_max}


def dict_from_file(torch, nydus_gpu, eng, dd, us, bl, ix, wl, where):
    """C3's chunk dict through PackOption.ChunkDictPath: the dict's m records
    (digest, uncompressed size, blob, index: the arrays the device build
    used, so the decisions do not change) written as a RAFS v6 bootstrap
    (16 GB of chunk table for 200M entries; not timed), then ngpu_dict_open
    timed end to end -- read (page cache), parse, H2D, unpack, table build
    (csrc/dict.hip dict_stream_v6) -- and made the engine's dict for the
    timed steps.  The file is deleted afterwards.  A write failure (disk
    space) is reported and the device-built dict stays."""
    import shutil
    from nydus_gpu import rafs
    m, S = dd.shape[0], wl["chunk"]
    path = os.path.join(where or os.environ.get("TMPDIR") or "/tmp", f"nydus-c3-dict-{os.getpid()}.boot")
    need = m * 80 + (1 << 20)
    free = shutil.disk_usage(os.path.dirname(path)).free
    if free < need * 1.1:
        return {"skipped": f"{free / 1e9:.1f} GB free at {os.path.dirname(path)}, {need / 1e9:.1f} GB needed"}
    sha = wl["digester"] == "sha256"
    blobs = rafs.make_blob_table([f"{b:064x}" for b in range(8)], S, digester=wl["digester"])
    step = 8 << 20

    def pieces():
        for a in range(0, m, step):
            b = min(m, a + step)
            r = torch.zeros((b - a, 80), dtype=torch.uint8, device="cuda")
            r[:, :32] = dd[a:b]
            r[:, 32:36] = bl[a:b].contiguous().view(torch.uint8).view(b - a, 4)
            r[:, 40:44] = us[a:b].contiguous().view(torch.uint8).view(b - a, 4)  # compressed_size
            r[:, 44:48] = us[a:b].contiguous().view(torch.uint8).view(b - a, 4)  # uncompressed_size
            r[:, 72:76] = ix[a:b].contiguous().view(torch.uint8).view(b - a, 4)
            yield r.cpu().numpy().view(rafs.CHUNK_INFO_DTYPE).reshape(-1)
    try:
        t0 = time.perf_counter()
        size = rafs.write_v6_dict_file(path, m, S, pieces(), flags=0x8 if sha else 0x4, blobs=blobs)
        write_s = time.perf_counter() - t0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = eng.dict_open(path)
        open_s = time.perf_counter() - t0
        entries = d.entries
        eng.set_dict(d)  # the engine's dict for the timed steps (replaces the device build)
        d.release()
    except (OSError, nydus_gpu.NgpuError) as ex:
        return {"error": f"{type(ex).__name__}: {ex}"[:300]}
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass
    assert entries == m, (entries, m)
    return {"path": "ngpu_dict_open (PackOption.ChunkDictPath, builder.go:122-124)", "entries": m,
            "file_bytes": size, "chunk_table_bytes": m * 80, "open_s": round(open_s, 3),
            "chunk_table_gbs": round(m * 80 / open_s / 1e9, 2),
            "write_s_untimed": round(write_s, 2),
            "note": "file just written (page cache); open = read + parse + H2D + unpack + "
                    "table build, streamed in 1M-record pieces; this dict serves the timed steps"}


def merge_extra(nydus_gpu, ch, res, n_layers, per_layer, S, dict_host):
    """C5's last step ("chunk-dict Merge of 1000 layers", BASELINE configs[4]):
    after the timed digest + dedup steps, each layer's bootstrap is built from
    its decisions (RAFS v6: its NEW chunks -- ngpu_chunk_table -- and one
    record per (digest, blob) it reuses from the dict; blob table = the dict
    blobs it hit + its own blob, in real-index order), then ONE host
    ngpu_merge of all of them against the chunk dict bootstrap
    (convert_unix.go:560-666 -> nydus-image merge, builder.go:220-294).
    Merge is host bookkeeping: timed and reported here,
    never part of `value`."""
    from nydus_gpu import rafs
    dict_ids = [f"{b:064x}" for b in range(8)]
    t0 = time.perf_counter()
    boots, digs = [], []
    for l in range(n_layers):
        a, b = l * per_layer, (l + 1) * per_layer
        cl, rl = ch[a:b], res[a:b]
        new = nydus_gpu.chunk_table(cl, rl).view(rafs.CHUNK_INFO_DTYPE).reshape(-1)
        dm = rl["kind"] == nydus_gpu.DICT
        key = np.concatenate([rl["digest"][dm], rl["blob_index"][dm, None].view(np.uint8)], 1)
        _, first = np.unique(key, axis=0, return_index=True)
        sel = np.nonzero(dm)[0][np.sort(first)]
        dr = np.zeros(len(sel), rafs.CHUNK_INFO_DTYPE)
        dr["block_id"] = rl["digest"][sel]
        dr["blob_index"] = rl["blob_index"][sel]
        dr["compressed_size"] = dr["uncompressed_size"] = cl["length"][sel]
        dr["uncompressed_offset"] = rl["uncompressed_offset"][sel]
        dr["file_offset"] = cl["file_offset"][sel]
        dr["index"] = rl["index"][sel]
        nb = int(rl["blob_index"].max()) + 1 if len(rl) else 0
        ids = [""] * nb
        for r_, i_ in zip(rl["blob_index"][dm], rl["dict_blob"][dm]):
            ids[r_] = dict_ids[i_]
        own = f"{0xB10B0000 + l:064x}"
        ids = [x or own for x in ids]
        recs = np.concatenate([new, dr])
        boots.append(rafs.write_v6_bootstrap(recs, S, blobs=rafs.make_blob_table(ids, S)))
        digs.append(f"{0x1A7E0000 + l:064x}")
    dg, us, bl, ix = dict_host
    drec = np.zeros(len(dg), rafs.CHUNK_INFO_DTYPE)
    drec["block_id"] = dg
    drec["blob_index"] = bl
    drec["compressed_size"] = drec["uncompressed_size"] = us
    drec["index"] = ix
    drec["uncompressed_offset"] = ix.astype(np.uint64) * S
    dboot = rafs.write_v6_bootstrap(drec, S, blobs=rafs.make_blob_table(dict_ids, S))
    build_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    merged, blob_ids = nydus_gpu.merge(boots, digs, dboot)
    merge_s = time.perf_counter() - t0
    own_used = sum(1 for x in blob_ids if x not in dict_ids)
    return {"what": "one host Merge (ngpu_merge) of the step's per-layer bootstraps against the "
                    "chunk dict bootstrap", "layers": n_layers,
            "bootstraps_bytes": int(sum(len(b) for b in boots)), "dict_bootstrap_bytes": len(dboot),
            "bootstrap_build_s": round(build_s, 3), "merge_ms": round(merge_s * 1e3, 2),
            "merged_bytes": len(merged), "blobs": len(blob_ids), "own_blobs": own_used,
            "dict_blobs": len(blob_ids) - own_used}


def pmc_traffic(path, workload, kernel):
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3
    PMC summary of the same bench command.  Preferred: pmc_req_<workload>.json
    (scripts/gpu_pmc_req.sh: L2->fabric read requests by size x bytes +
    WRITE_SIZE, exact); else pmc_<workload>.json (scripts/gpu_pmc.sh:
    FETCH_SIZE x2 + WRITE_SIZE, the gfx950 rule for 128-B requests)."""
    import glob
    if not path:
        for name in (f"pmc_req_{workload}.json", f"pmc_{workload}.json"):
            cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)))
            path = cands[-1] if cands else ""
            if path:
                break
    if not path or not os.path.exists(path):
        return None, None
    d = json.load(open(path))
    if "traffic_bytes" not in d or kernel.split("<")[0] not in (d.get("kernel") or ""):
        return None, None
    return d["traffic_bytes"], os.path.relpath(path, ROOT)


def newest_profile(name):
    """The newest committed profiles/r*/<name> (or None)."""
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)))
    if not cands:
        return None, None
    return json.load(open(cands[-1])), os.path.relpath(cands[-1], ROOT)


def mix_roofline(roof, achieved, kernel, workload, comp=0):
    """the ceiling of the kernel's own instruction mix and
    the clock the chip holds under it.  peak_mix = 1024 SIMDs x 64 lanes x
    2.4 GHz / (issue cycles per algorithmic op of the compiled hot loop:
    tools/isa_mix.py -> profiles/r*/isa_mix_b3_groups.json; 3-operand ops 4
    cycles per wave64 instruction, 2-operand logic/add 2, as measured on this
    chip); held_clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / kernel time from a PMC
    pass of the same command (scripts/gpu_pmc_clock.sh ->
    profiles/r*/pmc_clock_<workload>.json, MI355X_MICROARCH.md "DVFS
    give-back").  frac_mix_at_held_clock = achieved / (peak_mix x held / 2.4):
    the issue efficiency left once the clock is accounted for."""
    if not kernel.startswith("b3_groups"):
        return
    mix, src = newest_profile("isa_mix_b3_groups.json")
    issue, isrc_ = newest_profile("valu_issue_model.json")
    pm = None
    if issue:
        # round 5: the measured issue cost of the kernel's
        # own mixed 2-/4-cycle G stream, per SIMD with every wave's HW_ID
        # (tools/valu_bank.hip): ~4 cycles per wave64 instruction at any
        # occupancy; the linear 2-/4-cycle model below is not reachable
        pm = issue["model"]["peak_tops_at_2p4ghz"] * 1e12
        roof.update({"peak_mix": round(pm / 1e12, 3), "frac_mix": round(achieved / pm, 4),
                     "mix": {"model": "measured issue cost of the mixed G stream",
                             "cycles_per_wave_instruction":
                                 issue["model"]["cycles_per_wave_instruction_mixed_stream"],
                             "kernel_cycles_per_valu_instruction_pmc":
                                 issue["b3_groups_c2_pmc"]["cycles_per_valu_instruction_per_simd"],
                             "source": isrc_}})
    if mix:
        lin = mix["peak_mix_tops_at_2p4ghz"] * 1e12
        lin_d = {"peak": round(lin / 1e12, 3), "frac": round(achieved / lin, 4),
                 "four_cycle_ops_per_compression": mix["per_compression"]["four_cycle"],
                 "two_cycle_ops_per_compression": mix["per_compression"]["two_cycle"],
                 "cycles_per_algorithmic_op": mix["cycles_per_algorithmic_op"], "source": src}
        if pm is None:  # no issue study committed: the linear model
            pm = lin
            roof.update({"peak_mix": lin_d["peak"], "frac_mix": lin_d["frac"], "mix": lin_d})
        else:
            lin_d["note"] = ("linear 2-/4-cycle model: unreachable on gfx950, a mixed stream "
                             "issues ~4 cycles per instruction (profiles/r5/valu_issue_model.json)")
            roof["linear_mix_model"] = lin_d
    clk, csrc = newest_profile(f"pmc_clock_{workload}.json")
    if clk and clk.get("clock_ghz"):
        # the clock a profiled pass held (another run than this line's): a
        # pointer, not a factor of any frac here (a ratio
        # of this run's time over another run's clock exceeded 1)
        roof["held_clock_ghz_profiled_pass"] = clk["clock_ghz"]
        roof["held_clock_source"] = csrc
    # where the rest goes: issued VALU wave-instructions
    # (PMC SQ_INSTS_VALU of the same command, profiles/r4/scripts/gpu_r4_measure.sh insts)
    # over the algorithmic ones (comp x 680 / 64 lanes); frac_mix factors into
    # clock (held / 2.4) x algorithmic / issued x the issue efficiency left
    # (the mixed 2- / 4-cycle stream against the linear cycle model)
    ins, isrc = newest_profile(f"pmc_insts_{workload}.json")
    if (ins and comp and "SQ_INSTS_VALU" in ins.get("counters", {})
            and (ins.get("kernel") or "").startswith(kernel.split("<")[0])):
        alg_wi = comp * OPS_PER_COMPRESSION / 64
        issued = ins["counters"]["SQ_INSTS_VALU"]
        d = {"valu_wave_instructions_issued": int(issued),
             "valu_wave_instructions_algorithmic": int(alg_wi),
             "issued_over_algorithmic": round(issued / alg_wi, 4), "source": isrc}
        if pm and clk and clk.get("clock_ghz"):
            cf = clk["clock_ghz"] / 2.4
            d["clock_factor"] = round(cf, 4)
            d["issue_efficiency_left"] = round(roof["frac_mix"] / cf / (alg_wi / issued), 4)
            d["note"] = ("frac_mix = clock_factor x (algorithmic / issued) x issue_efficiency_left; "
                         "the held clock is a profiled pass's (guide: profiled passes run up to "
                         "~5 % below an unprofiled run's clock)")
        roof["frac_mix_breakdown"] = d
    # the measured ceiling of the same compression stream with no memory
    # traffic (tools/b3_ceiling.hip at the kernel's occupancy, clock from its
    # own PMC pass): frac_ceiling = achieved / that rate; per-clock = the same
    # ratio with each side divided by the clock it held
    ceil_, ceil_src = newest_profile("b3_ceiling.json")
    if ceil_:
        w = str(ceil_["kernel_occupancy_waves_per_simd"])
        ct = ceil_["ceiling_tops_at_kernel_occupancy"] * 1e12
        roof["ceiling_measured"] = {"tops": round(ct / 1e12, 3), "waves_per_simd": int(w),
                                    "clock_ghz": ceil_["held_clock_ghz"].get(w), "source": ceil_src}
        roof["frac_ceiling"] = round(achieved / ct, 4)
        # per cycle: the kernel's algorithmic ops over its GRBM_GUI_ACTIVE / 8
        # cycles per launch (the clock pass; the cycle count, unlike the clock,
        # does not depend on the profiler slowing the launch down) against the
        # ceiling's ops per cycle


def tar_host_path(nydus_gpu, tar, wl, device, file_bytes, reps=200):
    """A real (small) layer tar from host memory, PCIe included: ngpu_pack_tar
    = host tar walk + H2D through the engine's pinned staging + digest +
    dedup + results back.  Per-layer latency and the rate it implies."""
    import ctypes
    eng = nydus_gpu.Engine(device=device, digester=wl["digester"], chunk_size=wl["chunk"])
    L = nydus_gpu.lib()
    hp = ctypes.c_void_p()
    assert L.ngpu_alloc_pinned(eng._h, len(tar), ctypes.byref(hp)) == 0
    host = np.ctypeslib.as_array((ctypes.c_uint8 * len(tar)).from_address(hp.value))
    host[:] = np.frombuffer(tar, np.uint8)
    try:
        for _ in range(10):
            eng.pack_tar(host)
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.pack_tar(host)
        dt = (time.perf_counter() - t0) / reps
        # the converter.Pack drop-in: streaming writer (ngpu_pack_write / close)
        # fed the tar in 1 MiB writes, through the engine's pinned staging slots
        def stream():
            w = eng.pack()
            for a in range(0, host.size, 1 << 20):
                w.write(host[a:a + (1 << 20)])
            return w.close()
        for _ in range(10):
            stream()
        t0 = time.perf_counter()
        for _ in range(reps):
            stream()
        ds = (time.perf_counter() - t0) / reps
    finally:
        L.ngpu_free_pinned(eng._h, hp)
        eng.close()
    return {"host_path_gbs": round(file_bytes / dt / 1e9, 2), "host_path_ms_per_layer": round(dt * 1e3, 4),
            "path": "ngpu_pack_tar from pinned host memory (tar walk + H2D + digest + dedup + D2H)",
            "streaming_gbs": round(file_bytes / ds / 1e9, 2), "streaming_ms_per_layer": round(ds * 1e3, 4),
            "streaming_path": "ngpu_pack_write in 1 MiB writes + ngpu_pack_close (staging memcpy, "
                              "H2D per slot, digest + dedup at close)"}


def end_to_end(torch, nydus_gpu, buf, wl, stride, device, sample_bytes=2 << 30):
    """PCIe-inclusive rates on the first `sample_files` files of the layer, held
    in engine-pinned host memory (never the headline value):
      host_path   — ngpu_pack_tar: host tar parse + one H2D copy + digest + dedup;
      streaming   — ngpu_pack write/close through two pinned staging slots
                    (H2D of slot k overlaps the digest of slot k-1), bytes
                    memcpy'd into staging by the caller."""
    import ctypes
    n_files = (buf.numel() - 1024) // stride
    sample_files = max(1, min(n_files, sample_bytes // stride))
    nbytes = sample_files * stride
    eng = nydus_gpu.Engine(device=device, digester=wl["digester"], chunk_size=wl["chunk"],
                           staging_bytes=64 << 20)
    L = nydus_gpu.lib()
    hp = ctypes.c_void_p()
    assert L.ngpu_alloc_pinned(eng._h, nbytes + 1024, ctypes.byref(hp)) == 0
    host = np.ctypeslib.as_array((ctypes.c_uint8 * (nbytes + 1024)).from_address(hp.value))
    host[:nbytes] = buf[:nbytes].cpu().numpy()
    host[nbytes:] = 0
    file_bytes = sample_files * wl["file_size"]
    res = {"sample_bytes": nbytes + 1024}
    try:
        eng.pack_tar(host)  # warm
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            ch, out, st = eng.pack_tar(host)
        res["host_path_gbs"] = round(file_bytes * reps / (time.perf_counter() - t0) / 1e9, 1)
        t0 = time.perf_counter()
        for _ in range(reps):
            w = eng.pack()
            for a in range(0, host.size, 32 << 20):
                w.write(host[a:a + (32 << 20)])
            ch2, out2, st2 = w.close()
        res["streaming_gbs"] = round(file_bytes * reps / (time.perf_counter() - t0) / 1e9, 1)
        assert out2.tobytes() == out.tobytes()
        res["bound"] = "PCIe Gen5 x16 H2D (~50-55 GB/s) and host memcpy into staging"
        # converter.Pack end to end: tar in -> nydus blob stream out (layer kept
        # in HBM, NEW chunks gathered on the GPU and copied back, per-chunk host
        # compression, host SHA-256 of the stream), written to /dev/null
        import hashlib
        fd = os.open(os.devnull, os.O_WRONLY)
        try:
            for comp in ("none", "zstd"):
                t0 = time.perf_counter()
                w = eng.pack(retain=True)
                for a in range(0, host.size, 32 << 20):
                    w.write(host[a:a + (32 << 20)])
                _, _, _, info = w.finish(nydus_gpu.FdWriter(fd), compressor=comp)
                res[f"pack_stream_{comp}_gbs"] = round(file_bytes / (time.perf_counter() - t0) / 1e9, 2)
                # what converter.Pack runs since round 4 (ngpu_pack_set_output):
                # the stream's NEW chunks are emitted slot by slot while the tar
                # is still being written, so host SHA-256 overlaps digesting
                t0 = time.perf_counter()
                w = eng.pack(retain=True)
                w.set_output(nydus_gpu.FdWriter(fd), compressor=comp)
                for a in range(0, host.size, 32 << 20):
                    w.write(host[a:a + (32 << 20)])
                _, _, _, info2 = w.finish(None)
                res[f"pack_stream_early_{comp}_gbs"] = round(file_bytes / (time.perf_counter() - t0) / 1e9, 2)
                assert info2["stream_digest"] == info["stream_digest"], "early emission changed the stream"
        finally:
            os.close(fd)
        t0 = time.perf_counter()
        hashlib.sha256(memoryview(host[:1 << 30])).digest()
        res["host_sha256_gbs"] = round((1 << 30) / (time.perf_counter() - t0) / 1e9, 2)
        res["pack_stream_bound"] = ("host SHA-256 of the output stream (sequential; the layer "
                                    "digest, SURVEY.md §8(a) a9) and host compression")
    finally:
        L.ngpu_free_pinned(eng._h, hp)
        eng.close()
    return res


def node_e2e(torch, dist, nydus_gpu, buf, wl, stride, device, backend, sample_bytes):
    """N > 1: every rank converts a sample of its layer from its own pinned host
    memory at the same time (ngpu_pack_tar: tar walk + H2D + digest + dedup +
    results back), barrier-bracketed, max time over ranks -- the node's
    PCIe-inclusive rate over all its GPUs' links together (one Gen5 x16 link
    per GPU), with the host memory they share.  Reported beside the line,
    never as `value`."""
    import ctypes
    n_files = (buf.numel() - 1024) // stride
    sample_files = max(1, min(n_files, sample_bytes // stride))
    nbytes = sample_files * stride
    eng = nydus_gpu.Engine(device=device, digester=wl["digester"], chunk_size=wl["chunk"])
    L = nydus_gpu.lib()
    hp = ctypes.c_void_p()
    assert L.ngpu_alloc_pinned(eng._h, nbytes + 1024, ctypes.byref(hp)) == 0
    try:
        host = np.ctypeslib.as_array((ctypes.c_uint8 * (nbytes + 1024)).from_address(hp.value))
        host[:nbytes] = buf[:nbytes].cpu().numpy()
        host[nbytes:] = 0
        file_bytes = sample_files * wl["file_size"]
        eng.pack_tar(host)  # warm
        reps = 3
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.pack_tar(host)
        dist.barrier()
        el = time.perf_counter() - t0
        t = torch.tensor([el], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    finally:
        L.ngpu_free_pinned(eng._h, hp)
        eng.close()
    world = dist.get_world_size()
    return {"host_path_gbs": round(file_bytes * reps * world / el / 1e9, 1),
            "per_gpu_gbs": round(file_bytes * reps / el / 1e9, 1),
            "sample_bytes_per_gpu": nbytes + 1024, "reps": reps,
            "path": "ngpu_pack_tar from pinned host memory on every rank at once",
            "bound": "one PCIe Gen5 x16 link per GPU (~50-55 GB/s H2D) and the host DRAM they share"}


SUB_KEYS = ("value", "unit", "ms_per_step", "steps", "warmup", "config", "stage_ms", "roofline",
            "cpu_baseline", "speedup_vs_cpu", "speedup_vs_cpu_single_stream", "dict",
            "probe_roofline", "merge", "decisions", "digest_check_past_4gib", "n_gpus", "sharded_dict",
            "e2e_pcie", "tar_host_path", "ranks", "modes", "speedup_vs_cpu_device", "bound",
            "stream_vs_cpu_pipeline")


def child_line(cmd, timeout_s, env=None):
    """Run a bench command as a child process and return its JSON line (or an
    error dict): a failure there costs only the entry that asked for it."""
    import subprocess
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, env=env)
    except subprocess.TimeoutExpired:
        return {"error": f"timeout after {timeout_s} s", "cmd": " ".join(cmd[1:])}
    lines = [x for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    if r.returncode or not lines:
        return {"error": f"rc {r.returncode}: {(r.stderr or '')[-400:]}", "cmd": " ".join(cmd[1:])}
    d = json.loads(lines[-1])
    out = {k: d[k] for k in SUB_KEYS if k in d}
    out["cmd"] = " ".join(cmd[1:])
    out["child_wall_s"] = round(time.perf_counter() - t0, 1)
    return out


def sub_entries(args):
    """N = 1: driver-timed evidence beside the C2 headline: C1 (the small
    alpine-like layer, with its host path), and for the dict paths (VERDICT r3
    item 5) C3 (sha256, 200M-entry dict in HBM, probe_roofline)
    and C5-1000 (1000 x 64 MiB layers, 64 KiB chunks, pool dict, one
    multi-layer dedup per step, then the host Merge of the 1000 bootstraps),
    each a full bench line of its own (value, ms_per_step, roofline,
    cpu_baseline), run as children after the headline is measured."""
    out = {}
    for key, wl in (("packs_c1", "c1"), ("packs_c1_sha256", "c1-sha256")):
        # K = 32 concurrent converter.Pack calls of C1-size layers (batched closes)
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", wl, "--packs", "32",
               "--steps", "10", "--warmup", "3", "--no-sub"]
        out[key] = child_line(cmd, 300)
    for key, wl in (("c1", "c1"), ("c3", "c3"), ("c5_1000", "c5-1000")):
        # C1 (configs[0], the reference's CPU-runnable case: one ~10 MB layer)
        # keeps its host path (ngpu_pack_tar from pinned host memory) and more
        # steps: a step is ~0.06 ms
        steps = args.sub_steps * 10 if wl == "c1" else args.sub_steps
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", wl, "--steps",
               str(steps), "--no-sub", "--settle-s", "1.0"] + ([] if wl == "c1" else ["--no-e2e"])
        out[key] = child_line(cmd, 420)
    return out


def multi_gpu_checks(line):
    """N > 1 lines: every hit-equality check the extras ran,
    in one summary.  True / False per check that ran; entries that failed to run
    are listed under `errors` (not counted as a wrong exchange).  `ok` is False
    when any check is False, and the run then exits non-zero after printing
    its line, so a wrong exchange cannot hide inside a JSON field."""
    checks, errors = {}, {}
    sx = line.get("sharded_dict")
    if isinstance(sx, dict):
        if "hits_ok" in sx:
            checks["sharded_dict.hits_ok"] = bool(sx["hits_ok"])
        elif "error" in sx:
            errors["sharded_dict"] = sx["error"]
    nc = line.get("node_cabi")
    if isinstance(nc, dict):
        if "hits_equal" in nc:
            checks["node_cabi.routed_copy_replicate.hits_equal"] = bool(nc["hits_equal"])
        elif "error" in nc:
            errors["node_cabi"] = nc["error"]
        for k, v in (nc.get("node_step") or {}).items():
            if isinstance(v, dict) and "hits_equal_partition" in v:
                checks[f"node_cabi.node_step.{k}.hits_equal"] = bool(v["hits_equal_partition"])
            elif isinstance(v, dict) and "error" in v:
                errors[f"node_cabi.node_step.{k}"] = v["error"]
    pn = line.get("packs_node")
    if isinstance(pn, dict):
        if "placement_all_parts" in pn:
            # placement follows load (fewest open Packs), so an uneven split
            # is not an error; a part left without Packs, or a lost chunk, is
            checks["packs_node.placement_all_parts"] = bool(pn["placement_all_parts"])
            if "chunks_ok" in pn:
                checks["packs_node.chunks_ok"] = bool(pn["chunks_ok"])
        elif "error" in pn:
            errors["packs_node"] = pn["error"]
    c4 = line.get("c4")
    if isinstance(c4, dict):
        dd = c4.get("dict") or {}
        if "dict_hits" in dd and "expected_dict_hits" in dd:
            checks["c4.dict_hits"] = dd["dict_hits"] >= 0.99 * dd["expected_dict_hits"]
        elif "error" in c4:
            errors["c4"] = c4["error"]
    return {"checks": checks, "errors": errors, "ok": all(checks.values())}


def fracs_over_one(obj, path=""):
    """Every `frac*` field above 1 in a bench line (every
    frac in the line must be <= 1; a ratio above 1 is not a fraction)."""
    out = []
    if isinstance(obj, dict):
        for k, v in obj.items():
            p = f"{path}.{k}" if path else k
            if (k.startswith("frac") or k.endswith("_frac")) and isinstance(v, (int, float)) and v > 1:
                out.append(p)
            out += fracs_over_one(v, p)
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            out += fracs_over_one(v, f"{path}[{i}]")
    return out


def exit_on_failed_checks(mg):
    """After the line is printed (and the ranks have left their barrier): a
    False multi-GPU check ends the run with status 4."""
    if mg is None or mg["ok"]:
        return
    bad = [k for k, v in mg["checks"].items() if not v]
    print(f"bench.py: multi-GPU check(s) failed: {', '.join(bad)}", file=sys.stderr, flush=True)
    sys.exit(4)


def c4_entry(world, layers, steps, backend="nccl", timeout_s=420):
    """N > 1, rank 0, after the headline: C4 itself on the
    run's GPUs -- a child `torchrun --nproc-per-node N bench.py --workload c4`:
    each rank converts `layers` 1 GiB layers (C4's 1024-layer corpus split
    round robin, at most 128 per GPU: one GPU's share of the 8-GPU node), 30 %
    of the chunks from the 65,536-content pool, against the pool + 16M-filler
    dict partitioned by digest prefix over the ranks; a timed step is digest
    -> RCCL all_to_all_single probe routing (owner bucketing by
    ngpu_route_digests) -> per-layer dedup of every layer.  The other ranks
    wait in a gloo barrier meanwhile."""
    env = dict(os.environ)
    for k in DIST_ENV:
        env.pop(k, None)
    cmd = self_launch_cmd([], world, free_port()) + ["--gpus", str(world), "--workload", "c4",
           "--steps", str(steps), "--warmup", "15", "--no-sharded-extra", "--no-node-extra",
           "--no-e2e", "--no-c4", "--c4-layers", str(layers), "--dist-backend", backend]
    return child_line(cmd, timeout_s, env=env)


def packs_node_extra(world, timeout_s=240):
    """N > 1, rank 0, after the headline: the Go drop-in's
    own path over the whole node -- `bench.py --workload c1 --packs 32N --node
    0,..,N-1` in a child process: 32 C1 converter.Pack calls per GPU from
    native threads, fed through ReadFrom (ngpu_pack_reserve / commit), each
    placed on the node's least-loaded engine (ngpu_node_pack_open), so every
    GPU's own PCIe link carries its share.  value = the node's file bytes per
    second, PCIe included; placement = Packs per GPU in the last round."""
    env = dict(os.environ)
    for k in DIST_ENV:
        env.pop(k, None)
    devs = os.environ.get("NYDUS_NODE_EXTRA_DEVICES") or ",".join(str(i) for i in range(world))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c1", "--packs", str(32 * world),
           "--node", devs, "--packs-modes", "decisions", "--no-cpu-baseline", "--steps", "10",
           "--warmup", "3"]
    import subprocess
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, env=env)
    except subprocess.TimeoutExpired:
        return {"error": f"timeout after {timeout_s} s", "devices": devs}
    lines = [x for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    if r.returncode or not lines:
        return {"error": f"rc {r.returncode}: {(r.stderr or '')[-300:]}", "devices": devs}
    d = json.loads(lines[-1])
    m = d["modes"]["decisions"]
    placed = m.get("packs_per_node_part_last_round") or []
    return {"devices": devs, "packs": 32 * world, "gbs": m["gbs"], "ms_per_round": m["ms_per_round"],
            "device_gbs": m.get("device_gbs"), "per_gpu_gbs": round(m["gbs"] / world, 2),
            "packs_per_gpu_last_round": placed,
            "placement_even": bool(placed) and max(placed) - min(placed) <= 1,
            "placement_all_parts": len(placed) == len(devs.split(",")) and min(placed) > 0,
            "chunks_ok": sum(m["decisions_last_round"].values()) == m.get("chunks_per_round"),
            "feed": m.get("feed"), "seconds": round(time.perf_counter() - t0, 1),
            "cmd": " ".join(cmd[1:])}


def node_cabi_extra(world, timeout_s=150):
    """N > 1, rank 0, after the headline: the C ABI's one-process node
    (ngpu_node_*, csrc/node.hip) over the run's GPUs, in a child process
    (`bench.py --node 0,1,..`, C4-shaped layers, a 1M-entry dict partitioned
    by digest prefix, then replicated): the in-process xGMI probe exchange a cgo
    caller gets, measured on the node's real links.  A child, so that a failure
    there costs only this entry.  NYDUS_NODE_EXTRA_DEVICES overrides the device
    list (one-GPU rehearsal: "0,0")."""
    import subprocess
    devs = os.environ.get("NYDUS_NODE_EXTRA_DEVICES") or ",".join(str(i) for i in range(world))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--node", devs, "--workload", "c4-16",
           "--steps", "5", "--warmup", "5", "--dict-entries", "1000000"]
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"error": f"timeout after {timeout_s} s", "devices": devs}
    lines = [x for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    if r.returncode or not lines:
        return {"error": f"rc {r.returncode}: {(r.stderr or '')[-300:]}", "devices": devs}
    d = json.loads(lines[-1])
    part, rep = d["modes"]["partition"], d["modes"]["replicate"]
    cp = d["modes"].get("partition_copy", {})
    return {"devices": d["node_devices"],
            "path": "ngpu_node_* in one process: routed exchange (peer kernel loads/stores over "
                    "xGMI), copy exchange (hipMemcpyPeerAsync) and replicas",
            "workload": "c4-16 layers per device, 1M-entry dict", "seconds": round(time.perf_counter() - t0, 1),
            "partition_gbs": part["value_gbs"], "replicate_gbs": rep["value_gbs"],
            "dedup_alone_ms_partition": part["dedup_alone_ms"],
            "dedup_alone_ms_replicate": rep["dedup_alone_ms"],
            "all_requesters_at_once_ms": {"partition": part["dedup_all_requesters_at_once_ms"],
                                          "replicate": rep["dedup_all_requesters_at_once_ms"]},
            "peer_bytes_per_step": d["exchange"]["peer_bytes_per_step"],
            "peer_bytes_per_step_copy": d["exchange"].get("peer_bytes_per_step_copy"),
            "partition_copy_gbs": cp.get("value_gbs"),
            "dedup_alone_ms_partition_copy": cp.get("dedup_alone_ms"),
            "dict_hits_partition": part["dict_hits"], "dict_hits_replicate": rep["dict_hits"],
            "dict_hits_partition_copy": cp.get("dict_hits"),
            "hits_equal": part["dict_hits"] == rep["dict_hits"] == cp.get("dict_hits", part["dict_hits"]),
            "node_step": d.get("node_step")}


def concurrent_bench(args):
    """`--streams K` (tar workloads, e.g. c1): ONE engine converts K copies of
    the layer side by side, one caller stream each -- the shape of containerd
    converting an image's layers concurrently (one LayerConvertFunc per
    layer, convert_unix.go:822) through one cached engine.  The engine gives
    calls on distinct streams distinct workspace slots (NGPU_WS_SLOTS), so a
    small layer, which leaves most of the chip idle (C1: <= one wave per SIMD,
    four launches), overlaps the others on the GPU's hardware queues.
    `--engines K`: K engines on device 0 instead (one stream each).  A step =
    one ngpu_process_device + the result table back, per stream.  value =
    the layers' file bytes of all streams / time."""
    import torch
    import nydus_gpu
    wl = dict(WORKLOADS[args.workload])
    if not wl.get("tar"):
        raise SystemExit("--engines takes a tar workload (c1)")
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import layers
    tar = layers.LAYERS[wl["tar"]]()
    ch = nydus_gpu.tar_chunks(tar, wl["chunk"])
    n, file_bytes = len(ch), int(ch["length"].sum())
    K = max(args.engines, args.streams)
    one = nydus_gpu.Engine(device=0, digester=wl["digester"], chunk_size=wl["chunk"]) \
        if args.engines <= 1 else None
    per = []
    for i in range(K):
        per.append(dict(
            eng=one or nydus_gpu.Engine(device=0, digester=wl["digester"], chunk_size=wl["chunk"]),
            buf=torch.from_numpy(np.frombuffer(tar, np.uint8).copy()).cuda(),
            d_ch=torch.from_numpy(ch.view(np.uint8).copy()).cuda(),
            d_out=torch.empty(n * 64, dtype=torch.uint8, device="cuda"),
            h_out=torch.empty(n * 64, dtype=torch.uint8, pin_memory=True),
            stream=torch.cuda.Stream()))
    torch.cuda.synchronize()

    def one(p):
        s = p["stream"]
        p["eng"].process_device(p["buf"].data_ptr(), p["buf"].numel(), p["d_ch"].data_ptr(), n,
                                p["d_out"].data_ptr(), stream=s.cuda_stream)
        with torch.cuda.stream(s):
            p["h_out"].copy_(p["d_out"], non_blocking=True)

    def step():
        for p in per:
            one(p)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if args.threads:
        # one submitting thread per stream (goroutines calling Pack); ctypes
        # drops the GIL inside the engine, the engine serialises only its
        # enqueue section
        import threading
        go = threading.Barrier(K + 1)

        def run(p):
            go.wait()
            for _ in range(args.steps):
                one(p)
            p["stream"].synchronize()
        th = [threading.Thread(target=run, args=(p,)) for p in per]
        for t in th:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        t_submit = elapsed
    else:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        t_submit = time.perf_counter() - t0  # host time spent enqueueing
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    ref = per[0]["h_out"].numpy().view(nydus_gpu.RESULT_DTYPE)
    for p in per[1:]:  # every engine's decisions equal
        assert (p["h_out"].numpy() == per[0]["h_out"].numpy()).all()
    kinds = np.bincount(ref["kind"], minlength=3)
    for e in {id(p["eng"]): p["eng"] for p in per}.values():
        e.close()
    value = file_bytes * K * args.steps / elapsed / 1e9
    line = {"metric": "GB/s of layer data chunk-hashed+deduped (node)", "value": round(value, 2),
            "unit": "GB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "dtype": "u32", "data": "synthetic alpine-like layer tar (tests/golden/layers.py)",
            "config": {"workload": wl["desc"], "name": args.workload,
                       "engines": 1 if one else K, "streams": K,
                       "submit": f"{K} threads" if args.threads else "one thread",
                       "ws_slots": int(os.environ.get("NGPU_WS_SLOTS", 4)),
                       "chunks": n, "file_bytes_per_layer": file_bytes},
            "us_per_layer": round(elapsed / args.steps / K * 1e6, 2),
            "host_submit_us_per_layer": round(t_submit / args.steps / K * 1e6, 2),
            "decisions": {"NEW": int(kinds[0]), "INTRA": int(kinds[1]), "DICT": int(kinds[2])}}
    print(json.dumps(line), flush=True)


def packs_bench(args):
    """`--packs K` (tar workloads, c1 / c1-sha256): K converter.Pack calls at
    once on ONE engine, one host thread each (containerd converting an image's
    layers concurrently: one LayerConvertFunc per layer, convert_unix.go:822),
    each pack its own distinct C1-size layer (alpine-like, seeds differ) fed
    from host memory in 1 MiB writes.  A round = the K packs opened, written,
    closed together; their closes coalesce into shared launch sets
    (csrc/batch.hip).  Modes, each `steps` rounds after
    `warmup`:
      decisions        -- close(): chunk list + digests + dedup decisions back;
      decisions_no_batch -- the same with NGPU_FLAG_NO_BATCH (a launch set per pack);
      stream_zstd      -- converter.Pack's own path: early emission
                          (ngpu_pack_set_output) of the nydus stream, zstd, to
                          a null sink.
    value = all layers' file bytes / wall time (PCIe-inclusive: the tars start
    in host memory).  device_gbs: the same bytes over the batched launch
    sets' device time (digest + dedup, HIP events).  cpu_baseline: the CPU
    digest+dedup stage on the same K layers, one layer per thread, on the
    host's cores."""
    import threading
    import nydus_gpu
    wl = dict(WORKLOADS[args.workload])
    if not wl.get("tar"):
        raise SystemExit("--packs takes a tar workload (c1, c1-sha256)")
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import layers
    K = args.packs
    tars = [layers.alpine_like_tar(0xA1F1E + i) for i in range(K)]
    chs = [nydus_gpu.tar_chunks(t, wl["chunk"]) for t in tars]
    file_bytes = sum(int(c["length"].sum()) for c in chs)
    n_chunks = sum(len(c["length"]) for c in chs)
    tar_bytes = sum(len(t) for t in tars)
    arrs = [np.frombuffer(t, np.uint8) for t in tars]

    class Null:
        def write(self, b):
            return len(b)

    drive = None
    dpath = os.path.join(ROOT, "nydus-snapshotter_amd", "build", "libpacks_drive.so")
    if os.path.exists(dpath):
        import ctypes
        drive = ctypes.CDLL(dpath).packs_drive
        drive.restype = ctypes.c_int
        vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        drive.argtypes = [vp, u32, ctypes.POINTER(vp), ctypes.POINTER(u64), u64, u32, u32, u32, u32,
                          ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64),
                          ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, u64, vp,
                          ctypes.POINTER(ctypes.c_int32)]
        tar_ptrs = (vp * K)(*[a.ctypes.data for a in arrs])
        tar_lens = (u64 * K)(*[a.size for a in arrs])

    node_devs = [int(x) for x in args.node.split(",")] if args.node else None

    def run_native(eng, stream, read_from, node=None):
        """The rounds on K native threads (tools/packs_drive.cpp: the cgo
        caller's shape, no GIL on the submit path).  read_from: the layers go
        in through ngpu_pack_reserve / commit (Go's PackWriter.ReadFrom, what
        io.Copy picks), else ngpu_pack_write from pageable memory.  node: the
        packs open on its least-loaded engine."""
        import ctypes
        R = args.warmup + args.steps
        rs = (ctypes.c_double * R)()
        per = (ctypes.c_uint64 * (4 * K))()
        part = (ctypes.c_int32 * K)()
        tr = np.zeros((R, K, 3), np.float64)
        err = ctypes.create_string_buffer(512)
        rc = drive(eng._h if node is None else None, K, tar_ptrs, tar_lens, 1 << 20,
                   (1 if stream else 0) | (2 if read_from else 0),
                   nydus_gpu._lib.DIGESTERS[wl["digester"]], wl["chunk"], R, rs, per,
                   tr.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), err, 512,
                   node._h if node is not None else None, part)
        if rc:
            (node or eng).close()
            raise RuntimeError(f"packs_drive rc={rc}: {err.value.decode(errors='replace')}")
        kinds = np.array(per, np.uint64).reshape(K, 4)[:, :3].sum(0)
        t = tr[args.warmup:] * 1e3  # timed rounds, ms from each round's start
        phases = {"last_write_ms_median": round(float(np.median(t[:, :, 1].max(1))), 3),
                  "write_ms_per_pack_median": round(float(np.median(t[:, :, 1] - t[:, :, 0])), 3),
                  "close_ms_per_pack_median": round(float(np.median(t[:, :, 2] - t[:, :, 1])), 3),
                  "close_ms_per_pack_max": round(float((t[:, :, 2] - t[:, :, 1]).max()), 3),
                  "tail_after_last_write_ms_median":
                      round(float(np.median(t[:, :, 2].max(1) - t[:, :, 1].max(1))), 3)}
        placed = None
        if node is not None:
            placed = [int((np.array(part) == j).sum()) for j in range(len(node_devs))]
        return sum(rs[args.warmup:]), kinds, R, phases, placed

    def run(flags, stream, native=False, read_from=True):
        # 16 MiB staging slots: a C1 layer fits one (it closes in a batch),
        # and 32 packs x 2 slots pin 1 GiB instead of 16
        node = None
        if native and node_devs:
            node = nydus_gpu.Node(node_devs, digester=wl["digester"], chunk_size=wl["chunk"],
                                  staging_bytes=16 << 20, timing=True, flags=flags)
            engs = node.engines
        else:
            eng = nydus_gpu.Engine(device=0, digester=wl["digester"], chunk_size=wl["chunk"],
                                   flags=flags, timing=True, staging_bytes=16 << 20)
            engs = [eng]
        if native:
            b_before = [e.batch_stats() for e in engs]  # (counted over every round: warmup included)
            el, kinds, R, phases, placed = run_native(engs[0], stream, read_from, node)
            b_after = [e.batch_stats() for e in engs]
            nb = sum(b["batches"] - a["batches"] for a, b in zip(b_before, b_after))
            npk = sum(b["packs"] - a["packs"] for a, b in zip(b_before, b_after))
            dev = None
            if nb:  # the launch sets' device time, each engine's own (they run side by side)
                dev_s, packs_in = 0.0, 0.0
                for e, a, b in zip(engs, b_before, b_after):
                    m = b["batches"] - a["batches"]
                    if not m:
                        continue
                    tms = [e.timing_at(k) for k in range(min(m, 64))]
                    dev_s = max(dev_s, sum(t["total_ms"] for t in tms) / 1e3 * m / min(m, 64))
                    packs_in += b["packs"] - a["packs"]
                dev = round(file_bytes / K * packs_in / dev_s / 1e9, 2) if dev_s else None
            (node or engs[0]).close()
            out = {"gbs": round(file_bytes * args.steps / el / 1e9, 2),
                   "ms_per_round": round(el / args.steps * 1e3, 3), "device_gbs": dev,
                   "feed": "ReadFrom (ngpu_pack_reserve / commit, 1 MiB source reads)" if read_from
                           else "Write (1 MiB ngpu_pack_write calls from pageable memory)",
                   "launch_sets_per_round": round(nb / R, 2),
                   "packs_per_set": round(npk / nb, 1) if nb else 0,
                   "most_packs_in_one_set": max(b["max_packs"] for b in b_after), "phases": phases,
                   "decisions_last_round": {"NEW": int(kinds[0]), "INTRA": int(kinds[1]),
                                            "DICT": int(kinds[2])},
                   "chunks_per_round": n_chunks}
            if placed is not None:
                out["packs_per_node_part_last_round"] = placed
            return out
        meet = threading.Barrier(K + 1)
        errs = []
        kinds = np.zeros(3, np.int64)
        mu = threading.Lock()

        def worker(i):
            try:
                for r in range(args.warmup + args.steps):
                    meet.wait()
                    w = eng.pack(retain=stream)
                    if stream:
                        w.set_output(Null(), compressor="zstd")
                    a = arrs[i]
                    for o in range(0, a.size, 1 << 20):
                        w.write(a[o:o + (1 << 20)])
                    if stream:
                        _, rs, _, _ = w.finish(None)
                    else:
                        _, rs, _ = w.close()
                    if r == args.warmup + args.steps - 1:
                        with mu:
                            kinds[:] += np.bincount(rs["kind"], minlength=3)[:3]
                    meet.wait()
            except Exception as ex:
                errs.append(repr(ex))
                meet.abort()
        th = [threading.Thread(target=worker, args=(i,)) for i in range(K)]
        for t in th:
            t.start()
        try:
            for r in range(args.warmup):
                meet.wait()
                meet.wait()
            b0 = eng.batch_stats()
            t0 = time.perf_counter()
            for r in range(args.steps):
                meet.wait()  # round r starts
                meet.wait()  # every pack of round r closed
            el = time.perf_counter() - t0
        except threading.BrokenBarrierError:
            el = None
        for t in th:
            t.join()
        if errs or el is None:
            eng.close()
            raise RuntimeError(f"packs: {errs[:2]}")
        b1 = eng.batch_stats()
        nb = b1["batches"] - b0["batches"]
        dev = None
        if nb:
            tms = [eng.timing_at(k) for k in range(min(nb, 64))]
            dev_ms = sum(t["total_ms"] for t in tms)
            packs_in = (b1["packs"] - b0["packs"]) * min(nb, 64) / nb
            dev = round(file_bytes / K * packs_in / (dev_ms / 1e3) / 1e9, 2) if dev_ms else None
        eng.close()
        return {"gbs": round(file_bytes * args.steps / el / 1e9, 2),
                "ms_per_round": round(el / args.steps * 1e3, 3),
                "device_gbs": dev, "launch_sets_per_round": round(nb / args.steps, 2),
                "packs_per_set": round((b1["packs"] - b0["packs"]) / nb, 1) if nb else 0,
                "most_packs_in_one_set": b1["max_packs"],
                "decisions_last_round": {"NEW": int(kinds[0]), "INTRA": int(kinds[1]),
                                         "DICT": int(kinds[2])}}

    if drive is None:
        raise SystemExit(f"{dpath} is missing: run `make -C nydus-snapshotter_amd`")
    # native threads (the cgo caller's shape) are the line; Python threads beside
    # (the reported mode is the drop-in's own feed, ReadFrom)
    plan = {"decisions": lambda: run(0, False, native=True),
            "decisions_write": lambda: run(0, False, native=True, read_from=False),
            "decisions_no_batch": lambda: run(nydus_gpu.FLAG_NO_BATCH, False, native=True),
            "stream_zstd": lambda: run(0, True, native=True),
            "stream_zstd_no_batch": lambda: run(nydus_gpu.FLAG_NO_BATCH, True, native=True)}
    if not node_devs:
        plan["decisions_python_threads"] = lambda: run(0, False)
    pick = [m for m in args.packs_modes.split(",") if m] if args.packs_modes else list(plan)
    if "decisions" not in pick or any(m not in plan for m in pick):
        raise SystemExit(f"--packs-modes: a subset of {list(plan)} with 'decisions'")
    modes = {m: plan[m]() for m in pick}
    cpu = None
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py
        from concurrent.futures import ThreadPoolExecutor
        aff, quota = host_cpus()
        threads = args.cpu_threads or (min(aff, int(-(-quota // 1))) if quota else aff)
        ochs = [c.view(oracle_py.CHUNK_DTYPE) for c in chs]
        oracle_py.cpu_digest_dedup(arrs[0], ochs[0][:4], wl["digester"], 1)

        def one_round(ex):
            list(ex.map(lambda i: oracle_py.cpu_digest_dedup(arrs[i], ochs[i], wl["digester"], 1),
                        range(K)))
        with ThreadPoolExecutor(threads) as ex:
            one_round(ex)
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < 3.0 and reps < 200:
                one_round(ex)
                reps += 1
            el = time.perf_counter() - t0
        cpu = {"value": round(file_bytes * reps / el / 1e9, 2), "unit": "GB/s", "cores": threads,
               "kind": "port", "sample": f"the same {K} layers ({file_bytes / MiB:.1f} MiB of file "
                                         f"data), digest+dedup, one layer per thread, "
                                         f"{oracle_py.cpu_impl()}; {reps} rounds"}
        # the whole CPU converter pipeline per layer (digest + dedup + zstd of
        # the NEW chunks + SHA-256 of the stream), against stream_zstd
        if oracle_py.cpu_pack_pipeline(arrs[0], ochs[0][:4], wl["digester"]) is not None:
            with ThreadPoolExecutor(threads) as ex:
                def pipe_round():
                    list(ex.map(lambda i: oracle_py.cpu_pack_pipeline(arrs[i], ochs[i], wl["digester"]),
                                range(K)))
                pipe_round()
                reps, t0 = 0, time.perf_counter()
                while time.perf_counter() - t0 < 3.0 and reps < 100:
                    pipe_round()
                    reps += 1
                el = time.perf_counter() - t0
            cpu["pipeline_gbs"] = round(file_bytes * reps / el / 1e9, 2)
            cpu["pipeline"] = ("per layer on one thread: digests + stream dedup + zstd level 1 of the "
                               "NEW chunks (libzstd) + SHA-256 of the compressed stream (OpenSSL)")
    line = {"metric": "GB/s of layer data chunk-hashed+deduped (node)",
            "value": modes["decisions"]["gbs"], "unit": "GB/s",
            "n_gpus": len(set(node_devs)) if node_devs else 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": modes["decisions"]["ms_per_round"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic alpine-like layer tars (tests/golden/layers.py), host memory",
            "config": {"workload": f"{K} concurrent converter.Pack calls of distinct C1-size "
                                   f"layers on " + (f"a node of devices {node_devs} (least-loaded "
                                                    f"engine per Pack)" if node_devs else "one engine")
                                   + f" ({wl['digester']}, 1 MiB chunks)",
                       "name": args.workload, "packs": K, "file_bytes_per_round": file_bytes,
                       "tar_bytes_per_round": tar_bytes, "batch_window_us": 2000 if wl["digester"] == "sha256" else 250, "batch_lanes": 4,
                       "caller": "K native threads (tools/packs_drive.cpp); 'decisions' feeds "
                                 "through ReadFrom (ngpu_pack_reserve / commit, the Go drop-in's "
                                 "io.Copy path), 'decisions_write' through 1 MiB ngpu_pack_write "
                                 "calls from pageable memory"},
            "modes": modes, "cpu_baseline": cpu,
            "bound": "blake3: PCIe H2D of the tars through 2 shared copy lanes (~45 GB/s, "
                     "tools/h2d_streams); sha256: one 1 MiB chunk's chain per batch (~21 ms) "
                     "whatever its size; stream: host zstd level 1 on the 16-core quota"}
    if cpu:
        line["speedup_vs_cpu"] = round(modes["decisions"]["gbs"] / cpu["value"], 2)
        if cpu.get("pipeline_gbs") and "stream_zstd" in modes:
            line["stream_vs_cpu_pipeline"] = round(modes["stream_zstd"]["gbs"] / cpu["pipeline_gbs"], 2)
        if modes["decisions"]["device_gbs"]:
            line["speedup_vs_cpu_device"] = round(modes["decisions"]["device_gbs"] / cpu["value"], 2)
    print(json.dumps(line), flush=True)


def node_bench(args):
    """`--node 0,1,..`: ONE process drives the listed GPUs through the C ABI's
    multi-GPU node (ngpu_node_*, csrc/node.hip) -- the form a cgo
    caller uses.  Each device holds its own layer set of the workload; one node
    dict (pool digests + filler, 80-B RAFS v6 records) is built partitioned by
    digest prefix, then replicated, and every step runs
    ngpu_node_process_device on every device (digest + the dedup stage, whose
    probe goes over the exchange when partitioned).  The two modes' dedup
    times give the exchange cost.  Listing one device several times rehearses
    the node on one GPU (the copies then stay inside one HBM).  Not the
    driver's line (that is the one-process-per-GPU launch in main())."""
    import torch
    import nydus_gpu
    from nydus_gpu import rafs
    devs = [int(x) for x in args.node.split(",")]
    W = len(devs)
    wl = dict(WORKLOADS[args.workload])
    if not wl.get("pool") or wl.get("tar"):
        raise SystemExit("--node takes a layered dict workload (c4-16, c5-1000)")
    if wl.get("layers_total"):
        wl["layers"] = -(-wl["layers_total"] // W)
        wl["n_files"] *= wl["layers"]
    if args.dict_entries:
        wl["dict_entries"] = args.dict_entries
    S, m, L = wl["chunk"], wl["dict_entries"], wl["layers"]
    node = nydus_gpu.Node(devs, digester=wl["digester"], chunk_size=S, timing=True)
    per = []
    try:
        _, stride, _, _ = synthetic_layout(1, wl["file_size"], S)
        for i, dev in enumerate(devs):
            with torch.cuda.device(dev):
                buf, ch = build_layer_on_gpu(torch, wl["n_files"], wl["file_size"], S,
                                             seed=0x6E79647573 + i)
                _, planted = plant_pool(torch, buf, ch, stride, wl, seed=i)
                n = len(ch)
                first = np.arange(L + 1, dtype=np.int64) * (n // L)
                per.append(dict(
                    dev=dev, buf=buf, n=n, planted=planted, bytes=int(ch["length"].sum()),
                    d_ch=torch.from_numpy(ch.view(np.uint8).copy()).cuda(),
                    out=torch.empty(n * 64, dtype=torch.uint8, device="cuda"),
                    first=torch.from_numpy(first).cuda(),
                    st=torch.zeros(L * nydus_gpu.LAYER_STATS_DTYPE.itemsize, dtype=torch.uint8,
                                   device="cuda"),
                    stream=torch.cuda.Stream()))
        with torch.cuda.device(devs[0]):
            pool = pool_digests(torch, nydus_gpu, wl, devs[0]).cpu().numpy()
        rng = np.random.default_rng(0xD1C7)
        recs = np.zeros(m, rafs.CHUNK_INFO_DTYPE)
        recs["block_id"][: len(pool)] = pool
        recs["block_id"][len(pool):] = rng.integers(0, 256, (m - len(pool), 32), dtype=np.uint8)
        recs["uncompressed_size"] = S
        recs["compressed_size"] = S
        recs["blob_index"] = rng.integers(0, 8, m)
        recs["index"] = np.arange(m)
        recs["uncompressed_offset"] = np.arange(m, dtype=np.uint64) * S
        blobs = rafs.make_blob_table([f"{b:064x}" for b in range(8)], S)
        del pool
        torch.cuda.synchronize()

        def step(d):
            for i, p in enumerate(per):
                node.process_device(i, d, p["buf"].data_ptr(), p["buf"].numel(), p["d_ch"].data_ptr(),
                                    p["n"], p["out"].data_ptr(), p["first"].data_ptr(), L,
                                    p["st"].data_ptr(), stream=p["stream"].cuda_stream)

        def sync():
            for p in per:
                p["stream"].synchronize()

        modes = {}
        for name, mode in (("partition", nydus_gpu.NODE_DICT_PARTITION | nydus_gpu.NODE_EXCHANGE_ROUTED),
                           ("partition_copy", nydus_gpu.NODE_DICT_PARTITION | nydus_gpu.NODE_EXCHANGE_COPY),
                           ("replicate", nydus_gpu.NODE_DICT_REPLICATE)):
            t0 = time.perf_counter()
            d = node.dict_create(recs, blobs, mode=mode)
            build_s = time.perf_counter() - t0
            for _ in range(args.warmup):
                step(d)
            sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step(d)
            sync()
            elapsed = time.perf_counter() - t0
            hits = []
            for i, p in enumerate(per):
                res = p["out"].cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
                hits.append(int((res["kind"] == nydus_gpu.DICT).sum()))
                assert hits[-1] >= p["planted"] * 0.99, (name, i, hits[-1], p["planted"])
            tm = [e.timing_at(b) for e in node.engines for b in range(min(args.steps, 64))]
            total = sum(p["bytes"] for p in per) * args.steps
            # the dedup stage alone (dict routing + exchange + dedup kernels),
            # one engine at a time so no other engine's digest shares the GPU:
            # ngpu_dedup_layers_device with the node dict as the engine default
            alone = []
            for i, p in enumerate(per):
                e = node.engines[i]
                e.set_dict(d)
                with torch.cuda.device(p["dev"]):
                    # every rerun starts from digest-stage records (kind =
                    # NGPU_DIGESTED: the dedup stage takes only those), so the
                    # mark is restored before each timed dedup, outside its events
                    kind = p["out"].view(torch.int32).view(p["n"], 16)[:, 8]
                    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(25)]
                    with torch.cuda.stream(p["stream"]):
                        for r in range(25):
                            kind.fill_(nydus_gpu.DIGESTED)
                            ev[r][0].record(p["stream"])
                            e.dedup_layers_device(p["d_ch"].data_ptr(), p["n"], p["out"].data_ptr(),
                                                  p["first"].data_ptr(), L, p["st"].data_ptr(),
                                                  stream=p["stream"].cuda_stream)
                            ev[r][1].record(p["stream"])
                    p["stream"].synchronize()
                    e.device_status()
                    alone.append(float(np.mean([a.elapsed_time(b) for a, b in ev[5:]])))
                e.set_dict(None)
            # all W requesters' dedup stages at once (each engine on its own
            # stream): the exchange under contention, host-timed from the first
            # enqueue to the last stream's end
            for i, p in enumerate(per):
                node.engines[i].set_dict(d)
            conc = []
            for r in range(15):
                for p in per:
                    with torch.cuda.device(p["dev"]), torch.cuda.stream(p["stream"]):
                        p["out"].view(torch.int32).view(p["n"], 16)[:, 8].fill_(nydus_gpu.DIGESTED)
                sync()
                t0 = time.perf_counter()
                for i, p in enumerate(per):
                    node.engines[i].dedup_layers_device(p["d_ch"].data_ptr(), p["n"], p["out"].data_ptr(),
                                                        p["first"].data_ptr(), L, p["st"].data_ptr(),
                                                        stream=p["stream"].cuda_stream)
                sync()
                conc.append((time.perf_counter() - t0) * 1e3)
            for i, p in enumerate(per):
                node.engines[i].device_status()
                node.engines[i].set_dict(None)
            modes[name] = {"dict_build_s": round(build_s, 2), "ms_per_step": round(elapsed / args.steps * 1e3, 3),
                           "value_gbs": round(total / elapsed / 1e9, 1),
                           "digest_ms": round(float(np.mean([t["digest_ms"] for t in tm])), 3),
                           "dedup_ms": round(float(np.mean([t["dedup_ms"] for t in tm])), 3),
                           "dedup_alone_ms": [round(a, 4) for a in alone],
                           "dedup_all_requesters_at_once_ms": round(float(np.median(conc[3:])), 4),
                           "dict_hits": hits}
            d.release()
        # the bulk node step (ngpu_node_process_step, ABI 5): all devices at
        # once, one all-to-all-v of digests and one of hits per step -- over
        # RCCL (ncclAllToAllv) when the devices are distinct, and by peer
        # copies (any node, the one-GPU rehearsal too)
        step_modes = {}
        d = node.dict_create(recs, blobs, mode=nydus_gpu.NODE_DICT_PARTITION)
        parts = [{"d_data": p["buf"].data_ptr(), "len": p["buf"].numel(), "d_chunks": p["d_ch"].data_ptr(),
                  "n": p["n"], "d_out": p["out"].data_ptr(), "d_layer_first": p["first"].data_ptr(),
                  "n_layers": L, "d_stats": p["st"].data_ptr(), "stream": p["stream"].cuda_stream}
                 for p in per]
        for tname, rccl in (("copy", False), ("rccl", True)):
            if rccl and len(set(devs)) != W:
                step_modes[tname] = {"skipped": "RCCL takes one rank per GPU; devices repeat"}
                continue
            try:
                for _ in range(args.warmup):
                    node.process_step(d, parts, rccl=rccl)
                sync()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    node.process_step(d, parts, rccl=rccl)
                sync()
                elapsed = time.perf_counter() - t0
            except nydus_gpu.NgpuError as ex_:
                step_modes[tname] = {"error": str(ex_)}
                continue
            hits = []
            for p in per:
                res = p["out"].cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
                hits.append(int((res["kind"] == nydus_gpu.DICT).sum()))
            total = sum(p["bytes"] for p in per) * args.steps
            step_modes[tname] = {"ms_per_step": round(elapsed / args.steps * 1e3, 3),
                                 "value_gbs": round(total / elapsed / 1e9, 1), "dict_hits": hits,
                                 "hits_equal_partition": hits == modes["partition"]["dict_hits"]}
        for e in node.engines:
            e.device_status()
        d.release()
        ex = float(np.mean(modes["partition"]["dedup_alone_ms"])) - \
            float(np.mean(modes["replicate"]["dedup_alone_ms"]))
        ex_copy = float(np.mean(modes["partition_copy"]["dedup_alone_ms"])) - \
            float(np.mean(modes["replicate"]["dedup_alone_ms"]))
        n_all = sum(p["n"] for p in per)
        # rows whose owner part is another part than the requester's: the rows
        # that cross a link on a node of distinct devices (routed: 32 + 4 B out,
        # 24 B back each); the copy exchange sends all n rows to each of the
        # W - 1 other parts and gets n hits back from each
        from nydus_gpu.dist import owner_of
        remote = 0
        for i, p in enumerate(per):
            with torch.cuda.device(p["dev"]):
                dg = p["out"].view(p["n"], 64)[:, :32]
                remote += int((owner_of(dg, W) != i).sum())
        routed_bytes = remote * (32 + 4 + 24)  # + a few counter words per probe launch
        line = {
            "metric": "GB/s of layer data chunk-hashed+deduped (node, one process)",
            "value": modes["partition"]["value_gbs"], "unit": "GB/s", "n_gpus": len(set(devs)),
            "node_devices": devs, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": modes["partition"]["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (random bytes generated on the GPU, real GNU tar headers; pool "
                    "contents planted)",
            "config": {"workload": wl["desc"], "name": args.workload, "layers_per_device": L,
                       "chunks_per_device": per[0]["n"], "dict_entries": m,
                       "parallelism": f"node x{W} (ngpu_node_*, one process)"},
            "modes": modes,
            "node_step": step_modes,
            "exchange": {"dedup_alone_ms_partition_minus_replicate": round(ex, 4),
                         "all_requesters_at_once_ms_partition_minus_replicate": round(
                             modes["partition"]["dedup_all_requesters_at_once_ms"]
                             - modes["replicate"]["dedup_all_requesters_at_once_ms"], 4),
                         "dedup_alone_ms_copy_minus_replicate": round(ex_copy, 4),
                         "all_requesters_at_once_ms_copy_minus_replicate": round(
                             modes["partition_copy"]["dedup_all_requesters_at_once_ms"]
                             - modes["replicate"]["dedup_all_requesters_at_once_ms"], 4),
                         "peer_bytes_per_step": routed_bytes,
                         "peer_bytes_per_step_copy": n_all * (32 + 24) * (W - 1),
                         "peer_bytes_ratio_copy_over_routed": round(n_all * 56 * (W - 1) / max(1, routed_bytes), 2),
                         "note": "'partition' = routed (opt-in since ABI 7, NGPU_NODE_EXCHANGE_ROUTED): "
                                 "each requester buckets its digests by owner; "
                                 "owner o's probe kernel reads only its rows (32-B digest + 4-B row id, "
                                 "peer loads) and stores 24-B hits at their rows (peer stores), plus the "
                                 "W counters it reads; 'partition_copy' = copy (the default since ABI 7): every "
                                 "digest to each of the W-1 other owners, 24-B hits back from each. On a "
                                 "one-GPU rehearsal the peer traffic stays in one HBM and the W engines "
                                 "share the GPU"},
        }
        print(json.dumps(line), flush=True)
    finally:
        per.clear()
        node.close()


DIST_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
            "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
            "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "GROUP_WORLD_SIZE")


def free_port() -> int:
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def self_launch_cmd(argv, gpus: int, port: int):
    """The torchrun command `python bench.py --gpus N ...` (no WORLD_SIZE in
    the environment) runs as: N ranks on this node, rendezvous on 127.0.0.1,
    every argument passed through unchanged."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def maybe_self_launch(args, argv, env=None, runner=None):
    """`--gpus N > 1` without a launcher around us: start the N worker processes
    as a child torchrun and relay rank 0's line (the children inherit stdout).
    Called before torch is imported, so this parent never touches the GPU: it
    only waits, forwards SIGTERM / SIGINT to the child, and exits with the
    child's status.  -> None when this process is itself a rank (or N = 1)."""
    env = dict(os.environ if env is None else env)
    if args.gpus <= 1 or env.get("WORLD_SIZE") or args.node:
        return None
    for k in DIST_ENV:
        env.pop(k, None)
    env["NYDUS_BENCH_LAUNCHER"] = "self"
    cmd = self_launch_cmd(argv, args.gpus, free_port())
    if runner is not None:
        return runner(cmd, env)
    import signal
    import subprocess
    p = subprocess.Popen(cmd, env=env)

    def fwd(sig, _frame):
        try:
            p.send_signal(sig)
        except OSError:
            pass
    for s in (signal.SIGTERM, signal.SIGINT):
        signal.signal(s, fwd)
    return p.wait()


def rank_check(args, dist, world, rank, local, backend, torch, group=None):
    """Every rank: the world it joined must be the one asked for (`--gpus`);
    a mismatch exits non-zero on every rank.  -> what the line reports about
    the ranks: world size, RCCL world size (nccl backend), and how many
    distinct GPUs the ranks sit on (by device UUID)."""
    if world != args.gpus:
        print(f"bench.py: rank {rank} joined a world of {world} ranks, --gpus {args.gpus}",
              file=sys.stderr, flush=True)
        raise SystemExit(4)
    try:
        dev = str(torch.cuda.get_device_properties(local).uuid)
    except (AttributeError, RuntimeError):
        dev = f"local{local}"
    devs = [dev]
    if dist is not None:
        devs = [None] * world
        dist.all_gather_object(devs, dev, group=group)
    return {"world_size": world, "requested": args.gpus, "backend": backend if dist else None,
            "rccl_world_size": world if dist is not None and backend == "nccl" else None,
            "distinct_devices": len(set(devs)),
            "launcher": os.environ.get("NYDUS_BENCH_LAUNCHER") or ("torchrun" if dist else "none")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--settle-s", type=float, default=1.0,
                    help="after the W warmup steps, more untimed steps until the warm-up has "
                         "lasted this long (GPU clock ramp); 0 = W steps only")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps (default 20; 80 for the pool/dict workloads, whose setup -- "
                         "64 GiB of pool hashed, a 16M-200M entry dict built, GBs freed -- leaves "
                         "the GPU ~30%% slow for ~150 ms after it: profiles/r2/c4-16_warmup_r2u.json)")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--lanes", type=int, default=0, help="leaves per lane (0=auto)")
    ap.add_argument("--load-mode", type=int, default=-1,
                    help="BLAKE3 load mode override (diagnostics: 4 = no loads, needs a "
                         "-DNGPU_DIAG_NOLOAD=1 build via NYDUS_GPU_LIB; its digests are not BLAKE3)")
    ap.add_argument("--sha-mode", choices=list(SHA_MODES), default="auto",
                    help="SHA-256 kernel: one lane per chunk (lane; split = schedule/round "
                         "waves) or two (pair)")
    ap.add_argument("--dict-entries", type=int, default=0, help="override dict size")
    ap.add_argument("--digester", choices=["blake3", "sha256"], default=None,
                    help="override the workload's digester (e.g. the sha256 small-layer crossover sweep)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dict-file", action="store_true",
                    help="c3: skip the ChunkDictPath file (build the dict from device arrays only)")
    ap.add_argument("--dict-dir", default="", help="where c3 writes its ChunkDictPath file "
                    "(default $TMPDIR or /tmp)")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--d2h", choices=["auto", "same", "copy"], default="auto",
                    help="result-table D2H: on the call's stream (same) or on a copy stream "
                         "overlapping the next step (copy); auto = same below 1 MiB of results")
    ap.add_argument("--e2e-mib", type=int, default=2048, help="PCIe-inclusive sample size")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) on a node; gloo to "
                    "rehearse several ranks on one GPU")
    ap.add_argument("--pmc-json", default="", help="PMC summary for roofline.traffic "
                    "(default: newest profiles/r*/pmc_<workload>.json)")
    ap.add_argument("--cpu-sample-mib", type=int, default=2048)
    ap.add_argument("--no-sharded-extra", action="store_true",
                    help="N > 1: skip the RCCL-routed partitioned-dict step run after the "
                         "headline measurement")
    ap.add_argument("--no-node-extra", action="store_true",
                    help="N > 1: skip rank 0's child run of the C ABI node (ngpu_node_*) over "
                         "the run's GPUs after the headline measurement")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--probe-queries", type=int, default=16 << 20,
                    help="dict workloads: queries of the probe-only roofline measurement (0 = skip)")
    ap.add_argument("--dump-timings", action="store_true",
                    help="add every timed call's stage times (oldest first) to the line")
    ap.add_argument("--streams", type=int, default=1,
                    help="tar workloads: one engine converts K layers at once, one stream each")
    ap.add_argument("--threads", action="store_true",
                    help="--streams/--engines: one submitting host thread per stream")
    ap.add_argument("--packs", type=int, default=0,
                    help="tar workloads: K concurrent converter.Pack calls per round on one engine "
                         "(batched closes); see packs_bench")
    ap.add_argument("--packs-modes", default="",
                    help="--packs: comma-separated modes to run (default all; 'decisions' required)")
    ap.add_argument("--engines", type=int, default=1,
                    help="tar workloads: K engines on device 0 convert layers concurrently")
    ap.add_argument("--no-sub", action="store_true",
                    help="N = 1, c2: skip the c3 / c5_1000 sub-entries (child runs after the headline)")
    ap.add_argument("--sub-steps", type=int, default=20, help="timed steps of each sub-entry child")
    ap.add_argument("--no-c4", action="store_true",
                    help="N > 1: skip the c4 entry (a child torchrun of --workload c4 over the GPUs)")
    ap.add_argument("--c4-layers", type=int, default=128,
                    help="N > 1 c4 entry: 1 GiB layers per GPU (C4's share of 8 GPUs: 128)")
    ap.add_argument("--node", default="", help="comma list of devices: one process drives them "
                    "through ngpu_node_* (a device may repeat: one-GPU rehearsal); see node_bench")
    args = ap.parse_args()
    rc = maybe_self_launch(args, sys.argv[1:])
    if rc is not None:
        raise SystemExit(rc)
    if args.warmup is None:
        w = WORKLOADS[args.workload]
        args.warmup = 80 if (w.get("pool") or w.get("dict_entries")) else 20
    if args.packs:  # (with --node: the packs spread over the node's engines)
        return packs_bench(args)
    if args.node:
        return node_bench(args)
    if args.engines > 1 or args.streams > 1:
        return concurrent_bench(args)

    import torch
    import nydus_gpu

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
        # host-side barriers (the closing one): while rank 0 runs the node child
        # on every GPU, the other ranks wait on the CPU, not in an RCCL kernel
        cpu_group = dist.new_group(backend="gloo")
    ranks = rank_check(args, dist, world, rank, local, args.dist_backend, torch,
                       cpu_group if dist else None)

    wl = dict(WORKLOADS[args.workload])
    if args.dict_entries:
        wl["dict_entries"] = args.dict_entries
    if args.digester:
        wl["digester"] = args.digester
    if wl.get("layers_total"):  # split the layer set over the ranks
        mine = len(range(rank, wl["layers_total"], world))
        if wl.get("max_layers_per_gpu") and mine > wl["max_layers_per_gpu"]:
            mine = wl["max_layers_per_gpu"]  # HBM cap: one GPU's share of the 8-GPU run
        if args.workload == "c4" and args.c4_layers:
            mine = min(mine, args.c4_layers)
        wl["layers"] = mine
        wl["n_files"] = wl["n_files"] * mine
    if wl.get("tar"):  # a real tar layer (C1): host-built, chunked by the product's tar walk
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        import layers
        tar = layers.LAYERS[wl["tar"]]()
        ch = nydus_gpu.tar_chunks(tar, wl["chunk"])
        buf = torch.from_numpy(np.frombuffer(tar, np.uint8).copy()).cuda()
        stride = None
    else:
        buf, ch = build_layer_on_gpu(torch, wl["n_files"], wl["file_size"], wl["chunk"],
                                     seed=0x6E79647573 + rank)
        _, stride, _, _ = synthetic_layout(1, wl["file_size"], wl["chunk"])
    n = len(ch)
    file_bytes = int(ch["length"].sum())
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    d_out = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    h_out = torch.empty(n * 64, dtype=torch.uint8, pin_memory=True)
    eng = nydus_gpu.Engine(device=local, digester=wl["digester"], chunk_size=wl["chunk"],
                           leaves_per_lane=args.lanes, timing=True,
                           flags=(SHA_MODES[args.sha_mode] << 11)
                           | ((args.load_mode + 1) << 8 if args.load_mode >= 0 else 0))
    stream = torch.cuda.Stream()
    extra = {}
    n_layers = wl["layers"]
    per_layer = n // n_layers
    planted = 0
    if wl.get("pool"):
        _, planted = plant_pool(torch, buf, ch, stride, wl, seed=rank)

    sdict = None
    if wl.get("dict_entries"):
        # digests of the layer (and of the pool) decide what gets planted in the dict
        m = wl["dict_entries"]
        g = torch.Generator(device="cuda").manual_seed(0xD1C7)
        dd = torch.empty((m, 32), dtype=torch.uint8, device="cuda")
        dd.random_(0, 256, generator=g)
        if wl.get("pool"):
            assert m >= wl["pool"]
            dd[: wl["pool"]] = pool_digests(torch, nydus_gpu, wl, local)
            expect_dict = planted
        else:
            eng.digest_device(buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n, d_out.data_ptr())
            torch.cuda.synchronize()
            k = int(n * wl["plant"])
            sel = torch.randperm(n, device="cuda", generator=g)[:k]
            rows = torch.randint(0, m, (k,), device="cuda", generator=g).unique()
            sel = sel[: rows.numel()]
            dd[rows] = d_out.view(n, 64)[sel, :32]
            expect_dict = int(rows.numel())
        us = torch.full((m,), wl["chunk"], dtype=torch.int32, device="cuda")
        bl = torch.randint(0, 8, (m,), dtype=torch.int32, device="cuda", generator=g)
        ix = torch.arange(m, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if wl.get("sharded"):
            from nydus_gpu.dist import ShardedChunkDict, engine_load_fn, engine_probe_fn
            sdict = ShardedChunkDict(rank, world,
                                     comm_device=None if args.dist_backend == "nccl" else "cpu")
            local_m = sdict.load(dd, us, bl, ix, 8, engine_load_fn(eng, 8))
            sdict.probe_fn = engine_probe_fn(eng, stream_fn=lambda: stream.cuda_stream)
        else:
            eng.dict_load_device(dd.data_ptr(), us.data_ptr(), bl.data_ptr(), ix.data_ptr(), m, 8)
            local_m = m
        torch.cuda.synchronize()
        build_s = time.perf_counter() - t0
        probe = None
        if not wl.get("sharded") and args.probe_queries:
            probe = probe_bench(torch, nydus_gpu, eng, dd, args.probe_queries, build_s)
        dict_host = None
        if wl.get("merge") and world == 1:  # the C5 Merge needs the dict bootstrap
            dict_host = (dd.cpu().numpy(), us.cpu().numpy(), bl.cpu().numpy(), ix.cpu().numpy())
        dict_file = None
        if wl.get("dict_file") and not args.no_dict_file and rank == 0:
            # ChunkDictPath itself: the same m records as a
            # RAFS v6 bootstrap on disk, opened through ngpu_dict_open (read,
            # parse, H2D, build); that dict then serves the timed steps
            dict_file = dict_from_file(torch, nydus_gpu, eng, dd, us, bl, ix, wl, args.dict_dir)
        del dd, us, bl, ix
        torch.cuda.empty_cache()
        extra["dict"] = {"entries": m, "entries_this_gpu": local_m, "build_s": round(build_s, 3),
                         "build_Mentries_s": round(local_m / build_s / 1e6, 1),
                         "expected_dict_hits": expect_dict}
        if dict_file:
            extra["dict"]["chunk_dict_path"] = dict_file
        if probe:
            extra["probe_roofline"] = probe

    layer_first = (np.arange(n_layers + 1, dtype=np.int64) * per_layer)
    d_first = torch.from_numpy(layer_first).cuda()
    d_lstats = torch.zeros(n_layers * nydus_gpu.LAYER_STATS_DTYPE.itemsize, dtype=torch.uint8,
                           device="cuda")

    # Results go back to the host on a copy stream, double-buffered: the D2H of
    # step k's result table overlaps step k+1's kernels, as in a pipeline over
    # many layers (C5-shape: a 16 MiB table, ~0.3 ms of PCIe per step).
    # A small table (C1: 7 KB) goes back on the call's own stream: the copy
    # stream's two cross-stream waits and event markers cost more than the copy.
    same_d2h = args.d2h == "same" or (args.d2h == "auto" and d_out.numel() < (1 << 20))
    d_outs = [d_out, d_out if same_d2h else torch.empty_like(d_out)]
    h_outs = [h_out, torch.empty_like(h_out).pin_memory()]
    copy_stream = torch.cuda.Stream()
    copy_done = [None, None]
    nstep = [0]

    def step():
        k = nstep[0] % 2
        nstep[0] += 1
        dout = d_outs[k]
        with torch.cuda.stream(stream):
            s = stream.cuda_stream
            if copy_done[k] is not None:  # buffer k's previous D2H must be done
                stream.wait_event(copy_done[k])
            if sdict is None and n_layers == 1:
                eng.process_device(buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n, dout.data_ptr(),
                                   stream=s)
            else:
                eng.digest_device(buf.data_ptr(), buf.numel(), d_ch.data_ptr(), n, dout.data_ptr(),
                                  stream=s)
                hits = sdict.probe(dout.view(n, 64)[:, :32]) if sdict is not None else None
                # all layers in one launch set (per-layer semantics, shared dict)
                eng.dedup_layers_device(d_ch.data_ptr(), n, dout.data_ptr(), d_first.data_ptr(),
                                        n_layers, d_lstats.data_ptr(),
                                        d_hits=hits.data_ptr() if hits is not None else 0,
                                        n_dict_blobs=8 if hits is not None else 0, stream=s)
            if same_d2h:
                h_outs[k].copy_(dout, non_blocking=True)
                return
            done = torch.cuda.Event()
            done.record(stream)
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_event(done)
            h_outs[k].copy_(dout, non_blocking=True)
            copy_done[k] = torch.cuda.Event()
            copy_done[k].record(copy_stream)

    tw = time.perf_counter()
    for _ in range(args.warmup):
        step()
    stream.synchronize()
    # Clock settle: the GPU's clocks ramp over the first ~0.5 s of load (a
    # rocprofv3 trace of 7 back-to-back C2 launches: 7.68, 6.06, 5.79, 5.66,
    # 5.57, 5.55, 5.51 ms), longer than W short steps take.  Untimed steps
    # continue until the warm-up has lasted args.settle_s; the line reports
    # them apart from W ("warmup_settle").
    settle = 0
    # (a step with a collective -- the sharded dict's probe routing -- keeps
    # every rank at the same step count, so it is never settled per rank)
    while sdict is None and time.perf_counter() - tw < args.settle_s and settle < 10000:
        step()
        settle += 1
        if settle % 8 == 0:
            stream.synchronize()
    stream.synchronize()
    extra["warmup_settle"] = {"extra_untimed_steps": settle, "warm_s": round(time.perf_counter() - tw, 3),
                              "settle_s": args.settle_s}
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()  # no host sync between steps: the engine keeps each call's events
    stream.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # correctness spot checks of the last step
    res = h_outs[(nstep[0] - 1) % 2].numpy().view(nydus_gpu.RESULT_DTYPE)
    kinds = np.bincount(res["kind"], minlength=3)
    no_load = args.load_mode == 4  # diagnostic: not BLAKE3 digests, decisions unchecked
    if not wl.get("dict_entries") and not wl.get("pool") and not wl.get("tar") and not no_load:
        assert kinds[0] == n and (res["index"] == np.arange(n)).all()
    if wl.get("dict_entries"):
        extra["dict"]["dict_hits"] = int(kinds[2])
        assert kinds[2] >= extra["dict"]["expected_dict_hits"] * 0.99, (kinds, extra)
    extra["decisions"] = {"NEW": int(kinds[0]), "INTRA": int(kinds[1]), "DICT": int(kinds[2])}
    if buf.numel() > (1 << 32) and rank == 0 and not no_load:  # digests past 2^32 (independent C/OpenSSL)
        extra["digest_check_past_4gib"] = check_high_digests(buf, ch, res, wl["digester"])
    if wl.get("merge") and world == 1 and rank == 0:
        extra["merge"] = merge_extra(nydus_gpu, ch, res, n_layers, per_layer, wl["chunk"], dict_host)

    timings = [eng.timing_at(b) for b in range(min(args.steps, 64))]
    total_bytes = file_bytes * args.steps * world
    value = total_bytes / elapsed / 1e9
    dig_all = [t["digest_ms"] for t in timings]
    dig_ms = float(np.mean(dig_all))
    tree_ms = float(np.mean([t["tree_ms"] for t in timings]))
    dedup_ms = float(np.mean([t["dedup_ms"] for t in timings]))
    D = timings[-1]["group_log2"]
    if wl["digester"] == "blake3":
        leaves = int(((ch["length"].astype(np.int64) + 1023) // 1024).sum())
        blocks = int(((ch["length"].astype(np.int64) + 63) // 64).sum())
        groups = int((((ch["length"].astype(np.int64) + 1023) // 1024 + (1 << D) - 1) >> D).sum())
        # compressions done by b3_groups: all leaf blocks + in-group parents
        comp = blocks + (leaves - groups)
        achieved = comp * OPS_PER_COMPRESSION / (dig_ms / 1e3)
        # launch_blake3's rule: one leaf per lane quad for <= 40K leaves + chunks at D = 0
        quad = D == 0 and int(buf.numel()) // 1024 + n <= 40960
        # <= 4096 chunks: planning inside the leaf kernel (b3_quad_planned)
        kname = (("b3_quad_planned" if n <= 4096 else "b3_quad_leaves") if quad
                 else f"b3_groups<{D}>")
        roof = {"bound": "valu", "kernel": kname, "achieved": round(achieved / 1e12, 3),
                "peak": round(PEAK_INT_OPS / 1e12, 3), "unit": "Tops/s",
                "frac": round(achieved / PEAK_INT_OPS, 4), "traffic": None,
                "hbm_gbs": round(file_bytes / (dig_ms / 1e3) / 1e9, 1),
                "hbm_frac": round(file_bytes / (dig_ms / 1e3) / PEAK_HBM, 4)}
        if quad and n_layers == 1:
            # A small layer fills a fraction of the lanes: its bound is the
            # longest chunk's dependency chain, not chip throughput.  16 chained
            # compressions per 1 KiB leaf, then ceil(log2 leaves) tree levels, each
            # one compress_quad (~190 dependent VALU ops per lane at ~8.5 cycles per
            # dependent op for a lone wave, profiles/r1/valu_exec_issue.jsonl), plus the call's
            # three kernel boundaries (~4.65 us each: an empty kernel's duration in
            # a rocprofv3 trace, profiles/r2/c1_trace_diag_r2dg.txt).
            lmax = int(((ch["length"].astype(np.int64) + 1023) // 1024).max())
            chain = min(16, max(1, (int(ch["length"].max()) + 63) // 64)) + (
                int(np.ceil(np.log2(lmax))) if lmax > 1 else 0)
            chain_s = chain * QUAD_COMPRESS_DEP_OPS * DEP_OP_CYCLES / CLOCK_HZ
            launch_s = 3 * KERNEL_BOUNDARY_S
            step_s = elapsed / args.steps
            lb = {
                "critical_chain_compressions": chain, "chain_ms": round(chain_s * 1e3, 4),
                "kernel_boundaries_ms": round(launch_s * 1e3, 4),
                "bound_ms": round((chain_s + launch_s) * 1e3, 4),
                "frac_of_step": round((chain_s + launch_s) / step_s, 3),
                "model": "longest chunk: leaf blocks + tree levels, x ~190 dependent ops x 8.5 "
                         "cycles at 2.4 GHz, + 3 kernel boundaries x 4.65 us"}
            # the whole step, measured in THIS run by the
            # engine's own HIP stop events (digest = b3_quad_planned incl. its
            # dispatch, tree = b3_tree, dedup = dedup_small_lds), the rest =
            # the result table's D2H (HIP runs a 7 KB same-stream copy as the
            # blit kernel __amd_rocclr_copyBuffer) + the boundary to the next
            # step; the committed kernel trace gives the same split per kernel
            med = lambda k: float(np.median([t[k] for t in timings]))
            ker = {"digest": med("digest_ms"), "tree": med("tree_ms"), "dedup": med("dedup_ms")}
            total = med("total_ms")
            dec = {"step_ms": round(step_s * 1e3, 4),
                   "kernels_ms_hip_events": {k: round(v, 4) for k, v in ker.items()},
                   "call_first_to_last_kernel_ms": round(total, 4),
                   "after_call_ms": round(step_s * 1e3 - total, 4),
                   "explained_frac_of_step": round(min(total, step_s * 1e3) / (step_s * 1e3), 3),
                   "chain_frac_of_leaf_and_tree_kernels": round(
                       chain_s * 1e3 / max(1e-9, ker["digest"] + ker["tree"]), 3)}
            tr, tsrc = newest_profile("c1_step_trace_r6ae.json")
            if tr:
                dec["trace"] = {"kernel_us": tr["kernel_us_median"], "gap_us_profiled": tr["gap_us_median"],
                                "source": tsrc,
                                "note": "rocprofv3 adds ~3-5 us to every gap; unprofiled, the "
                                        "kernels are ~90 % of the step"}
                # the call's kernels (this run's events) + the result D2H, which
                # HIP runs as the copyBuffer blit kernel (the trace's duration):
                # what is left is the four kernel boundaries of a step
                d2h = tr["kernel_us_median"].get("copyBuffer", 0.0) / 1e3
                dec["explained_with_d2h_frac_of_step"] = round(
                    min(total + d2h, step_s * 1e3) / (step_s * 1e3), 3)
                dec["boundaries_ms"] = round(max(0.0, step_s * 1e3 - total - d2h), 4)
            lb["step_decomposition"] = dec
            roof.update({"latency_bound": lb})
    else:
        blocks = int(((ch["length"].astype(np.int64) + 8) // 64 + 1).sum())
        ops = blocks * 1384  # SURVEY.md §8(d) SHA-256 op count
        achieved = ops / (dig_ms / 1e3)
        mode = args.sha_mode
        if mode == "auto":  # launch_sha256's rule
            mode = "pair" if n <= SHA_PAIR_MAX_CHUNKS else "lane"
        pair = mode.startswith("pair")
        # SHA-256 is serial within a chunk: with fewer chunks than the chip has
        # lanes, a chunk's round chain (VALU ops on its critical wave, 4 cycles
        # per wave64 op) bounds the kernel, not chip-wide VALU throughput.
        # VALU ops per block on the critical wave: pair/split round waves; the
        # lane kernel's wave does the whole block (schedule + rounds)
        chain_ops = {"pair": 66 * 9, "split": 64 * 14, "lane": 1384}[mode]
        lanes_used = n * (2 if pair else 1)
        max_blocks = int(((ch["length"].astype(np.int64) + 8) // 64 + 1).max())
        chain_s = max_blocks * chain_ops * 4 / CLOCK_HZ
        # a wave alone on its SIMD issues one VALU op per ~5 cycles, not 4
        # (tools/valu_ops.hip, profiles/r1/valu_ops_issue_rates.jsonl); the
        # round wave is alone on its SIMD by design
        lone_s = max_blocks * chain_ops * 5 / CLOCK_HZ
        roof = {"bound": "valu", "kernel": "sha256_" + mode,
                "achieved": round(achieved / 1e12, 3),
                "peak": round(PEAK_INT_OPS / 1e12, 3), "unit": "Tops/s",
                "frac": round(achieved / PEAK_INT_OPS, 4), "traffic": None,
                "hbm_gbs": round(file_bytes / (dig_ms / 1e3) / 1e9, 1),
                "chain_bound_gbs": round(file_bytes / chain_s / 1e9, 1),
                "chain_frac": round(chain_s / (dig_ms / 1e3), 4),
                "lone_wave_issue_bound_gbs": round(file_bytes / lone_s / 1e9, 1),
                "lone_wave_issue_frac": round(lone_s / (dig_ms / 1e3), 4),
                "occupancy_ceiling": f"{lanes_used} lanes = {lanes_used / (256 * 4 * 64):.3f} "
                                     "waves per SIMD"}

    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e and not wl.get("dict_entries") and stride:
        e2e = end_to_end(torch, nydus_gpu, buf, wl, stride, local, sample_bytes=args.e2e_mib << 20)
    elif rank == 0 and world == 1 and not args.no_e2e and wl.get("tar"):
        e2e = tar_host_path(nydus_gpu, tar, wl, local, file_bytes)

    roof["traffic"], roof["traffic_source"] = pmc_traffic(args.pmc_json, args.workload, roof["kernel"])
    mix_roofline(roof, achieved, roof["kernel"], args.workload,
                 comp if wl["digester"] == "blake3" else 0)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # all the CPU the process may use: the CPUs of its affinity (`nproc`),
        # capped at its cgroup CPU quota when one is set -- on the GPU box
        # `nproc` shows 256 CPUs under a 16-core quota, and 256 threads thrash
        # the quota (r2a: 33.5 GB/s against 92 at 16 threads)
        aff, quota = host_cpus()
        threads = args.cpu_threads or (min(aff, int(-(-quota // 1))) if quota else aff)
        if wl.get("tar"):
            cpu = cpu_baseline(buf.cpu().numpy(), ch, wl["digester"], threads, "whole layer:")
        else:
            sample_files = max(1, min(wl["n_files"], (args.cpu_sample_mib * MiB) // wl["file_size"]))
            host = buf[: sample_files * stride].cpu().numpy()
            per_file = (wl["file_size"] + wl["chunk"] - 1) // wl["chunk"]
            cpu = cpu_baseline(host, ch[: sample_files * per_file], wl["digester"], threads)

    line = {
        "metric": "GB/s of layer data chunk-hashed+deduped (node)",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "ranks": ranks,
        "data": ("synthetic alpine-like layer tar built on the host (tests/golden/layers.py), "
                 "copied to HBM" if wl.get("tar") else
                 "synthetic (random bytes generated on the GPU, real GNU tar headers)"),
        "config": {"workload": wl["desc"], "name": args.workload,
                   "layer_bytes": int(buf.numel()), "file_bytes_per_gpu": file_bytes, "chunks": n,
                   "chunk_size": wl["chunk"], "digester": wl["digester"], "layers_per_gpu": n_layers,
                   "leaves_per_lane": 1 << D, "parallelism": f"layer-sharded x{world}",
                   "result_d2h": "call stream" if same_d2h else "copy stream, overlapped"},
        "stage_ms": {"digest": round(dig_ms, 3), "tree": round(tree_ms, 3), "dedup": round(dedup_ms, 3),
                     "digest_min_med_max": [round(float(f(dig_all)), 3)
                                            for f in (np.min, np.median, np.max)]},
        **extra,
        "roofline": roof,
        "cpu_baseline": cpu,
        "e2e_pcie": e2e,
    }
    if args.dump_timings:
        line["timings"] = [{k: round(t[k], 3) for k in ("digest_ms", "tree_ms", "dedup_ms", "total_ms")}
                           for t in timings[::-1]]
    if cpu:
        # device-resident GPU rate (the layer already in HBM) over the all-core CPU rate
        line["speedup_vs_cpu"] = round(value / cpu["value"], 2)
        line["speedup_vs_cpu_single_stream"] = round(value / cpu["single_stream_gbs"], 2)
        if e2e:  # the same ratio once the bytes cross PCIe (never `value`)
            line["speedup_vs_cpu_pcie_inclusive"] = {
                k: round(e2e[k] / cpu["value"], 2) for k in ("host_path_gbs", "streaming_gbs")
                if k in e2e}
    dog = None
    printed = [False]
    print_mu = __import__("threading").Lock()  # the line is printed once: here or by the watchdog
    sharded_extra = dist and sdict is None and n_layers == 1 and not args.no_sharded_extra
    node_pcie = dist and stride and not wl.get("dict_entries") and not wl.get("pool") and not args.no_e2e
    node_cabi = dist and stride and not wl.get("dict_entries") and not wl.get("pool") and not args.no_node_extra
    c4x = dist and args.workload == "c2" and not args.no_c4
    if sharded_extra or node_pcie or node_cabi or c4x:
        # the headline is already measured; a watchdog keeps a stuck collective
        # (here, or in the closing barrier after a rank failed in here) from
        # costing the line: on expiry rank 0 prints it if it has not yet, and
        # every rank exits NON-ZERO, so a driver can tell a hang from a clean run
        import threading

        def stuck():
            with print_mu:
                first = rank == 0 and not printed[0]
                printed[0] = True
            if first:
                print(json.dumps(dict(line, sharded_dict={"error": "timeout"})), flush=True)
            sys.stdout.flush()
            os._exit(3)
        dog = threading.Timer((600.0 if node_cabi else 180.0) + (450.0 if c4x else 0.0), stuck)
        dog.daemon = True
        dog.start()
        if sharded_extra:
            try:
                sx = sharded_dict_extra(torch, dist, eng, buf, d_ch, n, stream, rank, world,
                                        args.dist_backend)
                sx["gbs"] = round(file_bytes * sx["steps"] * world / sx.pop("_elapsed") / 1e9, 2)
                line["sharded_dict"] = sx
            except Exception as ex:  # reported, never fatal to the headline line
                line["sharded_dict"] = {"error": f"{type(ex).__name__}: {ex}"[:300]}
        if node_pcie:
            try:
                line["e2e_pcie_node"] = node_e2e(torch, dist, nydus_gpu, buf, wl, stride, local,
                                                 args.dist_backend, min(args.e2e_mib, 1024) << 20)
            except Exception as ex:  # reported, never fatal to the headline line
                line["e2e_pcie_node"] = {"error": f"{type(ex).__name__}: {ex}"[:300]}
        if node_cabi and rank == 0:  # the other ranks wait in the closing barrier
            try:
                line["node_cabi"] = node_cabi_extra(world)
            except Exception as ex:  # reported, never fatal to the headline line
                line["node_cabi"] = {"error": f"{type(ex).__name__}: {ex}"[:300]}
            try:  # the drop-in's Pack path over every GPU of the node
                line["packs_node"] = packs_node_extra(world)
            except Exception as ex:  # reported, never fatal to the headline line
                line["packs_node"] = {"error": f"{type(ex).__name__}: {ex}"[:300]}
        if c4x and rank == 0:  # the other ranks wait in the closing barrier
            try:
                line["c4"] = c4_entry(world, args.c4_layers, max(3, min(args.steps, 10)),
                                      args.dist_backend)
            except Exception as ex:  # reported, never fatal to the headline line
                line["c4"] = {"error": f"{type(ex).__name__}: {ex}"[:300]}
    if rank == 0 and world == 1 and args.workload == "c2" and not args.no_sub:
        line.update(sub_entries(args))
    mg = None
    if rank == 0 and dist:
        line["multi_gpu_checks"] = mg = multi_gpu_checks(line)
    if rank == 0:
        bad = fracs_over_one(line)
        if bad:  # printed, never hidden: a frac > 1 means a wrong model or clock
            line["fracs_over_one"] = bad
    if rank == 0:
        with print_mu:
            first = not printed[0]
            printed[0] = True
        if first:
            print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.barrier(group=cpu_group)
        dist.destroy_process_group()
    if dog:
        dog.cancel()
    exit_on_failed_checks(mg)


if __name__ == "__main__":
    main()
