#!/usr/bin/env python3
"""Chunk-dict probe by dict size: where do the probe's extra line requests
come from (2.14 lines per probe against ~1.55 for query +
slot + record)?  For each dict size, a dict of random 32-B digests is built on
the GPU (ngpu_dict_load_device), then Q queries (30 % planted) are probed
(dict_probe_records through ngpu_dict_probe_device), timed with HIP events.
Under `rocprofv3 --pmc TCC_EA0_RDREQ_*` the launches of each size are told
apart by their order (one warm + REPS timed launches per size, sizes in
order).  usage: tools/probe_sweep.py [Q_M] [SIZES_M,...]  -> JSON lines"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nydus-snapshotter_amd"))


def main():
    import torch
    import nydus_gpu
    Q = int(sys.argv[1] if len(sys.argv) > 1 else 16) << 20
    sizes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,16,64,200").split(",")]
    reps = 5
    eng = nydus_gpu.Engine(device=0, digester="sha256")
    g = torch.Generator(device="cuda").manual_seed(0x9B0B)
    for mm in sizes:
        m = mm * 1_000_000
        dd = torch.empty((m, 32), dtype=torch.uint8, device="cuda")
        dd.random_(0, 256, generator=g)
        us = torch.full((m,), 1 << 20, dtype=torch.int32, device="cuda")
        bl = torch.zeros(m, dtype=torch.int32, device="cuda")
        ix = torch.arange(m, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()  # the build reads the arrays from its own stream
        eng.dict_load_device(dd.data_ptr(), us.data_ptr(), bl.data_ptr(), ix.data_ptr(), m, 1)
        q = torch.empty((Q, 32), dtype=torch.uint8, device="cuda")
        q.random_(0, 256, generator=g)
        k = int(Q * 0.3)
        q[:k] = dd[torch.randint(0, m, (k,), device="cuda", generator=g)]
        q = q[torch.randperm(Q, device="cuda", generator=g)].contiguous()
        hits = torch.empty((Q, 6), dtype=torch.int32, device="cuda")
        s = torch.cuda.current_stream()
        eng.dict_probe_device(q.data_ptr(), 32, Q, hits.data_ptr(), stream=s.cuda_stream)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record(s)
        for r in range(reps):
            eng.dict_probe_device(q.data_ptr(), 32, Q, hits.data_ptr(), stream=s.cuda_stream)
            ev[r + 1].record(s)
        torch.cuda.synchronize()
        ms = sorted(ev[r].elapsed_time(ev[r + 1]) for r in range(reps))[reps // 2]
        nhit = int((hits[:, 0] != -1).sum())
        table_bytes = 1
        while table_bytes < 2 * m + 16:
            table_bytes *= 2
        print(json.dumps({"dict_entries": m, "queries": Q, "hits": nhit, "ms": round(ms, 4),
                          "gprobes_s": round(Q / ms / 1e6, 2), "launches": reps + 1,
                          "table_bytes": table_bytes * 8, "record_bytes": m * 64}), flush=True)
        eng.dict_clear()
        del dd, us, bl, ix, q, hits
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
