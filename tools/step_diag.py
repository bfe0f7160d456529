#!/usr/bin/env python3
"""Diagnostic for ngpu_node_process_step on a W-part node of device 0: per
part, zero digests, kinds and each engine's device_status after a step, with
the stream/slot layout varied.  usage: tools/step_diag.py W [same_stream]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "nydus-snapshotter_amd")):
    sys.path.insert(0, p)


def main():
    import torch
    import nydus_gpu
    import oracle_py as oracle
    from nydus_gpu import rafs
    from test_gpu_node import _dict_records, _layer, _to_dev
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    same = len(sys.argv) > 2 and sys.argv[2] == "same"
    rng = np.random.default_rng(900 + W)
    cs = 0x10000
    row = []
    for i in range(W):
        k = 0 if i == W - 1 else int(rng.integers(1, 4))
        row.append([_layer(rng, int(rng.integers(2, 7)) << 20, cs) for _ in range(k)])
    digs = [[oracle.digest_chunks(d, c.view(oracle.CHUNK_DTYPE), "blake3") for d, c in ls] for ls in row]
    recs = _dict_records(rng, np.concatenate([x for ds in digs for x in ds]),
                         np.concatenate([c["length"] for ls in row for _, c in ls]))
    node = nydus_gpu.Node([0] * W, chunk_size=cs)
    d = node.dict_create(recs, rafs.make_blob_table([f"{i:064x}" for i in range(7)], cs))
    s0 = torch.cuda.Stream()
    streams = [s0 if same else torch.cuda.Stream() for _ in range(W)]
    args, keep = [], []
    for i in range(W):
        ls = row[i]
        if not ls:
            args.append({"n": 0, "stream": streams[i].cuda_stream})
            continue
        base, bufs, chs, first = 0, [], [], [0]
        for data, ch in ls:
            c = ch.copy()
            c["offset"] += base
            bufs.append(np.frombuffer(data, np.uint8))
            chs.append(c)
            base += len(data)
            first.append(first[-1] + len(ch))
        buf, ch = np.concatenate(bufs), np.concatenate(chs)
        d_data, d_ch, d_first = _to_dev(buf), _to_dev(ch), _to_dev(np.array(first, np.uint64))
        out = torch.zeros(len(ch) * 64, dtype=torch.uint8, device="cuda")
        keep.append((d_data, d_ch, d_first, out))
        args.append({"d_data": d_data.data_ptr(), "len": d_data.numel(), "d_chunks": d_ch.data_ptr(),
                     "n": len(ch), "d_out": out.data_ptr(), "d_layer_first": d_first.data_ptr(),
                     "n_layers": len(ls), "stream": streams[i].cuda_stream, "_out": out, "_first": first})
    torch.cuda.synchronize()
    for rep in range(2):
        for a in args:
            if "_out" in a:
                a["_out"].zero_()
        torch.cuda.synchronize()
        node.process_step(d, args)
        torch.cuda.synchronize()
        for i in range(W):
            a = args[i]
            st = "ok"
            try:
                node.engines[i].device_status()
            except nydus_gpu.NgpuError as e:
                st = str(e)
            if "_out" not in a:
                print(f"rep {rep} part {i}: empty; status {st}")
                continue
            got = a["_out"].cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
            ref = np.concatenate(digs[i])
            zero = int((got["digest"] == 0).all(axis=1).sum())
            eq = int((got["digest"] == ref).all(axis=1).sum())
            kinds = np.bincount(got["kind"], minlength=5).tolist()
            print(f"rep {rep} part {i}: n {a['n']} layers {len(row[i])} len {a['len']} zero {zero} "
                  f"equal {eq} kinds {kinds} status {st}", flush=True)
    # each part alone: the engine's own digest_device and node.process_device
    for i in range(W):
        a = args[i]
        if "_out" not in a:
            continue
        ref = np.concatenate(digs[i])
        for how in ("digest_device", "process_device"):
            a["_out"].zero_()
            torch.cuda.synchronize()
            if how == "digest_device":
                node.engines[i].digest_device(a["d_data"], a["len"], a["d_chunks"], a["n"], a["d_out"],
                                              stream=streams[i].cuda_stream)
            else:
                node.process_device(i, d, a["d_data"], a["len"], a["d_chunks"], a["n"], a["d_out"],
                                    a["d_layer_first"], a["n_layers"], stream=streams[i].cuda_stream)
            torch.cuda.synchronize()
            got = a["_out"].cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
            st = "ok"
            try:
                node.engines[i].device_status()
            except nydus_gpu.NgpuError as e:
                st = str(e)
            print(f"{how} part {i}: zero {int((got['digest'] == 0).all(axis=1).sum())} equal "
                  f"{int((got['digest'] == ref).all(axis=1).sum())} of {a['n']} status {st}", flush=True)
    node.close()


if __name__ == "__main__":
    main()
