"""bench.py's synthetic layer layout equals what the real tar front end
produces on the same bytes (small instance, CPU only)."""
import io
import os
import tarfile

import numpy as np
import pytest

import bench
import nydus_gpu


def test_synthetic_layout_matches_parser():
    h, stride, total, ch = bench.synthetic_layout(5, 3 * 1024 * 1024 + 100, 1 << 20)
    buf = np.zeros(total, np.uint8)
    rng = np.random.default_rng(0)
    for i in range(5):
        buf[i * stride:i * stride + 512] = h[i]
        buf[i * stride + 512:i * stride + 512 + 3 * 1024 * 1024 + 100] = rng.integers(0, 256, 3 * 1024 * 1024 + 100)
    got = nydus_gpu.tar_chunks(buf, 1 << 20)
    assert got.tobytes() == ch.tobytes()
    names = [m.name for m in tarfile.open(fileobj=io.BytesIO(buf.tobytes())).getmembers()]
    assert len(names) == 5


def test_pool_content_is_a_function_of_the_id():
    """C4/C5 pool contents are regenerated per batch on every rank: content i
    must not depend on which batch (or rank) produced it, and distinct ids
    must give distinct contents."""
    import torch
    S = 4096
    a = bench.pool_content(torch, torch.arange(0, 8), S, device="cpu")
    b = bench.pool_content(torch, torch.tensor([5, 3, 7]), S, device="cpu")
    assert a.shape == (8, S) and a.dtype == torch.uint8
    assert torch.equal(a[5], b[0]) and torch.equal(a[3], b[1]) and torch.equal(a[7], b[2])
    assert len({bytes(r.numpy()) for r in a}) == 8
    # bytes look uniform (no constant high bytes from the shifts)
    counts = np.bincount(a.numpy().ravel(), minlength=256)
    assert counts.min() > 0.5 * counts.mean()


def test_merge_extra_on_oracle_decisions():
    """bench.merge_extra (C5's host Merge): per-layer bootstraps built from
    dedup decisions, merged against the dict bootstrap -> every layer's own
    blob plus exactly the dict blobs the layers hit.  Decisions come from the
    CPU oracle (no GPU), three layers of 12 chunks."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(bench.__file__), "oracle"))
    import oracle_py
    S, P, L = 4096, 12, 3
    rng = np.random.default_rng(4)
    m = 50
    dg = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    us = np.full(m, S, np.int32)
    bl = (np.arange(m) % 3).astype(np.int32)  # dict blobs 0..2
    ix = np.arange(m, dtype=np.int32)
    ch = np.zeros(P * L, nydus_gpu.CHUNK_DTYPE)
    ch["length"] = S
    ch["offset"] = np.arange(P * L, dtype=np.uint64) * S
    ch["file_offset"] = (np.arange(P * L) % P) * S
    res = np.zeros(P * L, nydus_gpu.RESULT_DTYPE)
    for l in range(L):
        dig = rng.integers(0, 256, (P, 32), dtype=np.uint8)
        dig[0] = dg[l]          # a dict hit on blob l % 3
        dig[5] = dg[3 + l]      # another one
        dig[7] = dig[6]         # INTRA
        dec, _ = oracle_py.dedup(dig, ch["length"][:P], dg, us.view(np.uint32), bl.view(np.uint32),
                                 ix.view(np.uint32))
        sl = slice(l * P, (l + 1) * P)
        for f in ("kind", "index", "ref", "blob_index", "uncompressed_offset"):
            res[f][sl] = dec[f]
        res["digest"][sl] = dig
        res["dict_blob"][sl] = np.where(dec["kind"] == nydus_gpu.DICT, bl[np.minimum(dec["ref"], m - 1)], 0)
    out = bench.merge_extra(nydus_gpu, ch, res, L, P, S, (dg, us, bl, ix))
    hit_blobs = {int(bl[l]) for l in range(L)} | {int(bl[3 + l]) for l in range(L)}
    assert out["own_blobs"] == L
    assert out["dict_blobs"] == len(hit_blobs)
    assert out["layers"] == L and out["merged_bytes"] > 0


def test_gpus_n_self_launches_n_ranks_before_any_gpu_call():
    """`python bench.py --gpus N` (no WORLD_SIZE) becomes a child torchrun of N
    ranks with every argument passed through; the parent
    only relays the child's status.  The spawn is stubbed here."""
    import argparse
    seen = {}

    def runner(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    argv = ["--gpus", "2", "--dist-backend", "gloo", "--workload", "c1", "--steps", "3", "--no-sub"]
    args = argparse.Namespace(gpus=2, node="")
    env = {"PATH": "/usr/bin", "RANK": "3", "MASTER_PORT": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    assert bench.maybe_self_launch(args, argv, env=env, runner=runner) == 7
    cmd, cenv = seen["cmd"], seen["env"]
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and "--nnodes=1" in cmd and "--nproc-per-node=2" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    j = [k for k, c in enumerate(cmd) if c.endswith("bench.py")][0]
    assert cmd[j + 1:] == argv  # passed through unchanged, --gpus included
    assert "RANK" not in cenv and "MASTER_PORT" not in cenv
    assert cenv["NYDUS_BENCH_LAUNCHER"] == "self" and cenv["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # a rank (WORLD_SIZE set by the launcher), N = 1 and --node never relaunch
    seen.clear()
    assert bench.maybe_self_launch(args, argv, env={"WORLD_SIZE": "2"}, runner=runner) is None
    assert bench.maybe_self_launch(argparse.Namespace(gpus=1, node=""), [], env={},
                                   runner=runner) is None
    assert bench.maybe_self_launch(argparse.Namespace(gpus=2, node="0,0"), [], env={},
                                   runner=runner) is None
    assert not seen


def test_rank_check_refuses_a_world_other_than_gpus():
    import argparse

    class FakeTorch:
        class cuda:
            @staticmethod
            def get_device_properties(i):
                raise RuntimeError("no GPU here")
    args = argparse.Namespace(gpus=2)
    with pytest.raises(SystemExit) as ex:
        bench.rank_check(args, None, 1, 0, 0, "nccl", FakeTorch)
    assert ex.value.code == 4
    r = bench.rank_check(argparse.Namespace(gpus=1), None, 1, 0, 0, "nccl", FakeTorch)
    assert r["world_size"] == 1 and r["distinct_devices"] == 1 and r["rccl_world_size"] is None


def test_packs_drive_harness_loads_and_checks_its_arguments():
    """bench.py --packs's native caller (tools/packs_drive.cpp ->
    build/libpacks_drive.so): it loads beside libnydusgpu.so, exports
    packs_drive, and refuses a null engine or empty layer set before any HIP
    call (no GPU here)."""
    import ctypes
    from conftest import ROOT
    path = os.path.join(ROOT, "nydus-snapshotter_amd", "build", "libpacks_drive.so")
    assert os.path.exists(path), "run `make -C nydus-snapshotter_amd`"
    drive = ctypes.CDLL(path).packs_drive
    drive.restype = ctypes.c_int
    rs = (ctypes.c_double * 1)()
    per = (ctypes.c_uint64 * 4)()
    null = ctypes.c_void_p()
    assert drive(null, 1, null, null, ctypes.c_uint64(1 << 20), 0, 0, 0x100000, 1, rs, per, None,
                 None, ctypes.c_uint64(0), null, None) == -1  # NGPU_EINVAL: no engine, no node
    assert drive(ctypes.c_void_p(1), 0, null, null, ctypes.c_uint64(1 << 20), 0, 0, 0x100000, 1, rs,
                 per, None, None, ctypes.c_uint64(0), null, None) == -1


def test_multi_gpu_checks_summary_and_exit():
    """an N > 1 line gathers every hit-equality check in
    `multi_gpu_checks`; a False check makes the run exit 4 after printing,
    entries that failed to run are listed as errors, not as wrong exchanges."""
    line = {"sharded_dict": {"hits_ok": True},
            "node_cabi": {"hits_equal": True,
                          "node_step": {"copy": {"hits_equal_partition": True},
                                        "rccl": {"error": "NGPU_EUNSUPP"}}},
            "c4": {"dict": {"dict_hits": 995, "expected_dict_hits": 1000}}}
    mg = bench.multi_gpu_checks(line)
    assert mg["ok"] and set(mg["checks"]) == {
        "sharded_dict.hits_ok", "node_cabi.routed_copy_replicate.hits_equal",
        "node_cabi.node_step.copy.hits_equal", "c4.dict_hits"}
    assert mg["errors"] == {"node_cabi.node_step.rccl": "NGPU_EUNSUPP"}
    bench.exit_on_failed_checks(mg)  # returns
    bench.exit_on_failed_checks(None)
    line["node_cabi"]["node_step"]["copy"]["hits_equal_partition"] = False
    mg = bench.multi_gpu_checks(line)
    assert not mg["ok"]
    with pytest.raises(SystemExit) as ex:
        bench.exit_on_failed_checks(mg)
    assert ex.value.code == 4
    assert not bench.multi_gpu_checks({"sharded_dict": {"hits_ok": False}})["ok"]
    assert bench.multi_gpu_checks({"c4": {"error": "timeout"}}) == {
        "checks": {}, "errors": {"c4": "timeout"}, "ok": True}
    # the drop-in's Packs over the node: placement follows load, so an uneven
    # split passes; a part without Packs, or a lost chunk, fails the run
    assert bench.multi_gpu_checks({"packs_node": {"placement_even": False, "placement_all_parts": True,
                                                  "chunks_ok": True}})["ok"]
    assert not bench.multi_gpu_checks({"packs_node": {"placement_all_parts": False, "chunks_ok": True}})["ok"]
    assert not bench.multi_gpu_checks({"packs_node": {"placement_all_parts": True, "chunks_ok": False}})["ok"]


def test_fracs_over_one_are_listed():
    """the line names every frac above 1 (none expected)."""
    line = {"roofline": {"frac": 0.93, "frac_mix": 0.99, "mix": {"frac": 1.2}},
            "c3": {"probe_roofline": {"traffic_frac": 1.01}}, "x": [{"frac": 2}]}
    assert sorted(bench.fracs_over_one(line)) == ["c3.probe_roofline.traffic_frac", "roofline.mix.frac",
                                                 "x[0].frac"]
    assert bench.fracs_over_one({"roofline": {"frac": 1.0}}) == []
