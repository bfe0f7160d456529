"""Multi-rank chunk-dict partition + all-to-all probe routing on CPU (gloo,
world_size 2).  The local probe is a plain first-occurrence map here (host
logic under test: partitioning, owner routing, id translation, ordering);
the GPU probe behind it is covered by tests/test_gpu_parity.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nydus_gpu.dist import ShardedChunkDict, owner_of


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_dict(seed=3, m=5000):
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    d[100:150] = d[10:60]           # duplicate keys: first entry must win
    us = rng.integers(1, 1 << 20, m).astype(np.int32)
    bl = rng.integers(0, 5, m).astype(np.int32)
    ix = np.arange(m, dtype=np.int32) * 3
    return d, us, bl, ix


def _queries(rank, d, nq=700):
    rng = np.random.default_rng(100 + rank)
    q = rng.integers(0, 256, (max(nq, 700), 32), dtype=np.uint8)
    pick = rng.choice(len(d), 500)
    q[:500] = d[pick]
    q[600:650] = d[100:150]        # duplicated dict keys
    return q[:nq]


def _expected(d, us, bl, ix, q):
    first = {}
    for i, row in enumerate(d):
        first.setdefault(row.tobytes(), i)
    out = np.zeros((len(q), 6), np.int64)
    for i, row in enumerate(q):
        e = first.get(row.tobytes(), -1)
        out[i] = (e, ix[e], bl[e], us[e], 4096 * e, 0) if e >= 0 else (-1, 0, 0, 0, 0, 0)
    return out


def _worker(rank, world, port, ret, cap=0, nq=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d, us, bl, ix = _global_dict()
        sd = ShardedChunkDict(rank, world, cap=cap)
        local = {}

        def load(dd, uu, bb, ii, uo):
            for k in range(dd.shape[0]):
                local.setdefault(dd[k].numpy().tobytes(),
                                 (k, int(ii[k]), int(bb[k]), int(uu[k]), int(uo[k]) & 0xFFFFFFFF,
                                  int(uo[k]) >> 32))

        uoff = torch.arange(len(d), dtype=torch.int64) * 4096
        n_local = sd.load(torch.from_numpy(d), torch.from_numpy(us), torch.from_numpy(bl),
                          torch.from_numpy(ix), 5, load, uoff=uoff)

        def probe(q):
            out = torch.zeros((q.shape[0], 6), dtype=torch.int32)
            out[:, 0] = -1
            for k in range(q.shape[0]):
                h = local.get(q[k].numpy().tobytes())
                if h:
                    out[k] = torch.tensor(h, dtype=torch.int32)
            return out

        sd.probe_fn = probe
        q = _queries(rank, d, nq[rank] if nq else 700)
        got = sd.probe(torch.from_numpy(q)).numpy().astype(np.int64)
        exp = _expected(d, us, bl, ix, q)
        ret[rank] = (bool((got == exp).all()), n_local)
    finally:
        dist.destroy_process_group()


def test_owner_is_prefix():
    d = torch.zeros((4, 32), dtype=torch.uint8)
    d[:, 0] = torch.tensor([0, 0x7F, 0x80, 0xFF], dtype=torch.uint8)
    assert owner_of(d, 2).tolist() == [0, 0, 1, 1]
    assert owner_of(d, 8).tolist() == [0, 3, 4, 7]


@pytest.mark.timeout(180)
@pytest.mark.parametrize("cap", [0, 700, 1024])
def test_sharded_dict_two_ranks(cap):
    """cap 0: variable splits sized on the host; cap >= queries: equal padded
    splits, no host sync (ShardedChunkDict._probe_equal)."""
    world = 2
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret, cap), nprocs=world, join=True)
    assert ret[0][0] and ret[1][0]
    assert ret[0][1] + ret[1][1] == 5000  # the partition covers the dict exactly once


@pytest.mark.timeout(180)
def test_sharded_dict_four_ranks_equal_splits():
    """Four owners, equal padded splits: every rank's hits equal the whole
    dict's first-occurrence answers."""
    world = 4
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret, 700), nprocs=world, join=True)
    assert all(ret[r][0] for r in range(world))
    assert sum(ret[r][1] for r in range(world)) == 5000


@pytest.mark.timeout(180)
def test_equal_splits_overflow_runs_extra_rounds_together():
    """a rank with more queries than cap used to raise before the
    collective while the others blocked in it.  Now the ranks agree on the
    round count first (host all-reduce) and every query is answered: rank 1
    has 700 queries at cap 128 (6 rounds), rank 0 only 90."""
    world = 2
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret, 128, [90, 700]), nprocs=world, join=True)
    assert ret[0][0] and ret[1][0]


@pytest.mark.timeout(240)
@pytest.mark.parametrize("cap,nq", [(0, None), (96, [40, 300, 0, 96, 97, 500, 1, 250])])
def test_sharded_dict_eight_ranks(cap, nq):
    """The driver's node size, rehearsed on the CPU (gloo, 8 ranks): variable
    splits, and equal padded splits where the ranks' query counts differ
    (one empty, some past cap: extra rounds agreed on the host); every rank's
    hits equal the whole dict's first-occurrence answers and the partition
    covers the dict once."""
    world = 8
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret, cap, nq), nprocs=world, join=True)
    assert all(ret[r][0] for r in range(world))
    assert sum(ret[r][1] for r in range(world)) == 5000
