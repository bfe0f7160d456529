"""Multi-rank chunk-dict partition + all-to-all probe routing on CPU (gloo,
world_size 2/4/8).  The local probe is a plain first-occurrence map and the
owner bucketing a plain torch restatement of ngpu_route_digests /
ngpu_route_hits (TorchRouter, test infrastructure): the host logic under
test is the partition, the split agreement, the exchange and the ordering.
The GPU kernels behind the product router are checked against TorchRouter in
tests/test_gpu_node.py::test_route_kernels_match_the_reference_router."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nydus_gpu.dist import HIT_WORDS, ShardedChunkDict, owner_of


class TorchRouter:
    """CPU restatement of the routing kernels (test infrastructure only):
    compact owner order (stable) or [rounds][world][seg_cap] padded slots."""

    def route(self, digests, world, seg_cap=0, rounds=0):
        n = digests.shape[0]
        own = owner_of(digests, world)
        order = torch.argsort(own, stable=True)
        counts = torch.bincount(own, minlength=world).to(torch.int32)
        if not seg_cap:
            return digests[order].contiguous(), order.to(torch.int32), counts
        slots = rounds * world * seg_cap
        out = torch.zeros((slots, 32), dtype=torch.uint8)
        rows = torch.full((slots,), -1, dtype=torch.int32)
        start = torch.cumsum(counts.to(torch.int64), 0) - counts.to(torch.int64)
        own_s = own[order]
        k = torch.arange(n) - start[own_s]
        pos = (k // seg_cap) * world * seg_cap + own_s * seg_cap + k % seg_cap
        out[pos] = digests[order]
        rows[pos] = order.to(torch.int32)
        return out, rows, counts

    def scatter(self, routed, rows, n, hits=None):
        if hits is None:
            hits = torch.empty((n, HIT_WORDS), dtype=torch.int32)
        keep = rows >= 0
        hits[rows[keep].to(torch.int64)] = routed[keep]
        return hits


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
        sd = ShardedChunkDict(rank, world, cap=cap, router=TorchRouter())
        local = {}

        def load(dd, uu, bb, ii, uo, gid):
            # the partition keeps global table order and answers with GLOBAL
            # ids (ngpu_dict_create_device_gid)
            assert bool((gid[1:] > gid[:-1]).all()) if gid.numel() > 1 else True
            for k in range(dd.shape[0]):
                local.setdefault(dd[k].numpy().tobytes(),
                                 (int(gid[k]), int(ii[k]), int(bb[k]), int(uu[k]),
                                  int(uo[k]) & 0xFFFFFFFF, int(uo[k]) >> 32))

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


def test_product_router_refuses_host_tensors():
    """The product router is the GPU kernel pair: host tensors are an error,
    never a CPU fallback."""
    from nydus_gpu.dist import HipRouter
    with pytest.raises(ValueError, match="CUDA"):
        HipRouter().route(torch.zeros((4, 32), dtype=torch.uint8), 2)


def test_reference_router_layouts():
    """TorchRouter (the CPU statement the GPU kernels are checked against):
    compact layout = stable owner order with counts; padded layout puts row k
    of owner o at [k // cap][o][k % cap]."""
    g = torch.Generator().manual_seed(5)
    d = torch.randint(0, 256, (300, 32), dtype=torch.uint8, generator=g)
    r = TorchRouter()
    out, rows, counts = r.route(d, 4)
    own = owner_of(d, 4)
    assert counts.tolist() == torch.bincount(own, minlength=4).tolist()
    assert torch.equal(out, d[rows.to(torch.int64)])
    assert bool((owner_of(out, 4)[1:] >= owner_of(out, 4)[:-1]).all())
    out, rows, counts = r.route(d, 4, seg_cap=32, rounds=-(-300 // 32))
    for slot in range(rows.numel()):
        if rows[slot] >= 0:
            o = (slot // 32) % 4
            assert owner_of(d[rows[slot].item()][None], 4).item() == o
            assert torch.equal(out[slot], d[rows[slot].item()])
        else:
            assert not out[slot].any()
    assert sorted(rows[rows >= 0].tolist()) == list(range(300))


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
