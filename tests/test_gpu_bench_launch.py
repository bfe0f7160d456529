"""`python bench.py --gpus 2` on the one-GPU box: the bench launches its own
two ranks (no torchrun around it), both join a world of 2 over gloo, and rank
0 prints one line with n_gpus 2.  RCCL refuses two ranks
on one GPU, so the box rehearses the launch over gloo; the driver's node
runs the same path with nccl."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(200)
def test_bench_gpus_2_self_launches_two_ranks():
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--workload", "c1", "--steps", "3", "--no-sub", "--settle-s", "0.2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    rk = d["ranks"]
    assert rk["world_size"] == 2 and rk["requested"] == 2 and rk["launcher"] == "self"
    assert rk["backend"] == "gloo" and rk["distinct_devices"] >= 1
    sd = d["sharded_dict"]  # the gloo-routed partitioned dict ran on both ranks
    assert "error" not in sd, sd
    # every planted digest hits (the C1 layer repeats chunks, so more may)
    assert sd["dict_hits_all_ranks"] >= sd["planted_all_ranks"] > 0, sd


@pytest.mark.gpu
@pytest.mark.timeout(200)
def test_bench_packs_over_a_node_reports_placement_and_every_chunk():
    """The child command of an N > 1 line's `packs_node` entry (bench.py
    packs_node_extra) on a 2-part node of device 0: every part gets Packs and
    every chunk of the round comes back (the two checks multi_gpu_checks
    holds it to; the split itself follows load)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c1", "--packs", "8",
           "--node", "0,0", "--packs-modes", "decisions", "--no-cpu-baseline", "--steps", "3",
           "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    m = json.loads(lines[-1])["modes"]["decisions"]
    placed = m["packs_per_node_part_last_round"]
    assert len(placed) == 2 and sum(placed) == 8 and min(placed) > 0, placed
    assert sum(m["decisions_last_round"].values()) == m["chunks_per_round"] > 0, m
