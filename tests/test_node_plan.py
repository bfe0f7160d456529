"""The node step's all-to-all arguments (csrc/a2a_plan.hpp) on the CPU: the
padded layout's counts / displacements under ncclAllToAllv's semantics and
the peer-copy transport's, W = 1..8 with skewed counts and empty parts
(tests/cpp/a2a_plan_test.cpp, g++ with ASan/UBSan; no GPU, no RCCL)."""
import os
import subprocess

from conftest import ROOT


def test_node_step_alltoall_args_agree_with_peer_copies(tmp_path):
    exe = str(tmp_path / "a2a_plan_test")
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all",
                           "-I", os.path.join(ROOT, "nydus-snapshotter_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "a2a_plan_test.cpp"), "-o", exe])
    for seed in ("1", "2", "3"):
        out = subprocess.check_output([exe, seed], text=True, timeout=120)
        assert out.startswith("ok 120"), out


def test_batch_lane_table_under_tsan(tmp_path):
    """The batcher's lane table (csrc/batch_lanes.hpp; csrc/batch.hip) under
    ThreadSanitizer: 400 batches on 4 lanes, each ended by 5 packs coming
    back from their own threads in random order; no lane is taken twice, every
    batch frees its lane once, and late reports of old batches free nothing
    (tests/cpp/batch_lanes_test.cpp; no GPU)."""
    exe = str(tmp_path / "batch_lanes_test")
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-fsanitize=thread",
                           "-I", os.path.join(ROOT, "nydus-snapshotter_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "batch_lanes_test.cpp"), "-o", exe,
                           "-lpthread"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    for seed in ("1", "2", "3"):
        r = subprocess.run([exe, seed], capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, r.stdout + r.stderr[-3000:]
        assert r.stdout.startswith("ok 400"), r.stdout
