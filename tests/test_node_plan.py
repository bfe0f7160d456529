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
