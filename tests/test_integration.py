"""The Go drop-in is committed as source (integration/go):
the converter patch applies to the reference tree, and the cgo package binds
only entry points include/nydus_gpu.h declares.  No Go toolchain here: the
Go files are checked as text."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

REF = "/root/reference"
GO = os.path.join(ROOT, "integration", "go")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "pkg", "converter")),
                    reason="reference tree not present (GPU box)")
def test_converter_patch_applies_to_the_reference(tmp_path):
    for f in ("pkg/converter/types.go", "pkg/converter/convert_unix.go", "pkg/converter/tool/builder.go"):
        os.makedirs(tmp_path / os.path.dirname(f), exist_ok=True)
        shutil.copy(os.path.join(REF, f), tmp_path / f)
    subprocess.check_call(["git", "init", "-q", str(tmp_path)])
    subprocess.check_call(["git", "-C", str(tmp_path), "apply", "-p1",
                           os.path.join(GO, "converter.patch")])
    pack = (tmp_path / "pkg/converter/convert_unix.go").read_text()
    assert "return packGPU(ctx, dest, opt)" in pack and "mergeGPUFiles(" in pack
    assert "return unpackGPU(ra, dest)" in pack
    assert 'args = append(args, "--digester", option.Digester)' in \
        (tmp_path / "pkg/converter/tool/builder.go").read_text()


def test_cgo_binds_only_declared_entry_points():
    header = open(os.path.join(ROOT, "include", "nydus_gpu.h")).read()
    declared = set(re.findall(r"\b(ngpu_\w+)\b", header))  # functions and function types
    consts = set(re.findall(r"\b(NGPU_\w+)\b", header))
    src = open(os.path.join(GO, "pkg", "gpu", "gpu.go")).read()
    used = set(re.findall(r"\bC\.(ngpu_\w+)\(", src))
    assert used and used <= declared, used - declared
    for c in set(re.findall(r"\bC\.(NGPU_\w+)\b", src)):
        assert c in consts, c
    glue = open(os.path.join(GO, "pkg", "converter", "convert_gpu_unix.go")).read()
    for fn in ("func useGPU(", "func packGPU(", "func mergeGPUFiles(", "func unpackGPU("):
        assert fn in glue
