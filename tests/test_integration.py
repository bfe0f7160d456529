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


def test_go_drop_in_shards_over_the_node_and_releases_on_every_path():
    """VERDICT r5 item 1, checked as text (no Go toolchain): the Go branch
    packs on a process-wide node (least-loaded engine per Pack, the C++ mirror
    runs the same logic on the GPU in tests/test_gpu_node.py), ChunkDictPath is
    a replicated node dict, and every path that never reaches Close releases
    the Pack: a source error in ReadFrom, ctx.Done() (AfterFunc aborts under
    the pack mutex) and a finalizer; targz-ref merges stay in-process."""
    src = open(os.path.join(GO, "pkg", "gpu", "gpu.go")).read()
    glue = open(os.path.join(GO, "pkg", "converter", "convert_gpu_unix.go")).read()
    patch = open(os.path.join(GO, "converter.patch")).read()
    assert "C.ngpu_node_pack_open(" in src and "func (nd *Node) Pack(" in src
    assert "gpu.NewNode(gpuDevices()" in glue and "nd.Pack(ctx" in glue
    assert "nd.OpenChunkDict(opt.ChunkDictPath, false)" in glue
    read_from = src[src.index("func (w *PackWriter) ReadFrom("):src.index("func (w *PackWriter) Close(")]
    # the source-error branch ends the pack
    tail = read_from[read_from.index("if err == io.EOF"):]
    assert "s.end(true)" in tail
    after = src[src.index("context.AfterFunc(ctx"):src.index("r, pw, err := os.Pipe()")]
    assert "s.mu.Lock()" in after and "s.end(true)" in after
    assert "runtime.SetFinalizer(w, func" in src and "runtime.SetFinalizer(w, nil)" in src
    assert "C.ngpu_merge_ex2(" in src and "rafsBlobDigests, rafsBlobSizes, rafsBlobTOCDigests)" in patch
    assert "len(rafsBlobDigests) == 0" not in patch
