"""GPU: a short run of the soak (scripts/gpu_soak.py) inside the suite --
random layer tars (edge file sizes, 4 KiB .. 4 MiB chunks, both digesters,
every lanes setting, the grid flag) through ngpu_pack_tar and the streaming
Pack, then four threads on shared engines (pack_tar, streaming Packs with and
without a chunk dict, device calls on per-thread streams, Packs through a
4-part node against a partitioned dict).  Every digest and decision is
checked against the CPU oracle."""
import importlib.util
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _soak():
    spec = importlib.util.spec_from_file_location("gpu_soak", os.path.join(ROOT, "scripts", "gpu_soak.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_soak_sequential(monkeypatch, capsys):
    m = _soak()
    monkeypatch.setattr("sys.argv", ["gpu_soak.py", "40", "4242"])
    m.main()
    assert '"soak": "ok"' in capsys.readouterr().out


def test_soak_threads(capsys):
    m = _soak()
    m.concurrent(4, 15, 4243)  # exits non-zero (SystemExit) on any mismatch
    assert '"soak": "ok"' in capsys.readouterr().out
