"""Diagnostic: an empty pack's layer stats after failed / aborted packs on
the same engine (test_streaming_pack_errors).  Not part of the product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nydus-snapshotter_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import layers  # noqa: E402
import nydus_gpu  # noqa: E402

tars = {k: fn() for k, fn in layers.LAYERS.items()}
for variant in ("fresh", "after_abort", "after_err", "full_sequence"):
    eng = nydus_gpu.Engine(chunk_size=0x100000)
    try:
        if variant in ("after_err", "full_sequence"):
            w = eng.pack()
            w.write(tars["oci_upper"][: len(tars["oci_upper"]) // 2])
            try:
                w.close()
            except nydus_gpu.NgpuError as e:
                print(variant, "close err", e.code)
        if variant == "full_sequence":
            w = eng.pack()
            try:
                w.write(b"z" * 2048)
            except nydus_gpu.NgpuError as e:
                print(variant, "write err", e.code)
        if variant in ("after_abort", "full_sequence"):
            w = eng.pack()
            w.write(tars["oci_lower"])
            w.abort()
        ch, out, st = eng.pack().close()
        print(variant, "empty pack:", len(ch), st, flush=True)
        ch, out, st = eng.pack().close()
        print(variant, "empty pack again:", len(ch), st, flush=True)
    finally:
        eng.close()
eng = nydus_gpu.Engine(chunk_size=0x100000)
w = eng.pack()
w.write(tars["oci_lower"])
ch, out, st = w.close()
print("oci_lower chunks", len(ch), st)
eng.close()
