"""Repeat the golden-layer pack_tar check on fresh engines (each engine's
first call allocates its buffers) and report mismatching chunks per
(case, leaves_per_lane).  usage: python3 scripts/golden_repeat.py REPS"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nydus-snapshotter_amd"), os.path.join(ROOT, "tests", "golden")]
import layers  # noqa: E402
import nydus_gpu  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "layers.json")))
tars = {k: fn() for k, fn in layers.LAYERS.items()}
bad = {}
for r in range(reps):
    for case in gold["cases"]:
        for lanes in ([1, 2, 4, 8, 16] if case["digester"] == "blake3" else [0]):
            eng = nydus_gpu.Engine(digester=case["digester"], chunk_size=case["chunk_size"],
                                   leaves_per_lane=lanes)
            try:
                ch, out, st = eng.pack_tar(tars[case["layer"]])
            finally:
                eng.close()
            got = [d.tobytes().hex() for d in out["digest"]]
            miss = [i for i, (a, b) in enumerate(zip(got, case["digests"])) if a != b]
            if miss:
                k = f'{case["layer"]}/{case["digester"]}/{case["chunk_size"]}/lanes{lanes}'
                bad.setdefault(k, []).append((r, miss[:8]))
    print(f"rep {r} done, failing configs so far: {len(bad)}", flush=True)
print(json.dumps(bad))
