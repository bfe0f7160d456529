#!/bin/bash
# SHA-256 small-layer crossover: GPU (device-resident digest+dedup) vs the
# 16-core CPU port on the same layers, 1 MiB chunks, 64 MiB .. 2 GiB layers.
# usage: scripts/gpu_sha_crossover.sh TAG
set -u
TAG=${1:-shax}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
: > "$OUT/sha_crossover.jsonl"
for m in 16 64 256 512 1024 2048; do
  timeout -k 10 240 python3 bench.py --workload l${m}m --digester sha256 --steps 10 --warmup 3 \
    --no-e2e --no-sub --settle-s 0.5 >> "$OUT/sha_crossover.jsonl" 2>> "$OUT/sha_crossover.err"
  rc=$?; echo "l${m}m rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT/sha_crossover.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    c = d["config"]
    print(c["name"], c["chunks"], "chunks", "gpu", d["value"], "cpu16", d["cpu_baseline"]["value"],
          "kernel", d["roofline"]["kernel"], "ms", d["ms_per_step"])
PY
