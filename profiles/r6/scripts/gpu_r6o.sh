#!/bin/bash
# r6o: long oracle soak on the closing build: 2,000 random layers through
# pack_tar and streaming Packs (new seed), then 16 threads x 200 cases on
# shared engines and a 4-part node.
set -u
TAG=r6o
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u scripts/gpu_soak.py 2000 24742 > "$OUT/soak_single.log" 2>&1
rc=$?; echo "soak_single rc=$rc"; tail -1 "$OUT/soak_single.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/gpu_soak.py --threads 16 200 24743 > "$OUT/soak_threads.log" 2>&1
rc=$?; echo "soak_threads rc=$rc"; tail -1 "$OUT/soak_threads.log"
exit $rc
