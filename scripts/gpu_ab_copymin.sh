#!/bin/bash
# A/B of the copy-pool threshold (NGPU_COPY_MIN) on the C1 streaming Pack
# (1 MiB writes, tools/pack_phases.py), alternated twice on one box.
set -u
TAG=${1:-r3cm}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for r in 1 2; do
  for v in 8388608 1048576 262144; do
    NGPU_COPY_MIN=$v timeout -k 10 200 python3 tools/pack_phases.py > "$OUT/phases_${v}_$r.json" 2>> "$OUT/err"
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
    echo "$v $r $(cat "$OUT/phases_${v}_$r.json")"
  done
done
