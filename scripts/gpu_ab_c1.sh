#!/bin/bash
# A/B of libnydusgpu.so builds on C1 calls: untimed and timed back-to-back
# calls (tools/c1_gaps.py) and the C1 bench line, alternated R rounds.
# usage: scripts/gpu_ab_c1.sh TAG ROUNDS LIB.so [LIB.so ...]
set -u
TAG=$1; R=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for r in $(seq 1 "$R"); do
  for lib in "$@"; do
    v=$(basename "$lib" .so)
    for t in 0 1; do
      NYDUS_GPU_LIB=$lib timeout -k 10 120 python tools/c1_gaps.py $t > "$OUT/gaps_${v}_t${t}_$r.txt" 2>>"$OUT/err" || exit $?
      echo "$v r$r $(cat "$OUT/gaps_${v}_t${t}_$r.txt")"
    done
    NYDUS_GPU_LIB=$lib timeout -k 10 200 python bench.py --workload c1 --no-cpu-baseline --no-e2e \
      > "$OUT/c1_${v}_$r.json" 2>>"$OUT/err" || exit $?
    python3 -c "import json; d=json.load(open('$OUT/c1_${v}_$r.json')); print('$v r$r bench', d['value'], d['stage_ms'])"
  done
done
