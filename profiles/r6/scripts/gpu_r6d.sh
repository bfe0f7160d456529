#!/bin/bash
# r6d: the eager H2D granule of streaming Packs (NGPU_EAGER_COPY) on the
# 32-Pack API bench (ReadFrom feed), and H2D copy-lane count via two engines.
set -u
TAG=r6d
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
for G in 1 2 4 8 16; do
  NGPU_EAGER_COPY=$((G<<20)) timeout -k 10 300 python bench.py --workload c1 --packs 32 --steps 20 --warmup 5 --packs-modes decisions,stream_zstd --no-cpu-baseline > "$OUT/packs_g$G.json" 2> "$OUT/packs_g$G.err"
  ok $? packs_g$G
  python3 -c "
import json; d=json.loads(open('$OUT/packs_g$G.json').read().splitlines()[-1]); m=d['modes']
print('granule $G MiB', {k:(v['gbs'], v['ms_per_round'], v['phases']['tail_after_last_write_ms_median']) for k,v in m.items()})"
done
