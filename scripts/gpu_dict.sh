#!/bin/bash
# Parity tests + dict workloads (C3 200M-entry dict, C4 pool/sharded on one GPU).
set -u
TAG=${1:-dict}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; ok $rc pytest-gpu; tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then grep -E "^E |Error" "$OUT/pytest_gpu.log" | head -30; exit 1; fi
for W in c3-blake3 c3 c4; do
  timeout -k 10 900 python bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err"
  ok $? bench-$W; cat "$OUT/bench_$W.json"; tail -3 "$OUT/bench_$W.err"
done
