#!/bin/bash
# Parity tests, then interleaved variant tuning (c2 and c5 shapes).
# usage: scripts/gpu_tune.sh TAG
set -u
TAG=${1:-tune}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; ok $rc pytest-gpu; tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then grep -E "^E |Error" "$OUT/pytest_gpu.log" | head -30; exit 1; fi
timeout -k 10 600 python scripts/tune_b3.py --rounds 5 --lanes 4,8,16 --modes 0,2 > "$OUT/tune_c2.jsonl" 2> "$OUT/tune.err"
ok $? tune-c2; cat "$OUT/tune_c2.jsonl"
timeout -k 10 600 python scripts/tune_b3.py --rounds 5 --lanes 4,8,16 --modes 2 --chunk 65536 > "$OUT/tune_c5.jsonl" 2>> "$OUT/tune.err"
ok $? tune-c5; cat "$OUT/tune_c5.jsonl"
