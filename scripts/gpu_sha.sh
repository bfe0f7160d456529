#!/bin/bash
# SHA-256 kernels: parity (KAT / random / ragged for both variants), then C3
# (16 GiB, 1 MiB chunks, 200M-entry dict) with each kernel, plus a 64 KiB-chunk
# SHA-256 layer where the chip has enough chunks for one lane each.
set -u
TAG=${1:-sha}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  -k "kat or random_vs_oracle or ragged" > "$OUT/pytest_sha.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_sha.log"
if [ $rc -ne 0 ]; then grep -E "^E |Error" "$OUT/pytest_sha.log" | head -30; exit 1; fi
for M in split pair; do
  timeout -k 10 600 python bench.py --workload c3 --sha-mode $M --steps 5 --warmup 2 \
    --no-cpu-baseline --no-e2e > "$OUT/bench_c3_$M.json" 2> "$OUT/bench_c3_$M.err"
  rc=$?; echo "bench c3 $M rc=$rc"; cat "$OUT/bench_c3_$M.json"; tail -3 "$OUT/bench_c3_$M.err"
  [ $rc -eq 0 ] || exit $rc
done
for M in split pair; do
  timeout -k 10 600 python bench.py --workload c3-64k --sha-mode $M --steps 5 --warmup 2 \
    --no-cpu-baseline --no-e2e > "$OUT/bench_c3_64k_$M.json" 2> "$OUT/bench_c3_64k_$M.err"
  rc=$?; echo "bench c3-64k $M rc=$rc"; cat "$OUT/bench_c3_64k_$M.json"; tail -3 "$OUT/bench_c3_64k_$M.err"
  [ $rc -eq 0 ] || exit $rc
done
