#!/bin/bash
# SHA-256 one-lane-per-chunk kernel: parity, then all variants at several chunk sizes.
set -u
TAG=${1:-shalane}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "sha" > "$OUT/pytest_sha.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_sha.log"
[ $rc -eq 0 ] || exit 1
for S in ${SIZES:-65536 262144 1048576 16384}; do
  timeout -k 10 300 python -u tools/sha_diag.py $S >> "$OUT/sha_variants.jsonl" 2>> "$OUT/sha_diag.err"
  rc=$?; echo "diag $S rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat "$OUT/sha_variants.jsonl"
