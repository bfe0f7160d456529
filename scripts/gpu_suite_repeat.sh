#!/bin/bash
# The GPU suite R times back to back (fresh processes, as the driver runs it),
# stopping at the first failing run; the digest guard turns an unwritten digest
# into NGPU_EDEVICE with the chunk id and kernel path, so a recurrence of the
# r2 zero digest names its path.  Then the 2-rank gloo bench.
# usage: scripts/gpu_suite_repeat.sh TAG R
set -u
TAG=${1:-rep}
R=${2:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 "$R"); do
  timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 \
    --timeout-method thread > "$OUT/suite_$i.log" 2>&1
  rc=$?
  echo "suite $i rc=$rc: $(tail -1 "$OUT/suite_$i.log")"
  grep -n "EDEVICE\|unhashed\|unwritten" "$OUT/suite_$i.log" | head -5
  [ $rc -ne 0 ] && exit $rc
done
bash scripts/gpu_n2_gloo.sh "$TAG"
