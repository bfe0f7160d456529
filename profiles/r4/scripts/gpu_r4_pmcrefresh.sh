#!/bin/bash
# Round-4 refresh of the request-size PMC behind every sub-entry's
# roofline.traffic: C1 (b3_quad_planned), C3 (sha256_pair), C5-1000
# (b3_groups<3>, previously null) and the C3 probe / build.  Separate --pmc
# passes, kernel trace only, each under its own time limit.
# usage: scripts/gpu_r4_pmcrefresh.sh TAG [c1 c3 c5-1000 probe]
set -u
TAG=${1:-pmcr}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
for W in "${@:-c1 c3 c5-1000 probe}"; do
  if [ "$W" = probe ]; then
    (cd "$ROOT" && bash scripts/gpu_pmc_probe.sh "$TAG/probe") > "$OUT/probe.log" 2>&1
    ok $? probe
  else
    (cd "$ROOT" && CAL=0 bash scripts/gpu_pmc_req.sh "$TAG/$W" "$W") > "$OUT/$W.log" 2>&1
    ok $? "$W"
  fi
  tail -1 "$OUT/$W.log" | cut -c1-400
done
