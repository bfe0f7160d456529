#!/bin/bash
# The probe's line requests by kernel variant (dedup.hip dict_probe_variant,
# NGPU_PROBE_VARIANT 0..7) at a small and the C3-size dict.
# usage: scripts/gpu_probe_variants.sh TAG [variants] [sizes]
set -u
TAG=${1:-pvar}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
for v in ${2:-0 4 1 2 3}; do
  NGPU_PROBE_VARIANT=$v bash scripts/gpu_probe_sweep.sh "$TAG/v$v" ${3:-1,200} > "gpurun_out/$TAG.v$v.log" 2>&1
  rc=$?
  echo "variant $v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json
for d in json.load(open('gpurun_out/$TAG/v$v/probe_sweep.json')):
    print('  v$v', d['dict_entries'], 'ms', d['ms'], 'lines/probe', d['read_lines_per_probe'], 'hits', d['hits'])"
done
