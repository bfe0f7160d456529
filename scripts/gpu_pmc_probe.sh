#!/bin/bash
# Chunk-dict probe / build traffic (request-size PMC, separate passes, kernel
# trace only) on the C3 bench: 200M-entry dict build (dict_insert) and the
# 16M-query probe roofline launches (dict_probe_records).
# usage: scripts/gpu_pmc_probe.sh TAG
set -u
TAG=${1:-probe}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 600 python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
ok $? bench_c3
cd /tmp
K='dict_probe_records|dict_insert'
S1="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
S2="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum"
P=0
for SET in "$S1" "$S2" "WRITE_SIZE"; do
  P=$((P+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "$K" --output-format csv -d "$OUT/k$P" -o pmc -- python3 "$ROOT/bench.py" --workload c3 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/k$P.log" 2>&1
  ok $? "pmc$P"
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_req_probe.json" 'dict_probe_records' "$OUT/k1" "$OUT/k2" "$OUT/k3"
python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_req_insert.json" 'dict_insert' "$OUT/k1" "$OUT/k2" "$OUT/k3"
