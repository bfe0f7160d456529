#!/bin/bash
# Why b3_groups holds ~2.03 GHz while its bare compression stream holds 2.36:
# the C2 bench on the product build and on a no-load diagnostic build
# (build/ab/nol.so, -DNGPU_DIAG_NOLOAD=1, load mode 4: the same kernel with
# register-made message words, no HBM reads; digests NOT BLAKE3), time and
# held clock (GRBM_GUI_ACTIVE pass) of each.  usage: scripts/gpu_clock_diag.sh TAG
set -u
TAG=${1:-clk}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
K='b3_groups'
B="--steps 40 --warmup 10 --no-cpu-baseline --no-e2e --no-sub"
cd "$ROOT"
timeout -k 10 300 python3 bench.py $B > "$OUT/prod.json" 2> "$OUT/prod.err"
ok $? prod
NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/ab/nol.so timeout -k 10 300 python3 bench.py $B --load-mode 4 > "$OUT/nol.json" 2> "$OUT/nol.err"
ok $? nol
cd /tmp
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$K" --output-format csv -d "$OUT/clk_prod" -o pmc -- python3 "$ROOT/bench.py" $B > "$OUT/clk_prod.log" 2>&1
ok $? clk_prod
NYDUS_GPU_LIB=$ROOT/nydus-snapshotter_amd/build/ab/nol.so timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$K" --output-format csv -d "$OUT/clk_nol" -o pmc -- python3 "$ROOT/bench.py" $B --load-mode 4 > "$OUT/clk_nol.log" 2>&1
ok $? clk_nol
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT/pmc_clock_prod.json" "$K" "$OUT/clk_prod" | cut -c1-300
python3 scripts/pmc_summary.py "$OUT/pmc_clock_nol.json" "$K" "$OUT/clk_nol" | cut -c1-300
for f in prod nol; do python3 -c "import json; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', d['stage_ms']['digest'], d['roofline']['achieved'])"; done
