#!/bin/bash
# Round-4 measurements: held clock + VALU instruction counts of the dominant
# kernel (separate --pmc passes, kernel trace only), rocprof kernel stats of the
# default bench line, the sha256 crossover sweep, the 8-part node rehearsal
# (routed vs copy exchange) and the 2-rank gloo rehearsal of the N > 1 line.
# usage: scripts/gpu_r4_measure.sh TAG [steps...]
set -u
TAG=${1:-r4m}
shift || true
STEPS=${*:-clock insts insts0 stats early sha node n2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
K='b3_groups|b3_quad_leaves|b3_quad_planned|sha256_split|sha256_pair|sha256_lane'
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    clock)
      (cd /tmp && timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$K" --output-format csv -d "$OUT/clk" -o pmc -- python3 "$ROOT/bench.py" --steps 40 --warmup 10 --no-cpu-baseline --no-e2e --no-sub > "$OUT/clk.log" 2>&1)
      ok $? clock
      python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_clock_c2.json" "$K" "$OUT/clk" ;;
    insts)
      (cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d "$OUT/ins" -o pmc -- python3 "$ROOT/bench.py" --steps 20 --warmup 10 --no-cpu-baseline --no-e2e --no-sub > "$OUT/ins.log" 2>&1)
      ok $? insts
      python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_insts_c2.json" "$K" "$OUT/ins" ;;
    insts0)  # the same pass on the A/B build without the quad in-window tree
      (cd /tmp && NYDUS_GPU_LIB="$ROOT/nydus-snapshotter_amd/build/ab/wgq0.so" timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d "$OUT/ins0" -o pmc -- python3 "$ROOT/bench.py" --steps 20 --warmup 10 --no-cpu-baseline --no-e2e --no-sub > "$OUT/ins0.log" 2>&1)
      ok $? insts0
      python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_insts_c2_wgq0.json" "$K" "$OUT/ins0" ;;
    req)  # request-size traffic of the dominant kernel (roofline.traffic)
      CAL=0 bash "$ROOT/scripts/gpu_pmc_req.sh" "$TAG/req" c2 > "$OUT/req.log" 2>&1
      ok $? req
      cp "$OUT/req/pmc_req_c2.json" "$OUT/pmc_req_c2.json" ;;
    ceiling)  # the compression stream alone (tools/b3_ceiling.hip), then its clock at 4 and 8 waves/SIMD
      timeout -k 10 120 "$ROOT/tools/b3_ceiling" 1 2 3 4 5 6 8 > "$OUT/b3_ceiling.jsonl" 2> "$OUT/b3_ceiling.err"
      ok $? ceiling
      cat "$OUT/b3_ceiling.jsonl"
      for w in 4 8; do
        (cd /tmp && timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/ceil_clk$w" -o pmc -- "$ROOT/tools/b3_ceiling" $w > "$OUT/ceil_clk$w.log" 2>&1)
        ok $? ceiling-clock-$w
        python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_clock_b3_ceiling_w$w.json" 'b3_ceiling' "$OUT/ceil_clk$w"
      done ;;
    stats)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c2 -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sub > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err")
      ok $? stats ;;
    sha)
      bash "$ROOT/scripts/gpu_sha_crossover.sh" "$TAG" > "$OUT/sha.log" 2>&1
      ok $? sha
      cat "$OUT/sha.log" ;;
    node)
      (cd "$ROOT" && timeout -k 10 400 python3 bench.py --node 0,0,0,0,0,0,0,0 --workload c4-16 --steps 10 --warmup 10 > "$OUT/node_w8.json" 2> "$OUT/node_w8.err")
      ok $? node
      python3 -c "import json; d=json.load(open('$OUT/node_w8.json')); print(json.dumps(d['exchange']))" ;;
    early)
      (cd "$ROOT" && timeout -k 10 300 python3 tools/e2e_early.py 3 32 > "$OUT/e2e_early.json" 2> "$OUT/e2e_early.err")
      ok $? early
      cat "$OUT/e2e_early.json" ;;
    n2)
      (cd "$ROOT" && C4L=4 bash scripts/gpu_n2_gloo.sh "$TAG" > "$OUT/n2.log" 2>&1)
      ok $? n2
      tail -c 3000 "$OUT/bench_c2_n2_gloo.json" ;;
  esac
done
