#!/bin/bash
# Round-4 closing check in one box: GPU suite, smoke, default bench line,
# rocprof stats of the bench, the first-call race A/B, the probe sweep and the
# 2-rank gloo rehearsal of the N > 1 line.  usage: scripts/gpu_r4_close.sh TAG [steps]
set -u
TAG=${1:-r4c}
shift || true
STEPS=${*:-suite smoke bench stats race probe n2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
for s in $STEPS; do
  case $s in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
      ok $? suite
      tail -1 "$OUT/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      ok $? smoke
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
      ok $? bench
      python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], r['frac'], r.get('frac_mix'), r.get('frac_ceiling'), r.get('frac_ceiling_per_cycle'), d['cpu_baseline']['value'], d['e2e_pcie'].get('pack_stream_early_none_gbs'), d['e2e_pcie'].get('host_sha256_gbs'))" ;;
    stats)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c2 -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sub > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err")
      ok $? stats
      python3 scripts/prof_agree.py "$OUT/prof" b3_groups "$OUT/prof_bench.json" "$OUT/rocprof_c2_agreement.json" | cut -c1-200 ;;
    race)
      bash scripts/gpu_race_ab.sh "$TAG/race" > "$OUT/race.log" 2>&1
      ok $? race
      cat "$OUT/race.log" ;;
    probe)
      bash scripts/gpu_probe_sweep.sh "$TAG/psweep" > "$OUT/psweep.log" 2>&1
      ok $? probe
      tail -5 "$OUT/psweep.log" ;;
    n2)
      (C4L=4 bash scripts/gpu_n2_gloo.sh "$TAG" > "$OUT/n2.log" 2>&1)
      ok $? n2
      python3 -c "import json; d=json.loads(open('$OUT/bench_c2_n2_gloo.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d.get('node_cabi', {}).get('node_step')), d.get('c4', {}).get('value'))" ;;
  esac
done
