#!/bin/bash
# Round-5 checks in one box; steps run in the order given, the first failure
# ends the call.  usage: scripts/gpu_r5.sh TAG step...
#   valu  : scripts/gpu_r5_valu.sh (VALU bank microbenchmark + SQ counters)
#   suite : pytest -m gpu (optionally PYK="-k expr")
#   smoke : __graft_entry__.smoke()
#   bench : default bench line (N = 1)
#   stats : rocprofv3 --kernel-trace --stats of the C2 bench
#   n2    : python3 bench.py --gpus 2 over gloo (self-launched ranks)
set -u
TAG=${1:-r5}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
for s in "$@"; do
  case $s in
    valu)
      bash scripts/gpu_r5_valu.sh "$TAG/valu" > "$OUT/valu.log" 2>&1
      ok $? valu
      cat "$OUT/valu.log" | cut -c1-220 ;;
    valu3)
      for cfg in "512 1" "1024 1" "256 1"; do
        set -- $cfg
        for v in mix_s compiled_bar mix_x4a4_bar compiled; do
          timeout -k 10 120 ./tools/valu_bank $v $1 $2 >> "$OUT/valu3.jsonl" 2>> "$OUT/valu3.err"
          ok $? "valu3 $v $1 $2"
        done
      done
      wc -l "$OUT/valu3.jsonl" ;;
    valu4)
      for v in compiled comp_nop; do
        timeout -k 10 150 ./tools/valu_bank $v 256 1 >> "$OUT/valu4.jsonl" 2>> "$OUT/valu4.err"
        ok $? "valu4 $v"
      done
      wc -l "$OUT/valu4.jsonl" ;;
    valu2)
      bash scripts/gpu_r5_valu2.sh "$TAG/valu2" > "$OUT/valu2.log" 2>&1
      ok $? valu2
      tail -3 "$OUT/valu2.log" ;;
    suite)
      if [ -n "${PYK:-}" ]; then
        timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "$PYK" > "$OUT/pytest_gpu.log" 2>&1
      else
        timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
      fi
      ok $? suite
      tail -1 "$OUT/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      ok $? smoke
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
      ok $? bench
      python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], r['frac'], r.get('frac_mix'), r.get('frac_ceiling'), d['cpu_baseline']['value'], [d.get(k, {}).get('value') for k in ('c1', 'c3', 'c5_1000')])" ;;
    stats)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c2 -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sub > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err")
      ok $? stats
      python3 scripts/prof_agree.py "$OUT/prof" b3_groups "$OUT/prof_bench.json" "$OUT/rocprof_c2_agreement.json" | cut -c1-200 ;;
    stats3)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof3" -o c3 -- python3 "$ROOT/bench.py" --workload c3 --steps 10 --no-cpu-baseline --no-e2e --no-dict-file > "$OUT/prof3_bench.json" 2> "$OUT/prof3_bench.err")
      ok $? stats3
      python3 scripts/prof_agree.py "$OUT/prof3" sha256_pair "$OUT/prof3_bench.json" "$OUT/rocprof_c3_agreement.json" | cut -c1-200 ;;
    c3)
      df -h /tmp "$ROOT" /dev/shm > "$OUT/df.txt" 2>&1 || true
      timeout -k 10 600 python3 bench.py --workload c3 --steps 10 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err"
      ok $? c3
      python3 -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['dict']))" ;;
    packs)
      timeout -k 10 300 python3 bench.py --workload c1 --packs 32 --steps 10 --warmup 3 > "$OUT/packs_c1.json" 2> "$OUT/packs_c1.err"
      ok $? packs_c1
      timeout -k 10 300 python3 bench.py --workload c1-sha256 --packs 32 --steps 5 --warmup 2 > "$OUT/packs_sha.json" 2> "$OUT/packs_sha.err"
      ok $? packs_sha
      tail -c 600 "$OUT/packs_c1.json" ;;
    h2dp)
      for cfg in "32 20 2 1" "32 20 2 2" "32 20 2 4" "32 20 1 4" "32 20 4 4" "32 20 2 12"; do
        timeout -k 10 60 ./tools/h2d_streams $cfg >> "$OUT/h2dp.jsonl" 2>> "$OUT/h2dp.err"
        ok $? "h2dp $cfg"
      done
      for g in 2097152 4194304; do
        NGPU_EAGER_COPY=$g timeout -k 10 300 python3 bench.py --workload c1 --packs 32 --steps 10 --warmup 3 --packs-modes decisions --no-cpu-baseline > "$OUT/packs_eager_$g.json" 2> "$OUT/packs_eager_$g.err"
        ok $? "packs eager $g"
      done
      timeout -k 10 300 python3 bench.py --workload c1 --packs 32 --steps 10 --warmup 3 --packs-modes decisions --no-cpu-baseline > "$OUT/packs_eager_default.json" 2> "$OUT/packs_eager_default.err"
      ok $? "packs eager default"
      cat "$OUT/h2dp.jsonl" ;;
    pstream)
      timeout -k 10 300 python3 bench.py --workload c1 --packs 32 --steps 10 --warmup 3 --packs-modes decisions,stream_zstd,stream_zstd_no_batch > "$OUT/pstream_c1.json" 2> "$OUT/pstream_c1.err"
      ok $? pstream_c1
      python3 -c "import json; d=json.loads(open('$OUT/pstream_c1.json').read().strip().splitlines()[-1]); print({m: (v['gbs'], v.get('phases')) for m, v in d['modes'].items()}, d['cpu_baseline'].get('pipeline_gbs'))" ;;
    strace)
      NGPU_PACK_TRACE=1 NGPU_SINK_STATS=1 timeout -k 10 300 python3 bench.py --workload c1 --packs 32 --steps 2 --warmup 2 --packs-modes decisions,stream_zstd --no-cpu-baseline > "$OUT/strace_c1.json" 2> "$OUT/strace_c1.err"
      ok $? strace_c1
      grep -c pack_trace "$OUT/strace_c1.err" ;;
    packs128)
      timeout -k 10 400 python3 bench.py --workload c1-sha256 --packs 128 --steps 3 --warmup 1 --packs-modes decisions > "$OUT/packs128_sha.json" 2> "$OUT/packs128_sha.err"
      ok $? packs128_sha
      timeout -k 10 400 python3 bench.py --workload c1 --packs 128 --steps 5 --warmup 2 --packs-modes decisions > "$OUT/packs128_c1.json" 2> "$OUT/packs128_c1.err"
      ok $? packs128_c1
      tail -c 400 "$OUT/packs128_sha.json" ;;
    ptrace)
      NGPU_BATCH_TRACE=1 timeout -k 10 300 python3 bench.py --workload c1 --packs 32 --steps 6 --warmup 2 --packs-modes decisions --no-cpu-baseline > "$OUT/ptrace_c1.json" 2> "$OUT/ptrace_c1.err"
      ok $? ptrace_c1
      NGPU_BATCH_TRACE=1 timeout -k 10 300 python3 bench.py --workload c1-sha256 --packs 32 --steps 3 --warmup 1 --packs-modes decisions --no-cpu-baseline > "$OUT/ptrace_sha.json" 2> "$OUT/ptrace_sha.err"
      ok $? ptrace_sha
      grep -c batch_trace "$OUT/ptrace_c1.err" ;;
    papi)
      for w in c1 c1-sha256; do
        (cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/papi_$w" -o t -- python3 "$ROOT/bench.py" --workload $w --packs 32 --steps 2 --warmup 1 --packs-modes decisions --no-cpu-baseline > "$OUT/papi_$w.json" 2> "$OUT/papi_$w.err")
        ok $? "papi $w"
      done
      ls -R "$OUT/papi_c1" | head -20 ;;
    h2d)
      for cfg in "32 20 1" "32 20 2" "32 20 4" "32 20 8" "32 20 32" "16 20 1" "8 20 1"; do
        timeout -k 10 60 ./tools/h2d_streams $cfg >> "$OUT/h2d.jsonl" 2>> "$OUT/h2d.err"
        ok $? "h2d $cfg"
      done
      cat "$OUT/h2d.jsonl" ;;
    shaclk)
      (cd /tmp && timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex sha256_pair --output-format csv -d "$OUT/shaclk" -o pmc -- python3 "$ROOT/bench.py" --workload c1-sha256 --packs 32 --steps 3 --warmup 1 --packs-modes decisions --no-cpu-baseline > "$OUT/shaclk.log" 2>&1)
      ok $? shaclk
      python3 scripts/pmc_summary.py "$OUT/pmc_clock_packs_sha.json" sha256_pair "$OUT/shaclk" | cut -c1-400 ;;
    shamix)
      for f in 0 6144 10240; do
        timeout -k 10 200 python3 tools/sha_mix.py $f >> "$OUT/sha_mix.jsonl" 2>> "$OUT/sha_mix.err"
        ok $? "shamix $f"
      done
      cat "$OUT/sha_mix.jsonl" ;;
    c1ab)
      for i in 1 2; do
        timeout -k 10 300 python3 bench.py --workload c1 --steps 400 --no-sub --no-cpu-baseline --no-e2e > "$OUT/c1_$i.json" 2> "$OUT/c1_$i.err"
        ok $? "c1 $i"
        python3 -c "import json; d=json.loads(open('$OUT/c1_$i.json').read().strip().splitlines()[-1]); print('c1', d['value'], d['ms_per_step'], d['stage_ms'])"
      done ;;
    shaab)
      timeout -k 10 200 python3 tools/sha_mix.py 0 > "$OUT/sha_mix_new.jsonl" 2>> "$OUT/sha_mix.err"
      ok $? "shamix new"
      timeout -k 10 400 python3 bench.py --workload c3 --steps 10 --no-cpu-baseline --no-dict-file > "$OUT/c3.json" 2> "$OUT/c3.err"
      ok $? c3
      timeout -k 10 300 python3 bench.py --workload c1-sha256 --packs 32 --steps 5 --warmup 2 --packs-modes decisions --no-cpu-baseline > "$OUT/packs_sha.json" 2> "$OUT/packs_sha.err"
      ok $? packs_sha
      cat "$OUT/sha_mix_new.jsonl"; python3 -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'])"; python3 -c "import json; d=json.loads(open('$OUT/packs_sha.json').read().strip().splitlines()[-1]); print('packs_sha', d['value'], d['modes']['decisions']['device_gbs'])" ;;
    soak)
      timeout -k 10 600 python3 -u scripts/gpu_soak.py --threads ${SOAK_THREADS:-16} ${SOAK_CASES:-40} 20646 > "$OUT/soak_threads.log" 2>&1
      ok $? soak_threads
      timeout -k 10 300 python3 -u scripts/gpu_soak.py 150 20647 > "$OUT/soak_single.log" 2>&1
      ok $? soak_single
      tail -1 "$OUT/soak_threads.log"; tail -1 "$OUT/soak_single.log" ;;
    n4)
      NYDUS_NODE_EXTRA_DEVICES=0,0,0,0 timeout -k 10 900 python3 bench.py --gpus 4 --steps 5 --warmup 3 --dist-backend gloo --c4-layers 2 > "$OUT/bench_c2_n4_gloo.json" 2> "$OUT/bench_c2_n4_gloo.err"
      ok $? n4
      python3 -c "import json; d=json.loads(open('$OUT/bench_c2_n4_gloo.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d.get('ranks'), json.dumps(d.get('node_cabi', {}))[:300], json.dumps(d.get('c4', {}))[:200], json.dumps(d.get('sharded_dict', {}))[:200])" ;;
    n2)
      NYDUS_NODE_EXTRA_DEVICES=0,0 timeout -k 10 600 python3 bench.py --gpus 2 --steps 10 --warmup 5 --dist-backend gloo --c4-layers 4 > "$OUT/bench_c2_n2_gloo.json" 2> "$OUT/bench_c2_n2_gloo.err"
      ok $? n2
      python3 -c "import json; d=json.loads(open('$OUT/bench_c2_n2_gloo.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d.get('ranks'), json.dumps(d.get('node_cabi', {}).get('node_step')), d.get('c4', {}).get('value'))" ;;
  esac
done
