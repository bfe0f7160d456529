#!/bin/bash
# r6e: the round-6 build end to end: whole GPU suite, smoke, default bench line
# (C2 + c3 / c5_1000 sub-entries + CPU baseline + PCIe rates), C1, the 32-Pack
# API lines (blake3, sha256), rocprofv3 kernel stats of C2 and C3.
set -u
TAG=${1:-r6e}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu.log"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
ok $? smoke
timeout -k 10 600 python3 bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
ok $? bench_c2
timeout -k 10 300 python3 bench.py --workload c1 --steps 200 --warmup 20 > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"
ok $? bench_c1
timeout -k 10 400 python3 bench.py --workload c1 --packs 32 --steps 20 --warmup 5 > "$OUT/packs_c1.json" 2> "$OUT/packs_c1.err"
ok $? packs_c1
timeout -k 10 400 python3 bench.py --workload c1-sha256 --packs 32 --steps 10 --warmup 3 > "$OUT/packs_c1_sha256.json" 2> "$OUT/packs_c1_sha256.err"
ok $? packs_c1_sha256
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o prof -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-sub > "$OUT/prof_c2.log" 2>&1
ok $? prof_c2
python3 "$ROOT/scripts/prof_agree.py" "$OUT/prof_c2" 'b3_groups' "$OUT/prof_c2.log" "$OUT/rocprof_c2_agreement.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o prof -- python3 "$ROOT/bench.py" --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > "$OUT/prof_c3.log" 2>&1
ok $? prof_c3
python3 "$ROOT/scripts/prof_agree.py" "$OUT/prof_c3" 'sha256_pair' "$OUT/prof_c3.log" "$OUT/rocprof_c3_agreement.json"
echo done
