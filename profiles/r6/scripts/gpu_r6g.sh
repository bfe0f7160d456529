#!/bin/bash
# r6g: the N > 1 line rehearsed on one GPU (2 gloo ranks, node extras on
# device 0 twice: node_cabi, packs_node, c4, sharded_dict, multi_gpu_checks),
# then the threaded oracle soak (16 threads on shared engines and a 4-part node).
set -u
TAG=${TAG:-r6g}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
bash scripts/gpu_n2_gloo.sh $TAG/n2 > "$OUT/n2_call.log" 2>&1
rc=$?; echo "n2 rc=$rc"; tail -c 600 "$OUT/n2/bench_c2_n2_gloo.err"; if [ $rc -ne 0 ] && [ $rc -ne 4 ]; then exit $rc; fi
timeout -k 10 900 python -u scripts/gpu_soak.py --threads 16 40 > "$OUT/soak_threads.log" 2>&1
ok $? soak_threads
tail -2 "$OUT/soak_threads.log"
echo done
