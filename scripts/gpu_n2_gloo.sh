#!/bin/bash
# Two ranks on the one-GPU box over gloo (RCCL refuses two ranks per GPU):
# the torchrun bench path, including the sharded-dict extra of N > 1 runs.
# usage: scripts/gpu_n2_gloo.sh TAG
set -u
TAG=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
NYDUS_NODE_EXTRA_DEVICES=${NYDUS_NODE_EXTRA_DEVICES:-0,0} timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 5 \
  --dist-backend gloo --c4-layers ${C4L:-4} > "$OUT/bench_c2_n2_gloo.json" 2> "$OUT/bench_c2_n2_gloo.err"
rc=$?
echo "n2 rc=$rc"
cat "$OUT/bench_c2_n2_gloo.json"
exit $rc
