#!/bin/bash
# r6f: round-6 PMC traffic of C5-1000 and the held clock of C2 (so every
# profile the default line cites is this round's), then the oracle soak on the
# round-6 build (random layers through pack_tar + streaming Packs).
set -u
TAG=r6f
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ok() { local rc=$1 what=$2; echo "$what rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
CAL=0 timeout -k 10 900 bash scripts/gpu_pmc_req.sh $TAG/pmc_c5-1000 c5-1000 > "$OUT/pmc_c5.log" 2>&1
ok $? pmc_c5-1000
timeout -k 10 400 bash scripts/gpu_pmc_clock.sh $TAG/clock c2 > "$OUT/clock.log" 2>&1
ok $? pmc_clock_c2
timeout -k 10 900 bash scripts/gpu_soak.sh $TAG/soak 200 > "$OUT/soak_call.log" 2>&1
ok $? soak
tail -3 "$OUT/soak/soak.log"
echo done
