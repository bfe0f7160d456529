#!/bin/bash
set -u
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_m4
mkdir -p $OUT
cd /tmp
P=0
for SET in "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" ; do
  P=$((P+1))
  timeout -k 10 120 rocprofv3 --pmc $SET --kernel-include-regex 'b3_groups' --output-format csv -d $OUT/pmc$P -o pmc -- python3 $ROOT/tools/mixed_sizes.py 4 4 0x100000 > $OUT/pmc$P.log 2>&1 || exit $?
done
python3 $ROOT/scripts/pmc_summary.py $OUT/pmc_m4.json 'b3_groups<3' $OUT/pmc1
