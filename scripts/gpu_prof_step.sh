set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$(pwd)/gpurun_out/profc5
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c5 -o c5 -- python3 $OLDPWD/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/c5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/m4 -o m4 -- python3 $OLDPWD/tools/mixed_sizes.py 4 4 0x100000 > $OUT/m4.log 2>&1 || exit $?
echo ok
