set -u
mkdir -p gpurun_out/r6b
timeout -k 10 600 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_bench_launch.py tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -v -p no:cacheprovider -k "node or bench or batch or sha or kat or random_vs" --timeout 300 --timeout-method thread > gpurun_out/r6b/pytest.log 2>&1
rc=$?; echo pytest rc=$rc; tail -4 gpurun_out/r6b/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
for m in pair pair_pf pair_pf_asm; do
  timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 5 --sha-mode $m --no-cpu-baseline --no-e2e > gpurun_out/r6b/c3_$m.json 2> gpurun_out/r6b/c3_$m.err
  rc=$?; echo c3 $m rc=$rc
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/r6b/c3_$m.err; exit $rc; fi
  python - <<PY
import json; d=json.loads(open("gpurun_out/r6b/c3_$m.json").read().splitlines()[-1]); print("$m", d["value"], d["ms_per_step"], d.get("roofline",{}).get("frac"))
PY
done
