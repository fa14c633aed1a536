set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/r01_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/r01_gpu_tests.log
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r01_bench_first.json 2> gpurun_out/r01_bench_first.err
  echo "bench rc=$?"
  cat gpurun_out/r01_bench_first.json; tail -5 gpurun_out/r01_bench_first.err
fi
