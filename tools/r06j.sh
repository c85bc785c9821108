set -o pipefail
mkdir -p gpurun_out/r06j
T="python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T -x tests/test_gpu_smallround.py tests/test_gpu_faults.py tests/test_gpu_batch_faults.py tests/test_gpu_staging_cache.py > gpurun_out/r06j/pytest_small.log 2>&1 || exit 10
timeout -k 10 300 $T -x tests/test_gpu_parity.py -k "small or zero_copy or golden" > gpurun_out/r06j/pytest_parity.log 2>&1 || exit 11
timeout -k 10 600 python -u tools/bench_small.py > gpurun_out/r06j/small.log 2>&1 || exit 12
