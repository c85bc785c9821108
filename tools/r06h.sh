set -o pipefail
mkdir -p gpurun_out/r06h
T="python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T -x tests/test_gpu_smallround.py tests/test_gpu_faults.py tests/test_gpu_batch_faults.py tests/test_gpu_staging_cache.py > gpurun_out/r06h/pytest_small.log 2>&1 || exit 10
timeout -k 10 900 $T tests/ > gpurun_out/r06h/pytest_gpu.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/small_floor.py > gpurun_out/r06h/small_floor.log 2>&1 || exit 12
