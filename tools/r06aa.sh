set -o pipefail
mkdir -p gpurun_out/r06aa
T="python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_smallround.py tests/test_gpu_fedopt_f32state.py tests/test_gpu_staging_cache.py tests/test_gpu_faults.py tests/test_gpu_batch_faults.py > gpurun_out/r06aa/pytest.log 2>&1 || exit 10
timeout -k 10 300 python -u tools/fedopt_small_stress.py > gpurun_out/r06aa/stress.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/small_floor.py > gpurun_out/r06aa/small_floor.log 2>&1 || exit 12
