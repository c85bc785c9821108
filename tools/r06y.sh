set -o pipefail
mkdir -p gpurun_out/r06y
T="python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/ > gpurun_out/r06y/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -u tools/fedopt_small_stress.py > gpurun_out/r06y/stress.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/small_floor.py > gpurun_out/r06y/small_floor.log 2>&1 || exit 12
