set -o pipefail
mkdir -p gpurun_out/r06q
T="python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_smallround.py > gpurun_out/r06q/pytest_small.log 2>&1 || exit 10
