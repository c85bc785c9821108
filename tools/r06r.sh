set -o pipefail
mkdir -p gpurun_out/r06r
T="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_gpu_parity.py -k "waves" > gpurun_out/r06r/pytest_waves.log 2>&1 || exit 10
