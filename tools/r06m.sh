set -o pipefail
mkdir -p gpurun_out/r06m
T="python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 400 $T -x tests/test_gpu_parity.py -k "waves" > gpurun_out/r06m/pytest_waves.log 2>&1 || exit 10
timeout -k 10 400 python -u tools/wave_probe.py > gpurun_out/r06m/wave_probe.log 2>&1 || exit 11
