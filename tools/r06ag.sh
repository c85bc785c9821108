set -o pipefail
mkdir -p gpurun_out/r06ag
T="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_poison_reuse.py > gpurun_out/r06ag/poison_default.log 2>&1 || exit 11
FEDN_AMD_POISON_HOLD=1 timeout -k 10 300 $T tests/test_gpu_poison_reuse.py > gpurun_out/r06ag/poison_hold.log 2>&1 || exit 12
FEDN_AMD_POISON_REUSE=1 timeout -k 10 300 $T tests/test_gpu_poison_reuse.py tests/test_gpu_parity.py -k "multidevice or poison or waves" > gpurun_out/r06ag/poison_default_suite.log 2>&1 || exit 13
