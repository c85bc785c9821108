set -o pipefail
mkdir -p gpurun_out/r06af
T="python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu"
FEDN_AMD_POISON_REUSE=1 FEDN_AMD_POISON_HOLD=1 timeout -k 10 900 $T tests/ > gpurun_out/r06af/pytest_gpu_poison_hold.log 2>&1 || exit 11
