set -o pipefail
mkdir -p gpurun_out/r06l
T="python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu"
FEDN_AMD_POISON_REUSE=1 timeout -k 10 900 $T tests/ > gpurun_out/r06l/pytest_gpu_poison.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/small_floor.py > gpurun_out/r06l/small_floor.log 2>&1 || exit 12
