set -o pipefail
mkdir -p gpurun_out/r06s2
T="python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu"
FEDN_AMD_POISON_REUSE=1 timeout -k 10 900 $T tests/ > gpurun_out/r06s2/pytest_gpu_poison.log 2>&1 || exit 11
FEDN_AMD_FUZZ_BASE=400000 FEDN_AMD_FUZZ_SCALE=8 timeout -k 10 600 $T tests/test_gpu_fuzz.py tests/test_gpu_fuzz_thresholds.py > gpurun_out/r06s2/fuzz.log 2>&1 || exit 12
