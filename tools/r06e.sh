set -o pipefail
mkdir -p gpurun_out/r06e
T="python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu"
FEDN_AMD_POISON_REUSE=1 timeout -k 10 900 $T tests/ > gpurun_out/r06e/pytest_gpu_poison.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/save_phases.py --threads 8,16 > gpurun_out/r06e/save_phases.log 2>&1 || exit 12
timeout -k 10 400 python -u tools/window_concurrent.py --reps 15 > gpurun_out/r06e/window_concurrent15.log 2>&1 || exit 13
