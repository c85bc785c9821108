set -o pipefail
mkdir -p gpurun_out/r06c
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_smallround.py tests/test_gpu_poison_reuse.py > gpurun_out/r06c/pytest_new.log 2>&1 || exit 11
timeout -k 10 200 $T tests/test_gpu_release.py > gpurun_out/r06c/pytest_release.log 2>&1 || exit 12
timeout -k 10 300 python -u tools/small_floor.py > gpurun_out/r06c/small_floor.log 2>&1 || exit 13
timeout -k 10 400 python -u tools/window_concurrent.py --reps 5 > gpurun_out/r06c/window_concurrent.log 2>&1 || exit 14
