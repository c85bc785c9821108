set -o pipefail
mkdir -p gpurun_out/r06u
timeout -k 10 300 python -u tools/small_floor.py > gpurun_out/r06u/default.log 2>&1 || exit 11
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python -u tools/small_floor.py > gpurun_out/r06u/devkernarg.log 2>&1 || exit 12
