set -o pipefail
mkdir -p gpurun_out/r06t
timeout -k 10 300 python -u tools/small_floor.py > gpurun_out/r06t/small_floor.log 2>&1 || exit 12
