set -o pipefail
mkdir -p gpurun_out/r06x
timeout -k 10 500 python -u tools/fedopt_small_stress.py > gpurun_out/r06x/stress.log 2>&1 || exit 11
