set -o pipefail
mkdir -p gpurun_out/r06o
timeout -k 10 300 python -u tools/wave_quad_probe.py > gpurun_out/r06o/wave_quad.log 2>&1 || exit 11
