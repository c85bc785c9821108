set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 300 python -u tools/save_phases.py --threads 8,16 > gpurun_out/r06f/save_phases.log 2>&1 || exit 12
bash tools/gpu_session.sh r06f smoke bench prof
