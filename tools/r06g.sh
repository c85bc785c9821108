set -o pipefail
mkdir -p gpurun_out/r06g
timeout -k 10 300 python -u tools/save_phases.py --threads 8,16 --numpy > gpurun_out/r06g/save_phases.log 2>&1 || exit 12
timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu --durations=5 tests/test_gpu_parity.py -k "waves_1b" > gpurun_out/r06g/waves128.log 2>&1 || exit 13
bash tools/gpu_session.sh r06g selflaunch8
