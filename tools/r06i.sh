set -o pipefail
mkdir -p gpurun_out/r06i
timeout -k 10 600 python -u tools/bench_round_e2e.py > gpurun_out/r06i/roundblob.log 2>&1 || exit 11
timeout -k 10 600 python -u tools/bench_small.py > gpurun_out/r06i/small.log 2>&1 || exit 12
