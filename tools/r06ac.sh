set -o pipefail
mkdir -p gpurun_out/r06ad
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream_order.py > gpurun_out/r06ad/pytest.log 2>&1 || exit 10
timeout -k 10 300 python -u tools/stream_order_demo.py > gpurun_out/r06ad/demo.log 2>&1 || exit 11
