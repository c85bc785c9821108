TAG=${1:-r01r}; mkdir -p gpurun_out/$TAG
export FEDN_AMD_BENCH_ONE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --params 20000000 --clients 16 > gpurun_out/$TAG/dist.log 2>&1; echo "dist rc=$?"; tail -3 gpurun_out/$TAG/dist.log
