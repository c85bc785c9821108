"""bench.py — device-resident FedAvg reduce on MI355X (BASELINE.json metric).

One "step" = one complete FedAvg aggregation of K client updates (default 64 x 100 M
fp32, all resident in HBM) into a fresh aggregate: fedavg.py's fold loop
``x <- x + (n_k*(y_k - x))/N_k`` over k = 1..K-1 in queue order, as ONE libfedagg
launch. value = aggregated client-params/s = n_gpus * K * P / t_step.

Multi-GPU (torchrun, one process per GPU): every rank aggregates its own parameter
slice of P params (the global model is n_gpus * P params sharded by contiguous slice);
no collective is on the data path ("scaling": "weak"). The RCCL all-gather that would
reassemble the model on every GPU is timed separately and reported beside the line
(``allgather``), not folded into ``value``; so is the fold with that all-gather chunked
and overlapped (``fold_allgather``: block-cyclic shards, round i gathered on a
communication stream while round i+1 folds; sharded.CyclicShardedFedAvg), and the copy of
every rank's slice to host memory, FEDn's actual consumer (``gather_to_host``).

Also measured in the same run:
  roofline      algorithmic bytes (K*P*4 + P*4 per launch) / average kernel time (HIP events
                on the launch stream) vs the 8.0 TB/s HBM3E peak; ``traffic`` = HBM bytes per
                launch from rocprofv3 PMC counters (profiles/pmc_*.json, collected by
                tools/pmc_traffic.py), or null if not collected for this workload
  cpu_baseline  the numpy restatement of numpyhelper.increment_average (oracle/, bit-equal to
                FEDn) on a bounded sample (K clients x S params) on one host core; its result is
                also compared bit-for-bit with the GPU aggregate of the same elements.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "aggregated params/sec (device-resident) — FedAvg 64-client reduce, 100M fp32"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=int, default=100_000_000, help="params per GPU")
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32")
    ap.add_argument("--cpu-sample", type=int, default=100_000_000,
                    help="params per client in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--ag-rounds", type=int, default=4, help="rounds of the overlapped fold + all-gather")
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args()


def make_updates(K, P, dtype, device, seed):
    """Synthetic client updates: base ~ N(0,1), client k = base + 0.01 N(0,1)."""
    g = torch.Generator(device=device).manual_seed(seed)
    base = torch.randn(P, generator=g, device=device)
    ups = []
    for _ in range(K):
        u = torch.randn(P, generator=g, device=device).mul_(0.01).add_(base)
        ups.append(u.to(torch.bfloat16) if dtype == "bf16" else u)
    del base
    torch.cuda.synchronize(device)
    return ups


def pmc_traffic(workload):
    """HBM bytes per launch measured by rocprofv3 PMC (tools/pmc_traffic.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            ent = json.load(f).get(workload)
    except (OSError, ValueError):
        return None
    return None if ent is None else ent["bytes"]


def cpu_baseline(ups, ns, agg, S):
    """Time the oracle (numpy, 1 core) on a K x S sample and check the GPU result on it."""
    from oracle import numpy_ref as ref  # test infrastructure: the baseline/checker only

    S = min(S, agg.numel())
    sample = [u[:S].float().cpu().numpy() for u in ups]
    t0 = time.perf_counter()
    want = ref.fedavg_flat(sample, ns)
    dt = time.perf_counter() - t0
    got = agg[:S].cpu().numpy()
    exact = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
    return {"value": len(ups) * S / dt, "unit": "params/s", "cores": 1, "kind": "port",
            "sample": f"{len(ups)} clients x {S} fp32 params (first {S} of each client buffer); "
                      f"numpy {np.__version__} oracle/numpy_ref.fedavg_flat, single-threaded, "
                      f"{os.cpu_count()} host cores present", "seconds": dt,
            "gpu_bit_exact_on_sample": exact}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
    # FEDN_AMD_BENCH_ONE_GPU=1: rehearsal of the N>1 code path on a one-GPU box (every rank on
    # cuda:0, gloo instead of RCCL); never used for reported numbers
    rehearsal = os.environ.get("FEDN_AMD_BENCH_ONE_GPU") == "1"
    device = torch.device("cuda", 0 if rehearsal else local)
    torch.cuda.set_device(device)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    from fedn_amd import _abi, ops
    from fedn_amd.sharded import CyclicShardedFedAvg, ShardedFedAvg
    _abi.load()

    K = a.clients
    sh = ShardedFedAvg(a.params * world)          # global model = world x params, one slice per rank
    P = sh.hi - sh.lo                             # this rank's slice (4 KiB-aligned bounds)
    P_total = a.params * world
    cyc = None
    if world > 1 and not a.no_allgather:
        cyc = CyclicShardedFedAvg(P_total, chunk=-(-P_total // (world * a.ag_rounds)))
    L = max(P, cyc.local_len) if cyc else P
    ups_full = make_updates(K, L, a.dtype, device, a.seed + 1000 * rank)
    ups = [u[:P] for u in ups_full]
    ns = [int(v) for v in np.random.default_rng(a.seed).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    agg = torch.empty(P, dtype=torch.float32, device=device)
    stream = torch.cuda.current_stream(device)

    def step():
        ops.fedavg_fold(agg, ups, ns, Ns, init=True, stream=stream)

    for _ in range(a.warmup):
        step()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        step()
        e.record(stream)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(s.elapsed_time(e) for s, e in ev) / a.steps
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cpu" if rehearsal else device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])

    in_bytes = 2 if a.dtype == "bf16" else 4
    alg_bytes = K * P * in_bytes + P * 4           # read every update once, write the aggregate once
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9
    workload = f"fedavg_k{K}_p{P}_{a.dtype}"

    def measure_allgather():
        gather_src = agg.cpu() if rehearsal else agg
        for _ in range(2):
            full = sh.allgather(gather_src)
        del full
        torch.cuda.synchronize(device)
        dist.barrier()
        t1 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            full = sh.allgather(gather_src)
            del full
        torch.cuda.synchronize(device)
        ag = torch.tensor([(time.perf_counter() - t1) / reps], dtype=torch.float64,
                          device="cpu" if rehearsal else device)
        dist.all_reduce(ag, op=dist.ReduceOp.MAX)
        ag_s = float(ag[0])
        nbytes = sh.shard * world * 4
        return {"ms": ag_s * 1e3, "bytes_in_per_rank": sh.shard * (world - 1) * 4,
                "algbw_GBps": nbytes / ag_s / 1e9, "busbw_GBps": nbytes * (world - 1) / world / ag_s / 1e9,
                "backend": "gloo (rehearsal)" if rehearsal else "rccl",
                "note": "reassembles the world*params model on every GPU; not in value"}

    def measure_fold_allgather():
        agg_c = torch.empty(cyc.local_len, dtype=torch.float32, device=device)
        ups_c = [u[:cyc.local_len] for u in ups_full]
        out_c = None if rehearsal else torch.empty(cyc.full_len, dtype=torch.float32, device=device)
        for _ in range(2):
            cyc.fold_allgather(agg_c, ups_c, ns, Ns, init=True, out=out_c)
        torch.cuda.synchronize(device)
        dist.barrier()
        t1 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            cyc.fold_allgather(agg_c, ups_c, ns, Ns, init=True, out=out_c)
        torch.cuda.synchronize(device)
        fa = torch.tensor([(time.perf_counter() - t1) / reps], dtype=torch.float64,
                          device="cpu" if rehearsal else device)
        dist.all_reduce(fa, op=dist.ReduceOp.MAX)
        fa_s = float(fa[0])
        return {"ms": fa_s * 1e3, "value": K * P_total / fa_s, "unit": "params/s", "rounds": cyc.rounds,
                "chunk": cyc.C, "backend": "gloo (rehearsal)" if rehearsal else "rccl",
                "note": "fold + all-gather of each folded round overlapped on a second stream "
                        "(block-cyclic shards); the world*params model on every GPU; not in value"}

    def side(fn):
        """A beside-the-line measurement: an error is reported in its field, never instead of value."""
        try:
            return fn()
        except Exception as e:  # noqa: BLE001
            return {"error": f"{type(e).__name__}: {e}"}

    allgather = side(measure_allgather) if world > 1 and not a.no_allgather else None
    fold_ag = side(measure_fold_allgather) if cyc is not None else None

    # the model to the host, FEDn's consumer (roundhandler.py:465-468): every rank D2H's its own
    # slice over its own PCIe link into pinned memory, concurrently (SURVEY.md §5 alternative to
    # the all-gather); value excludes it
    host = torch.empty(P, dtype=torch.float32, pin_memory=True)
    for _ in range(2):
        host.copy_(agg, non_blocking=True)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        host.copy_(agg, non_blocking=True)
    torch.cuda.synchronize(device)
    gh = torch.tensor([(time.perf_counter() - t1) / reps], dtype=torch.float64, device="cpu" if rehearsal else device)
    if world > 1:
        dist.all_reduce(gh, op=dist.ReduceOp.MAX)
    gh_s = float(gh[0])
    gather_host = {"ms": gh_s * 1e3, "bytes_per_rank": P * 4, "GBps_aggregate": world * P * 4 / gh_s / 1e9,
                   "note": "each rank D2H's its slice of the aggregate into pinned host memory, all ranks "
                           "concurrently over their own links; max over ranks; not in value"}
    del host

    base = None
    if rank == 0 and world == 1 and a.cpu_sample > 0:
        base = cpu_baseline(ups, ns, agg, a.cpu_sample)

    if rank == 0:
        line = {
            "metric": METRIC, "value": K * P_total / (elapsed / a.steps), "unit": "params/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
            "data": "synthetic: base~N(0,1), client=base+0.01*N(0,1), num_examples~U{1..5000}, device-resident",
            "config": {"workload": f"FedAvg {K} clients x {a.params} params {a.dtype} per GPU (BASELINE configs[1]/north "
                                   "star; device-resident, one fused fold launch per aggregation)",
                       "clients": K, "params_per_gpu": a.params, "global_params": P_total,
                       "parallelism": f"param-slice shards x{world}, no data-path collective"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(workload),
                         "kernel": "k_fedavg_pipe (fp32, 4 x 16-B strips per lane, next client prefetched)", "kernel_ms": kern_ms,
                         "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": base,
        }
        line["gather_to_host"] = gather_host
        if allgather:
            line["allgather"] = allgather
        if fold_ag:
            line["fold_allgather"] = fold_ag
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
