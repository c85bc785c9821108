"""Server-function aggregation rules on MI355X. One JSON line per mode.

  wsum_device   fa_weighted_sum, K clients x P fp32 in HBM, one call (chunks of 64 clients):
                bytes K*P*4 + 2*P*4 (accumulator read + written per chunk)
  runmean_device fa_running_mean, one client step over P fp32: bytes 3*P*4
  wavg_host     serverfunctions.WeightedAverage.aggregate on host numpy updates (pack, H2D,
                fold on arrival, divide, D2H) vs the reference example's numpy loop (oracle)
  inc_host      serverfunctions.IncrementalAverage over the same updates vs the example
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fedn_amd import _abi, ops  # noqa: E402
from fedn_amd.serverfunctions import IncrementalAverage, WeightedAverage  # noqa: E402
from tools.microbench import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--host-clients", type=int, default=16)
    ap.add_argument("--host-params", type=int, default=25_000_000)
    a = ap.parse_args()
    _abi.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K, P = a.clients, a.params
    g = torch.Generator(device=dev).manual_seed(0)
    ups = [torch.randn(P, generator=g, device=dev) for _ in range(K)]
    w = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
    acc = torch.zeros(P, device=dev)
    med, best = timed(lambda: ops.weighted_sum(acc, ups, w))
    by = K * P * 4 + 2 * P * 4
    print(json.dumps({"mode": "wsum_device", "K": K, "P": P, "ms": med, "GBps": by / med / 1e6,
                      "best_GBps": by / best / 1e6, "params_per_s": K * P / med * 1e3}), flush=True)
    gm = torch.randn(P, generator=g, device=dev)
    med, best = timed(lambda: ops.running_mean(gm, ups[0], 1000, 17, 1017))
    print(json.dumps({"mode": "runmean_device", "P": P, "ms": med, "GBps": 3 * P * 4 / med / 1e6,
                      "best_GBps": 3 * P * 4 / best / 1e6}), flush=True)
    del ups, acc, gm
    torch.cuda.empty_cache()

    from oracle import numpy_ref as ref   # test infrastructure: the CPU baseline / checker only
    Kh, Ph = a.host_clients, a.host_params
    rng = np.random.default_rng(1)
    prev = [rng.standard_normal(Ph).astype(np.float32)]
    host = {f"c{k}": [[(prev[0] + np.float32(0.01) * rng.standard_normal(Ph, dtype=np.float32))],
                      {"num_examples": int(rng.integers(1, 5001))}] for k in range(Kh)}
    wa = WeightedAverage(device=dev)
    wa.aggregate(prev, host)                                   # warm (pinned slots, pinned cache)
    t0 = time.perf_counter()
    got = wa.aggregate(prev, host)
    t_gpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    want = ref.sf_weighted_average(prev, {k: (v[0], v[1]) for k, v in host.items()})
    t_cpu = time.perf_counter() - t0
    exact = bool(np.array_equal(got[0].view(np.uint32), want[0].view(np.uint32)))
    print(json.dumps({"mode": "wavg_host", "K": Kh, "P": Ph, "s": t_gpu, "GBps_in": Kh * Ph * 4 / t_gpu / 1e9,
                      "cpu_example_s": t_cpu, "speedup": t_cpu / t_gpu, "bit_exact": exact,
                      "timings": wa.timings}), flush=True)

    def run_inc(sf, copy):
        for cid, (u, md) in host.items():
            sf.incremental_aggregate(cid, [x.copy() for x in u] if copy else u, md, prev)
        return sf.get_incremental_aggregate_model()

    inc = IncrementalAverage(device=dev)
    run_inc(inc, False)
    inc = IncrementalAverage(device=dev)
    t0 = time.perf_counter()
    got = run_inc(inc, False)
    t_gpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    want = run_inc(ref.SfIncrementalAverage(), True)
    t_cpu = time.perf_counter() - t0
    exact = bool(np.array_equal(got[0].view(np.uint32), want[0].view(np.uint32)))
    print(json.dumps({"mode": "inc_host", "K": Kh, "P": Ph, "s": t_gpu, "GBps_in": Kh * Ph * 4 / t_gpu / 1e9,
                      "cpu_example_s": t_cpu, "speedup": t_cpu / t_gpu, "bit_exact": exact}), flush=True)


if __name__ == "__main__":
    main()
