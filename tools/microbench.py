"""GPU microbenchmarks: achievable HBM rates and FedAvg launch-geometry sweep.

Runs on the GPU box:  python tools/microbench.py [--params 100000000] [--clients 64]
Prints one JSON object per line (stream_read / stream_copy / fedavg geometry).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402


def timed(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) for s, e in ev)
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--sweep", default="all")
    a = ap.parse_args()
    _abi.use_probe()
    lib = _abi.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)

    if a.sweep == "bf16":
        return bf16_sweep(a)
    # achievable-peak references
    nb = 8 << 30
    src = torch.empty(nb, dtype=torch.uint8, device=dev).random_()
    sink = ops.stream_read_sink(src)
    for rpl in (4, 8, 16):
        ops.tune(read=rpl)
        med, best = timed(lambda: ops.stream_read(src, sink))
        print(json.dumps({"kernel": f"stream_read x{rpl}/lane", "bytes": nb, "ms": med, "GBps": nb / med / 1e6,
                          "best_GBps": nb / best / 1e6}), flush=True)
    half = src[: nb // 2]
    dst = torch.empty(nb // 2, dtype=torch.uint8, device=dev)
    med, best = timed(lambda: ops.stream_copy(dst, half))
    print(json.dumps({"kernel": "stream_copy", "bytes": nb, "ms": med, "GBps": nb / med / 1e6, "best_GBps": nb / best / 1e6}), flush=True)
    med, best = timed(lambda: dst.copy_(half))
    print(json.dumps({"kernel": "torch_d2d_copy", "bytes": nb, "ms": med, "GBps": nb / med / 1e6}), flush=True)
    del src, dst, half, sink
    torch.cuda.empty_cache()

    K, P = a.clients, a.params
    g = torch.Generator(device=dev).manual_seed(0)
    base = torch.randn(P, generator=g, device=dev)
    ups = [base + 0.01 * torch.randn(P, generator=g, device=dev) for _ in range(K)]
    del base
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    agg = torch.empty(P, device=dev)
    ref_out = None
    alg = K * P * 4 + P * 4
    med, best = timed(lambda: ops.stream_sum(agg, ups))
    print(json.dumps({"kernel": "stream_sum (fold traversal, 1 add)", "ms": med, "GBps": alg / med / 1e6,
                      "best_GBps": alg / best / 1e6}), flush=True)
    combos = [(S, U, 0, 1, 0, 0, 256) for S, U in ((1, 8), (4, 1))]
    combos += [(S, 0, 0, 1, 0, 0, B) for S, B in ((4, 256), (8, 256), (4, 512), (8, 512), (2, 1024), (4, 1024))]
    for S, U, NT, F, L, G, B in combos:
                ops.tune(strips=S, unroll=U, nt=NT, fastdiv=F, lanetab=L, grid=G, block=B)
                med, best = timed(lambda: ops.fedavg_fold(agg, ups, ns, Ns, init=True))
                torch.cuda.synchronize()
                if ref_out is None:
                    ref_out = agg.clone()
                same = bool(torch.equal(agg.view(torch.int32), ref_out.view(torch.int32)))
                print(json.dumps({"kernel": "fedavg", "strips": S, "unroll": U, "nt": NT, "fastdiv": F, "lanetab": L, "grid": G, "block": B, "K": K, "P": P, "ms": med,
                                  "GBps": alg / med / 1e6, "best_GBps": alg / best / 1e6, "identical": same}), flush=True)
    # one contiguous [K, P] slab instead of K separate allocations
    slab = torch.stack(ups)
    rows = list(slab.unbind(0))
    med, _ = timed(lambda: ops.stream_sum(agg, rows))
    print(json.dumps({"kernel": "stream_sum_slab", "ms": med, "GBps": alg / med / 1e6}), flush=True)
    for S, U, L in ((4, 0, 0),):
        ops.tune(strips=S, unroll=U, lanetab=L)
        med, best = timed(lambda: ops.fedavg_fold(agg, rows, ns, Ns, init=True))
        print(json.dumps({"kernel": "fedavg_slab", "strips": S, "unroll": U, "lanetab": L, "ms": med,
                          "GBps": alg / med / 1e6}), flush=True)
    del slab, rows
    # reset defaults
    ops.tune(strips=4, unroll=0, nt=0, fastdiv=1, lanetab=0, grid=0, block=256, nt_store=1)
    # K = 8 (BASELINE config 2) and bf16 inputs
    med, _ = timed(lambda: ops.fedavg_fold(agg, ups[:8], ns[:8], Ns[:8], init=True))
    b8 = 8 * P * 4 + P * 4
    print(json.dumps({"kernel": "fedavg", "K": 8, "P": P, "ms": med, "GBps": b8 / med / 1e6}), flush=True)
    ups16 = [u.to(torch.bfloat16) for u in ups]
    del ups
    med, _ = timed(lambda: ops.fedavg_fold(agg, ups16, ns, Ns, init=True))
    bb = K * P * 2 + P * 4
    print(json.dumps({"kernel": "fedavg_bf16", "K": K, "P": P, "ms": med, "GBps": bb / med / 1e6,
                      "params_per_s": K * P / med * 1e3}), flush=True)


def bf16_sweep(a):
    """bf16 updates (half the bytes per element, same arithmetic): is the fold ALU-sensitive?"""
    K, P, dev = a.clients, a.params, torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    base = torch.randn(P, generator=g, device=dev)
    ups = [(base + 0.01 * torch.randn(P, generator=g, device=dev)).to(torch.bfloat16) for _ in range(K)]
    del base
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    agg = torch.empty(P, device=dev)
    bb = K * P * 2 + P * 4
    ref_out = None
    for S, F, B in ((4, 1, 256), (4, 0, 256), (2, 1, 256), (8, 1, 256), (2, 0, 256), (4, 1, 512)):
        ops.tune(strips=S, unroll=0, nt=0, fastdiv=F, lanetab=0, grid=0, block=B)
        med, best = timed(lambda: ops.fedavg_fold(agg, ups, ns, Ns, init=True))
        torch.cuda.synchronize()
        if ref_out is None:
            ref_out = agg.clone()
        same = bool(torch.equal(agg.view(torch.int32), ref_out.view(torch.int32)))
        print(json.dumps({"kernel": "fedavg_bf16", "strips": S, "fastdiv": F, "block": B, "ms": med,
                          "GBps": bb / med / 1e6, "best_GBps": bb / best / 1e6, "identical": same}), flush=True)
    ops.tune(strips=4, unroll=0, nt=0, fastdiv=1, lanetab=0, grid=0, block=256, nt_store=1)


if __name__ == "__main__":
    main()
