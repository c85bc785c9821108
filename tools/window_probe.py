"""FedAvg's fold with its stores confined to a chip-wide clock window (fa_tune AVG_WIN_*, probe
library): the BASELINE workload (64 x 100 M fp32, device-resident, one launch) and configs[1]
(8 x 100 M), the product kernel k_fedavg_pipe against the same body whose stores wait for
clock mod period < window (and, mode >= 1 / 2, whose reads start / continue outside it).
Interleaved repeats, median ms; each variant's result compared bit for bit with the product's.

  python tools/window_probe.py [--win K:period:window:mode,...]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402

PEAK = 8000.0


def median_ms(fn, n=5):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for s_, e_ in ev:
        s_.record()
        fn()
        e_.record()
    torch.cuda.synchronize()
    return sorted(s_.elapsed_time(e_) for s_, e_ in ev)[n // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--clients", default="64,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dtype", default="f32", choices=("f32", "bf16"), help="the client updates' dtype")
    # K:period:window:mode (ticks of 10 ns); a round of resident workgroups reads ~K x 16 KiB each
    ap.add_argument("--win", default="64:14000:700:0,64:17000:850:0,64:20000:1000:0,64:24000:1200:0,64:17000:1700:0,"
                                     "64:17000:850:2,8:2000:250:0,8:2600:320:0,8:3200:400:0,8:4000:500:0,8:2600:520:0")
    a = ap.parse_args()
    _abi.use_probe()
    dev = torch.device("cuda", 0)
    P = a.params
    g = torch.Generator(device=dev).manual_seed(5)
    base = torch.randn(P, generator=g, device=dev)
    Kmax = max(int(k) for k in a.clients.split(","))
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(base) for _ in range(Kmax)]
    if a.dtype == "bf16":
        ups = [u.to(torch.bfloat16) for u in ups]
    del base
    allwins = [tuple(int(v) for v in x.split(":")) for x in a.win.split(",") if x]
    agg = torch.empty(P, device=dev)
    for K in (int(k) for k in a.clients.split(",")):
        wins = [w[1:] for w in allwins if w[0] == K]
        ns = [int(v) for v in np.random.default_rng(K).integers(1, 5001, K)]
        Ns = [int(v) for v in np.cumsum(ns)]
        fn = lambda: ops.fedavg_fold(agg, ups[:K], ns, Ns, True)  # noqa: E731
        alg = K * P * ups[0].element_size() + P * 4
        ops.tune(avg_win_period=-1)                       # no window: the reference bits and times
        fn()
        torch.cuda.synchronize()
        ref = agg.clone()
        exact = {}
        wins = [(0, 0, 0)] + wins                         # (0, ...): the product's own window
        for w in wins:
            ops.tune(avg_win_period=w[0], avg_win_w=w[1], avg_win_mode=w[2])
            agg.zero_()
            fn()
            torch.cuda.synchronize()
            exact[w] = bool(torch.equal(agg.view(torch.int32), ref.view(torch.int32)))
        ops.tune(avg_win_period=0)
        res = {}
        for _ in range(a.reps):
            ops.tune(avg_win_period=-1)
            fn()
            res.setdefault("product", []).append(median_ms(fn))
            for w in wins:
                ops.tune(avg_win_period=w[0], avg_win_w=w[1], avg_win_mode=w[2])
                fn()
                res.setdefault(w, []).append(median_ms(fn))
            ops.tune(avg_win_period=0)
        ops.tune(avg_win_period=0)
        prod = float(np.median(res["product"]))
        out = {"clients": K, "params": P, "dtype": a.dtype, "alg_bytes": alg, "nowin_ms": round(prod, 4),
               "nowin_frac_of_peak": round(alg / prod / 1e6 / PEAK, 4)}
        for w in wins:
            ms = float(np.median(res[w]))
            out["product_window" if w[0] == 0 else f"win{w[0]}_{w[1]}_{w[2]}"] = {"ms": round(ms, 4), "frac_of_peak": round(alg / ms / 1e6 / PEAK, 4),
                                               "bit_exact": exact[w]}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
