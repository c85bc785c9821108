"""How close the fused FedOpt kernel runs to the ceiling of its own HBM access pattern: configs[3]
(32 fp32 updates x ~350 M params, FedAdam round 1 and fp64 steady state), the product kernel
k_fedopt_c against k_fedopt_mix (fa_tune FA_TUNE_OPT_MIX: the very same loads and stores — element
map, client batching, state after the fold, non-temporal stores — with the arithmetic cut to one add
per value) and, for scale, a STREAM-style copy of one buffer. Interleaved repeats, median ms.
libfedagg_probe.so only (the mix kernel's outputs are not the reference's)."""
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
    ap.add_argument("--params", type=int, default=2048 * 170898)      # ~350 M, whole 2048-element tiles
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--burst", default="1,2,4", help="burst-store probe G values (tiles per wave), '' = none")
    ap.add_argument("--opt-g", default="1,2,4", help="product step with G tiles per wave (fa_tune OPT_G), '' = none")
    ap.add_argument("--win", default="", help="clock-windowed store probe: period_ticks:window_ticks:mode,... "
                    "(fa_tune OPT_WIN_*: stores only while the 100 MHz clock mod period < window)")
    a = ap.parse_args()
    _abi.use_probe()
    dev = torch.device("cuda", 0)
    P, K = a.params, a.clients
    g = torch.Generator(device=dev).manual_seed(4)
    old32 = torch.randn(P, generator=g, device=dev)
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(old32) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(4).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    out = torch.empty(P, dtype=torch.float64, device=dev)
    v = torch.empty(P, dtype=torch.float64, device=dev)
    m32 = torch.empty(P, dtype=torch.float32, device=dev)
    ops.fedopt_step(old32, ups, ns, Ns, first=True, final=True, m_out=m32, v_out=v, out=out)
    old64, m64, v64 = out.clone(), m32.double(), v.clone()
    m_o = torch.empty(P, dtype=torch.float64, device=dev)
    v_o = torch.empty(P, dtype=torch.float64, device=dev)
    o2 = torch.empty(P, dtype=torch.float64, device=dev)
    phases = {
        "round1": (lambda: ops.fedopt_step(old32, ups, ns, Ns, first=True, final=True, m_out=m32, v_out=v, out=out),
                   K * P * 4 + P * 24),
        "steady": (lambda: ops.fedopt_step(old64, ups, ns, Ns, first=True, final=True, m_in=m64, m_out=m_o, v_in=v64,
                                           v_out=v_o, out=o2), P * (4 * K + 48)),
    }
    src = torch.empty(1 << 30, dtype=torch.float32, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    res = {}
    bursts = [int(x) for x in a.burst.split(",") if x]
    wins = [tuple(int(v) for v in x.split(":")) for x in a.win.split(",") if x]
    gs = [int(x) for x in a.opt_g.split(",") if x]
    # the product arithmetic with G tiles per wave (fa_tune OPT_G): bit-identical to k_fedopt_c?
    exact = {}
    if gs:
        fn = phases["steady"][0]
        ops.tune(opt_g=0)
        fn()
        torch.cuda.synchronize()
        ref_out = (o2.clone(), m_o.clone(), v_o.clone())
        for g in gs:
            ops.tune(opt_g=g)
            o2.zero_(); m_o.zero_(); v_o.zero_()
            fn()
            torch.cuda.synchronize()
            exact[g] = all(torch.equal(x.view(torch.int64), y.view(torch.int64)) for x, y in zip((o2, m_o, v_o), ref_out))
        ops.tune(opt_g=0)
    for _ in range(a.reps):
        for name, (fn, _b) in phases.items():
            for mix in (0, 1):
                ops.tune(opt_mix=mix)
                fn()
                res.setdefault((name, mix), []).append(median_ms(fn))
            ops.tune(opt_mix=0)
            for g in gs:                          # the product step with G tiles per wave
                if name != "steady":
                    continue
                ops.tune(opt_g=g)
                fn()
                res.setdefault((name, f"g{g}"), []).append(median_ms(fn))
            ops.tune(opt_g=0)
            for g in bursts:                      # the burst-store probe: G tiles per wave, stores after
                if name != "steady":
                    continue
                ops.tune(opt_burst=g)
                fn()
                res.setdefault((name, f"burst{g}"), []).append(median_ms(fn))
            ops.tune(opt_burst=0)
            for lg, w, mode in wins:              # stores confined to a chip-wide clock window
                if name != "steady":
                    continue
                ops.tune(opt_win_period=lg, opt_win_w=w, opt_win_mode=mode)
                fn()
                res.setdefault((name, f"win{lg}_{w}_{mode}"), []).append(median_ms(fn))
            ops.tune(opt_win_period=0)
        ops.tune(opt_mix=0)
        ops.stream_copy(dst, src)
        res.setdefault(("copy", 0), []).append(median_ms(lambda: ops.stream_copy(dst, src)))
    ops.tune(opt_mix=0)
    copy_gbs = 2 * src.numel() * 4 / (float(np.median(res[("copy", 0)])) / 1e3) / 1e9
    for name, (_, b) in phases.items():
        prod, mix = float(np.median(res[(name, 0)])), float(np.median(res[(name, 1)]))
        print(json.dumps({"phase": name, "params": P, "clients": K, "alg_bytes": b,
                          "product_ms": round(prod, 4), "product_frac_of_peak": round(b / prod / 1e6 / PEAK, 4),
                          "pattern_ms": round(mix, 4), "pattern_frac_of_peak": round(b / mix / 1e6 / PEAK, 4),
                          "product_over_pattern": round(mix / prod, 4),
                          "product_frac_of_copy": round(b / prod / 1e6 / copy_gbs, 4),
                          "reps_product": [round(x, 4) for x in res[(name, 0)]],
                          "reps_pattern": [round(x, 4) for x in res[(name, 1)]],
                          **{f"burst{g}_ms": round(float(np.median(res[(name, f'burst{g}')])), 4)
                             for g in bursts if (name, f"burst{g}") in res},
                          **{f"burst{g}_frac_of_peak": round(b / float(np.median(res[(name, f'burst{g}')])) / 1e6 / PEAK, 4)
                             for g in bursts if (name, f"burst{g}") in res},
                          **{f"g{g}_ms": round(float(np.median(res[(name, f'g{g}')])), 4)
                             for g in gs if (name, f"g{g}") in res},
                          **{f"g{g}_reps": [round(x, 4) for x in res[(name, f'g{g}')]]
                             for g in gs if (name, f"g{g}") in res},
                          **{f"win{lg}_{w}_{m}_ms": round(float(np.median(res[(name, f'win{lg}_{w}_{m}')])), 4)
                             for lg, w, m in wins if (name, f"win{lg}_{w}_{m}") in res},
                          **({f"g{g}_bit_exact": exact[g] for g in gs} if name == "steady" else {})}), flush=True)
    print(json.dumps({"copy_GBps": round(copy_gbs, 1), "reps_ms": [round(x, 4) for x in res[("copy", 0)]]}))


if __name__ == "__main__":
    main()
