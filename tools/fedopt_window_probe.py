"""FedAdam (configs[3] shapes) through the product step with and without the chip-wide store window
(k_fedopt_cw vs k_fedopt_c; fa_tune OPT_WIN_PERIOD -1 = no window, 0 = the product's own
opt_store_window, > 0 with OPT_WIN_PROD = 1 = an explicit period / window): round 1 (fp32 model)
and the fp64 steady state, bit-for-bit against the unwindowed step, interleaved repeats, median ms.
Probe library.

  python tools/fedopt_window_probe.py [--clients 8,16,32] [--params N] [--winprod period:w,...]
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
    ap.add_argument("--params", type=int, default=2048 * 170898)
    ap.add_argument("--clients", default="32,16,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--winprod", default="3000:450,4500:680,6000:900,8192:1200")
    ap.add_argument("--wincg", default="", help="the compute-then-store kernel k_fedopt_cgw (OPT_WIN_PROD 2): period:w,...")
    ap.add_argument("--wpe", default="", help="also the --winprod windows compiled for W waves per SIMD: W,...")
    ap.add_argument("--wincw2", default="", help="the windowed step on 256-element wave tiles (OPT_WIN_PROD 3): period:w,...")
    a = ap.parse_args()
    _abi.use_probe()
    dev = torch.device("cuda", 0)
    P = a.params
    explicit = [tuple(int(v) for v in x.split(":")) for x in a.winprod.split(",") if x]
    cg = [tuple(int(v) for v in x.split(":")) for x in a.wincg.split(",") if x]
    wpes = [int(x) for x in a.wpe.split(",") if x]
    cw2 = [tuple(int(v) for v in x.split(":")) for x in a.wincw2.split(",") if x]
    g = torch.Generator(device=dev).manual_seed(4)
    old32 = torch.randn(P, generator=g, device=dev)
    Kmax = max(int(k) for k in a.clients.split(","))
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(old32) for _ in range(Kmax)]
    out = torch.empty(P, dtype=torch.float64, device=dev)
    v = torch.empty(P, dtype=torch.float64, device=dev)
    m32 = torch.empty(P, dtype=torch.float32, device=dev)
    m_o = torch.empty(P, dtype=torch.float64, device=dev)
    v_o = torch.empty(P, dtype=torch.float64, device=dev)
    o2 = torch.empty(P, dtype=torch.float64, device=dev)

    def variants(phase=None):
        yield "nowin", dict(opt_win_period=-1, opt_win_prod=0, wpe=0)
        yield "product", dict(opt_win_period=0, opt_win_prod=0, wpe=0)
        for p_, w_ in explicit:
            yield f"win{p_}_{w_}", dict(opt_win_period=p_, opt_win_w=w_, opt_win_prod=1, wpe=0)
            for W in wpes:
                yield f"win{p_}_{w_}_wpe{W}", dict(opt_win_period=p_, opt_win_w=w_, opt_win_prod=1, wpe=W)
        for p_, w_ in cw2:
            yield f"cw2_{p_}_{w_}", dict(opt_win_period=p_, opt_win_w=w_, opt_win_prod=3, wpe=0)
        for p_, w_ in cg if phase == "steady" else ():      # fp64 m / v / model out only
            yield f"cgw{p_}_{w_}", dict(opt_win_period=p_, opt_win_w=w_, opt_win_prod=2, wpe=0)

    for K in (int(k) for k in a.clients.split(",")):
        ns = [int(x) for x in np.random.default_rng(K).integers(1, 5001, K)]
        Ns = [int(x) for x in np.cumsum(ns)]
        ops.tune(opt_win_period=-1)
        ops.fedopt_step(old32, ups[:K], ns, Ns, first=True, final=True, m_out=m32, v_out=v, out=out)
        old64, m64, v64 = out.clone(), m32.double(), v.clone()
        phases = {
            "round1": (lambda: ops.fedopt_step(old32, ups[:K], ns, Ns, first=True, final=True, m_out=m32, v_out=v, out=out),
                       K * P * 4 + P * 24, (out, m32, v)),
            "steady": (lambda: ops.fedopt_step(old64, ups[:K], ns, Ns, first=True, final=True, m_in=m64, m_out=m_o,
                                               v_in=v64, v_out=v_o, out=o2), P * (4 * K + 48), (o2, m_o, v_o)),
        }
        for name, (fn, alg, outs) in phases.items():
            ops.tune(opt_win_period=-1, opt_win_prod=0)
            fn()
            torch.cuda.synchronize()
            ref = [t.clone() for t in outs]
            exact = {}
            for vn, kn in variants(name):
                ops.tune(**kn)
                for t in outs:
                    t.zero_()
                fn()
                torch.cuda.synchronize()
                exact[vn] = all(torch.equal(x.view(torch.uint8), y.view(torch.uint8)) for x, y in zip(outs, ref))
            res = {}
            for _ in range(a.reps):
                for vn, kn in variants(name):
                    ops.tune(**kn)
                    fn()
                    res.setdefault(vn, []).append(median_ms(fn))
            ops.tune(opt_win_period=0, opt_win_prod=0, wpe=0)
            line = {"clients": K, "phase": name, "params": P, "alg_bytes": alg}
            for vn in res:
                ms = float(np.median(res[vn]))
                line[vn] = {"ms": round(ms, 4), "frac_of_peak": round(alg / ms / 1e6 / PEAK, 4), "bit_exact": exact[vn]}
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
