"""Element-map probe for configs[4]'s wave kernels (libfedagg_probe.so, FA_TUNE_OPT_QUAD): the
product's k_fedopt_c (lane L owns the pairs {2L, 2L+1} + 128 j: a bf16 client load is one dword per
lane) against k_fedopt_cq (lane L owns the quads {4L .. 4L+3} + 256 j: one dwordx2 per lane; the
fp64 streams take two dwordx4 per strip). 1 B params, 8 bf16 updates device-resident, FedYogi round
1 as the waves run it: the FIRST wave, a later wave, the last wave with the server step fused.
Interleaved repeats, median per setting; pg and out must be bit-identical.

    python tools/wave_quad_probe.py [--params 1000000000] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402

HBM = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=1_000_000_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    _abi.use_probe()
    dev = torch.device("cuda", 0)
    P, W = a.params, 8
    g = torch.Generator(device=dev).manual_seed(5)
    old = torch.randn(P, generator=g, device=dev, dtype=torch.float64)
    ups = [(old + 0.01 * torch.randn(P, generator=g, device=dev, dtype=torch.float64)).to(torch.bfloat16)
           for _ in range(W)]
    ns = [int(v) for v in np.random.default_rng(5).integers(1, 5001, W)]
    Ns = [int(v) for v in np.cumsum(ns)]
    Ns2 = [N + Ns[-1] for N in Ns]
    pg = {q: torch.empty(P, dtype=torch.float64, device=dev) for q in (0, 1)}
    st = {q: [torch.empty(P, dtype=torch.float64, device=dev) for _ in range(3)] for q in (0, 1)}

    def first(q):
        ops.fedopt_step(old, ups, ns, Ns, first=True, final=False, pg=pg[q])

    def mid(q):
        ops.fedopt_step(old, ups, ns, Ns2, first=False, final=False, pg=pg[q])

    def last(q):
        m, v, o = st[q]
        ops.fedopt_step(old, ups, ns, Ns2, first=False, final=True, pg=pg[q], m_out=m, v_out=v, out=o,
                        serveropt="yogi")

    kinds = {"first": (first, 2 * W + 16), "mid": (mid, 2 * W + 24), "mid_final": (last, 2 * W + 40)}
    res = {(k, q): [] for k in kinds for q in (0, 1)}
    for _ in range(a.reps):
        for kind, (fn, per_el) in kinds.items():
            for q in (0, 1):
                ops.tune(opt_quad=q)
                fn(q)                                   # warm
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn(q)
                e1.record()
                torch.cuda.synchronize()
                res[(kind, q)].append(e0.elapsed_time(e1))
    ops.tune(opt_quad=0)
    # bit identity: the same sequence under both maps
    outs = {}
    for q in (0, 1):
        ops.tune(opt_quad=q)
        first(q)
        mid(q)
        p_mid = pg[q].clone()
        last(q)
        torch.cuda.synchronize()
        outs[q] = (p_mid, *st[q])
    ops.tune(opt_quad=0)
    same = all(torch.equal(x.view(torch.int64), y.view(torch.int64)) for x, y in zip(outs[0], outs[1]))
    for kind, (fn, per_el) in kinds.items():
        for q in (0, 1):
            ms = float(np.median(res[(kind, q)]))
            b = P * per_el
            print(json.dumps({"kind": kind, "map": "quad" if q else "pairs (product)", "ms": round(ms, 3),
                              "frac": round(b / ms / 1e6 / HBM, 4), "runs_ms": [round(t, 3) for t in res[(kind, q)]]}),
                  flush=True)
    print(json.dumps({"bit_identical": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
