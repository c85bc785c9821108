"""Layout probe for the FedOpt steady state (libfedagg_probe.so, FA_TUNE_OPT_MV): m and v as two
fp64 buffers (the product) against ONE buffer holding both, interleaved per 512-element wave tile
([m of tile w | v of tile w]), so the kernel reads one state stream and writes one instead of two.
configs[3] shape (32 fp32 updates, P = 350,001,152 = a multiple of the 2048-element workgroup
tile). Interleaved repeats, median per setting; out, m and v must be bit-identical."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from tools.microbench import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=350_001_152)
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    assert a.params % 2048 == 0
    _abi.use_probe()
    dev = torch.device("cuda", 0)
    P, K, T = a.params, a.clients, 512
    g = torch.Generator(device=dev).manual_seed(6)
    old32 = torch.randn(P, generator=g, device=dev)
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(old32) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(6).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    out1 = torch.empty(P, dtype=torch.float64, device=dev)
    v1 = torch.empty(P, dtype=torch.float64, device=dev)
    m1 = torch.empty(P, dtype=torch.float32, device=dev)
    ops.fedopt_step(old32, ups, ns, Ns, first=True, final=True, m_out=m1, v_out=v1, out=out1)
    old64, m64 = out1, m1.double()
    del old32, m1
    # the interleaved state: [m tile | v tile] per 512 elements
    mv_in = torch.stack([m64.view(-1, T), v1.view(-1, T)], dim=1).reshape(-1).contiguous()
    mv_out = torch.empty_like(mv_in)
    m_o = torch.empty(P, dtype=torch.float64, device=dev)
    v_o = torch.empty(P, dtype=torch.float64, device=dev)
    o_a = torch.empty(P, dtype=torch.float64, device=dev)
    o_b = torch.empty(P, dtype=torch.float64, device=dev)

    def sep():
        ops.fedopt_step(old64, ups, ns, Ns, first=True, final=True, m_in=m64, m_out=m_o, v_in=v1, v_out=v_o, out=o_a)

    def mv():
        # m_in / m_out carry the 2P-double interleaved buffers (views of their first P for the size
        # check); v_in / v_out are required non-null but not read or written by the probe kernel
        ops.fedopt_step(old64, ups, ns, Ns, first=True, final=True, m_in=mv_in[:P], m_out=mv_out[:P], v_in=v1,
                        v_out=v_o, out=o_b)

    res = {"separate": [], "interleaved": []}
    for _ in range(a.reps):
        ops.tune(opt_mv=0)
        res["separate"].append(timed(sep, reps=5, warm=1)[0])
        ops.tune(opt_mv=1)
        res["interleaved"].append(timed(mv, reps=5, warm=1)[0])
    ops.tune(opt_mv=0)
    sep()
    ops.tune(opt_mv=1)
    mv()
    ops.tune(opt_mv=0)
    torch.cuda.synchronize()
    mo = mv_out.view(-1, 2, T)
    same = (torch.equal(o_a.view(torch.int64), o_b.view(torch.int64)) and
            torch.equal(m_o.view(-1, T).view(torch.int64), mo[:, 0].contiguous().view(torch.int64)) and
            torch.equal(v_o.view(-1, T).view(torch.int64), mo[:, 1].contiguous().view(torch.int64)))
    b = P * (4 * K + 48)
    for name, ts in res.items():
        ms = float(np.median(ts))
        print(json.dumps({"state_layout": name, "ms": ms, "GBps": b / ms / 1e6, "frac": b / ms / 1e6 / 8000.0,
                          "runs_ms": [round(t, 4) for t in ts]}), flush=True)
    print(json.dumps({"bit_identical": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
