"""Occupancy A/B of the two hot kernels on MI355X (libfedagg_probe.so only).

Fewer resident workgroups per CU: FA_TUNE_LDS gives each workgroup LDS it never touches (the CU's
160 KiB then holds fewer workgroups). More waves per SIMD: FA_TUNE_WPE compiles the same body for
at least W waves (the compiler fits it into fewer VGPRs, spilling if it must). Workloads: the
headline FedAvg fold (64 x 100 M fp32) and the configs[3] FedAdam steady state (32 x 350 M, fp64
state). Interleaved repeats, median per setting; results must be bit-identical to the default.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from tools.microbench import timed  # noqa: E402

SETTINGS = [(0, 0), (40, 0), (53, 0), (64, 0), (0, 5), (0, 6), (0, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--workload", choices=["fedavg", "fedopt", "both"], default="both")
    a = ap.parse_args()
    _abi.use_probe()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    rng = np.random.default_rng(5)
    work = []
    if a.workload in ("fedavg", "both"):
        P, K = 100_000_000, 64
        base = torch.randn(P, generator=g, device=dev)
        ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(base) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 5001, K)]
        Ns = [int(v) for v in np.cumsum(ns)]
        agg = torch.empty(P, device=dev)
        work.append(("fedavg_k64_p100M", lambda: ops.fedavg_fold(agg, ups, ns, Ns, init=True), [agg], K * P * 4 + P * 4,
                     ups))
    if a.workload in ("fedopt", "both"):
        P, K = 350_000_000, 32
        old32 = torch.randn(P, generator=g, device=dev)
        oups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(old32) for _ in range(K)]
        ons = [int(v) for v in rng.integers(1, 5001, K)]
        oNs = [int(v) for v in np.cumsum(ons)]
        out = torch.empty(P, dtype=torch.float64, device=dev)
        v = torch.empty(P, dtype=torch.float64, device=dev)
        m32 = torch.empty(P, dtype=torch.float32, device=dev)
        ops.fedopt_step(old32, oups, ons, oNs, first=True, final=True, m_out=m32, v_out=v, out=out)
        old64, m64 = out.clone(), m32.double()
        del old32, m32
        m_o = torch.empty(P, dtype=torch.float64, device=dev)
        v_o = torch.empty(P, dtype=torch.float64, device=dev)
        o2 = torch.empty(P, dtype=torch.float64, device=dev)
        work.append(("fedadam_steady_k32_p350M",
                     lambda: ops.fedopt_step(old64, oups, ons, oNs, first=True, final=True, m_in=m64, m_out=m_o, v_in=v,
                                             v_out=v_o, out=o2), [m_o, v_o, o2], P * (4 * K + 48), oups))
    for name, fn, outs, nbytes, _keep in work:
        ops.tune(lds=0, wpe=0)
        fn()
        torch.cuda.synchronize()
        ref = [o.clone() for o in outs]
        res = {st: [] for st in SETTINGS}
        for _ in range(a.reps):
            for lds, wpe in SETTINGS:
                ops.tune(lds=lds, wpe=wpe)
                med, _best = timed(fn, reps=5, warm=1)
                res[(lds, wpe)].append(med)
                for o, r in zip(outs, ref):
                    if not torch.equal(o.view(torch.uint8), r.view(torch.uint8)):
                        raise SystemExit(f"{name} lds={lds} wpe={wpe}: result differs")
        ops.tune(lds=0, wpe=0)
        for (lds, wpe), ts in res.items():
            ms = float(np.median(ts))
            print(json.dumps({"workload": name, "lds_kib": lds, "wpe": wpe, "ms": ms, "GBps": nbytes / ms / 1e6,
                              "frac": nbytes / ms / 1e6 / 8000.0, "runs_ms": [round(t, 4) for t in ts]}), flush=True)
        print(json.dumps({"workload": name, "bit_identical": True}), flush=True)


if __name__ == "__main__":
    main()
