"""The fold kernel across sizes (product library): FedAvg over K device-resident updates of P
params, fp32 and bf16 (f32 aggregate), K = 2 ... 64, P = 1 M ... 100 M; and the fused FedAdam
step (fp32 updates, fp64 state) over K = 4 ... 32 at P = 10 M and 100 M. HIP-event time per
launch (median of 10), algorithmic GB/s and fraction of the 8 TB/s peak. Working sets under
~256 MB can be served partly from the Infinity Cache (marked "mall_possible")."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from tools.microbench import timed  # noqa: E402

PEAK = 8000.0


def main():
    _abi.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(9)
    rng = np.random.default_rng(9)
    for P in (1_000_000, 10_000_000, 100_000_000):
        base = torch.randn(P, generator=g, device=dev)
        ups32 = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(base) for _ in range(64)]
        for dt in ("f32", "bf16"):
            ups = ups32 if dt == "f32" else [u.to(torch.bfloat16) for u in ups32]
            agg = torch.empty(P, device=dev)
            for K in (2, 4, 8, 16, 32, 64):
                ns = [int(v) for v in rng.integers(1, 5001, K)]
                Ns = [int(v) for v in np.cumsum(ns)]
                ms, _ = timed(lambda: ops.fedavg_fold(agg, ups[:K], ns, Ns, init=True), reps=10, warm=2)
                b = K * P * (4 if dt == "f32" else 2) + P * 4
                print(json.dumps({"kernel": "fedavg", "dtype": dt, "K": K, "P": P, "ms": ms, "GBps": b / ms / 1e6,
                                  "frac": b / ms / 1e6 / PEAK, "mall_possible": b < 256e6}), flush=True)
            if dt == "bf16":
                del ups
        if P >= 10_000_000:
            old = base.double()
            m = torch.zeros(P, dtype=torch.float64, device=dev)
            v = torch.full((P,), 1e-8, dtype=torch.float64, device=dev)
            mo, vo, out = torch.empty_like(m), torch.empty_like(v), torch.empty_like(old)
            for K in (4, 8, 16, 32):
                ns = [int(v_) for v_ in rng.integers(1, 5001, K)]
                Ns = [int(v_) for v_ in np.cumsum(ns)]
                ms, _ = timed(lambda: ops.fedopt_step(old, ups32[:K], ns, Ns, first=True, final=True, m_in=m, m_out=mo,
                                                      v_in=v, v_out=vo, out=out), reps=10, warm=2)
                b = P * (4 * K + 48)
                print(json.dumps({"kernel": "fedadam_steady", "dtype": "f32 updates, f64 state", "K": K, "P": P, "ms": ms,
                                  "GBps": b / ms / 1e6, "frac": b / ms / 1e6 / PEAK, "mall_possible": b < 256e6}),
                      flush=True)
            del old, m, v, mo, vo, out
        del ups32, base
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
