"""A/B of the fold kernel's workgroup -> tile order (fa_tune FA_TUNE_TILEMAP) on MI355X.

0 identity (consecutive tiles on different XCDs), R > 0 runs of R consecutive tiles per
XCD. Interleaved repetitions, median per map; the aggregates must be bit-identical across
maps. fp32 K = 64 and 8, bf16 K = 64.

Run on the GPU box:  python tools/tilemap_probe.py [--reps 5]
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


MAPS = (0, 2, 4, 8, 16, 32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    _abi.use_probe()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    P = a.params
    g = torch.Generator(device=dev).manual_seed(0)
    base = torch.randn(P, generator=g, device=dev)
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(base) for _ in range(64)]
    del base
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, 64)]
    for K, dt in ((64, "f32"), (8, "f32"), (64, "bf16")):
        if dt == "bf16":
            ups = [u.to(torch.bfloat16) for u in ups]
        Ns = [int(v) for v in np.cumsum(ns[:K])]
        agg = torch.empty(P, dtype=torch.float32, device=dev)
        ref = None
        res = {m: [] for m in MAPS}
        for _ in range(a.reps):
            for m in MAPS:
                ops.tune(tilemap=m)
                med, _best = timed(lambda: ops.fedavg_fold(agg, ups[:K], ns[:K], Ns, init=True))
                res[m].append(med)
                if ref is None:
                    ref = agg.clone()
                elif not torch.equal(agg.view(torch.int32), ref.view(torch.int32)):
                    raise SystemExit(f"tilemap {m}: aggregate differs")
        ops.tune(tilemap=0)
        nbytes = K * P * (2 if dt == "bf16" else 4) + P * 4
        for m, ts in res.items():
            med = float(np.median(ts))
            print(json.dumps({"K": K, "dtype": dt, "tilemap": m, "ms": med, "GBps": nbytes / med / 1e6,
                              "frac": nbytes / med / 1e6 / 8000.0, "runs_ms": [round(t, 4) for t in ts]}), flush=True)


if __name__ == "__main__":
    main()
