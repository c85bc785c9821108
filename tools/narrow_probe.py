"""A/B of the bf16 -> f32 FedAvg element map (fa_tune FA_TUNE_NARROW) on MI355X.

0: 16-B client strips of 8 bf16, so each lane's 8 f32 results leave as two 16-B stores 32 B
apart (every wave store instruction covers half of each 128-B line over 2 KiB).
1: 8-B client strips of 4 bf16 and 16-B aggregate strips, 8 per lane (every wave load is one
contiguous 512 B, every wave store one contiguous 1 KiB). Interleaved repetitions, median per
setting; aggregates must be bit-identical. libfedagg_probe.so only.

Run on the GPU box:  python tools/narrow_probe.py [--reps 5]
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
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(base).to(torch.bfloat16) for _ in range(64)]
    del base
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, 64)]
    for K, init in ((64, True), (8, True), (8, False)):
        Ns = [int(v) for v in np.cumsum(ns[:K])]
        agg = torch.empty(P, dtype=torch.float32, device=dev)
        start = torch.randn(P, generator=g, device=dev)
        ref = None
        res = {0: [], 1: []}

        def run():
            if not init:
                agg.copy_(start)
            ops.fedavg_fold(agg, ups[:K], ns[:K], Ns, init=init)

        for _ in range(a.reps):
            for m in (0, 1):
                ops.tune(narrow=m)
                med, _best = timed(run)     # init=False: the copy is timed too, subtracted below
                res[m].append(med)
                if ref is None:
                    ref = agg.clone()
                elif not torch.equal(agg.view(torch.int32), ref.view(torch.int32)):
                    raise SystemExit(f"narrow {m}: aggregate differs")
        ops.tune(narrow=1)
        cp = float(np.median([timed(lambda: agg.copy_(start))[0] for _ in range(3)])) if not init else 0.0
        nbytes = K * P * 2 + P * 4 + (0 if init else P * 4)
        for m, ts in res.items():
            med = float(np.median(ts)) - cp
            print(json.dumps({"K": K, "init": init, "narrow": m, "ms": med, "GBps": nbytes / med / 1e6,
                              "frac": nbytes / med / 1e6 / 8000.0, "runs_ms": [round(t, 4) for t in ts],
                              "copy_ms_subtracted": cp}), flush=True)
    print(json.dumps({"bit_identical": True}))


if __name__ == "__main__":
    main()
