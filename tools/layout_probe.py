"""Does the device layout of a round's client updates change the fold rate?

64 x 100 M fp32 (the BASELINE workload), device-resident, default kernel. Layouts:
  separate   one allocation per update (as bench.py; what arrivals produce by default)
  slab+pad   one [K, P + pad] allocation, update k at byte offset k * (4P + pad)
For each: the fold (fa_fedavg_fold) and the read-only traversal (stream_sum, store suppressed).
The staging path (fedn_amd/staging.py) allocates the round buffer itself, so a layout that
reads faster can be adopted there without changing any numerics.
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


def run(name, bufs, out, ns, Ns, K, P, ref):
    by = K * P * 4 + P * 4
    ops.tune(sum_nostore=1)
    med_r, _ = timed(lambda: ops.stream_sum(out, bufs), reps=10)
    ops.tune(sum_nostore=0)
    med, best = timed(lambda: ops.fedavg_fold(out, bufs, ns, Ns, init=True), reps=20)
    torch.cuda.synchronize()
    same = None if ref is None else bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
    print(json.dumps({"layout": name, "fold_ms": med, "fold_GBps": by / med / 1e6, "fold_best_GBps": by / best / 1e6,
                      "read_only_GBps": K * P * 4 / med_r / 1e6, "identical": same}), flush=True)
    return out.clone() if ref is None else ref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--pads", default="0,256,1024,4096,4352,65536,65792,1048576,2097152,2101248,3145728")
    a = ap.parse_args()
    _abi.use_probe()
    torch.cuda.set_device(0)
    K, P = a.clients, a.params
    g = torch.Generator(device="cuda").manual_seed(0)
    base = torch.randn(P, generator=g, device="cuda")
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    out = torch.empty(P, device="cuda")
    bufs = [torch.randn(P, generator=g, device="cuda").mul_(0.01).add_(base) for _ in range(K)]
    ref = run("separate", bufs, out, ns, Ns, K, P, None)
    host_src = bufs
    for pad in [int(x) for x in a.pads.split(",")]:
        assert pad % 16 == 0
        stride = P * 4 + pad
        slab = torch.empty(K * stride, dtype=torch.uint8, device="cuda")
        views = [slab[k * stride:k * stride + P * 4].view(torch.float32) for k in range(K)]
        for v, s in zip(views, host_src):
            v.copy_(s)
        run(f"slab+{pad}", views, out, ns, Ns, K, P, ref)
        del views, slab
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
