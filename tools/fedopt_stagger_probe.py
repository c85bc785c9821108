"""Probe: does the placement of the FedOpt kernel's 38 concurrent streams (32 client buffers, old,
m, v in; m, v, out out) in HBM change its time? Each buffer is carved out of its own allocation at
a different byte offset (buffer j at j * stride) so that the same element index of different
buffers falls on different channels / banks. BASELINE configs[3] steady state (fp64 state)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402


def alloc(n, dtype, off, dev):
    isz = torch.empty(0, dtype=dtype).element_size()
    raw = torch.empty(n * isz + off, dtype=torch.uint8, device=dev)
    return raw[off:off + n * isz].view(dtype)


def main():
    _abi.load()
    dev = torch.device("cuda", 0)
    P, K = 350_000_000, 32
    g = torch.Generator(device=dev).manual_seed(4)
    ns = [int(v) for v in np.random.default_rng(4).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    res = {}
    for rep in range(2):
        for stride in (0, 4096, 65536, 1 << 20 | 4096, 12288):
            torch.cuda.empty_cache()
            j = iter(range(100))
            ups = [alloc(P, torch.float32, next(j) * stride, dev) for _ in range(K)]
            for u in ups:
                u.normal_(generator=g)
            old = alloc(P, torch.float64, next(j) * stride, dev).normal_(generator=g)
            m = alloc(P, torch.float64, next(j) * stride, dev).normal_(generator=g).mul_(1e-3)
            v = alloc(P, torch.float64, next(j) * stride, dev).uniform_(generator=g).mul_(1e-4)
            mo = alloc(P, torch.float64, next(j) * stride, dev)
            vo = alloc(P, torch.float64, next(j) * stride, dev)
            out = alloc(P, torch.float64, next(j) * stride, dev)
            fn = lambda: ops.fedopt_step(old, ups, ns, Ns, first=True, final=True, m_in=m, m_out=mo, v_in=v,  # noqa: E731
                                         v_out=vo, out=out)
            fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(7)]
            for s_, e_ in ev:
                s_.record()
                fn()
                e_.record()
            torch.cuda.synchronize()
            ms = sorted(s_.elapsed_time(e_) for s_, e_ in ev)[3]
            res.setdefault(stride, []).append(ms)
            del ups, old, m, v, mo, vo, out
    b = P * (4 * K + 48)
    for stride, mss in res.items():
        ms = float(np.median(mss))
        print(json.dumps({"stride": stride, "ms": ms, "GBps_alg": b / ms / 1e6, "frac": b / ms / 1e6 / 8000, "reps": mss}))


if __name__ == "__main__":
    main()
