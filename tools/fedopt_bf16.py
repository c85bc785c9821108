"""Device-resident FedOpt with bf16 client updates (product library): 32 x 350 M bf16 updates,
FedAdam round 1 (fp32 old) and steady state (fp64 old / m / v), plus the non-final wave fold
configs[4] runs (8 bf16 updates into an fp32 pseudo-gradient in HBM). HIP-event time per launch
(median of 10), algorithmic bytes and fraction of the 8 TB/s peak, and a checksum of the results."""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from tools.microbench import timed  # noqa: E402


def sha(*ts):
    h = hashlib.sha256()
    for t in ts:
        h.update(t.cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def main():
    _abi.load()
    dev = torch.device("cuda", 0)
    P, K = 350_000_000, 32
    g = torch.Generator(device=dev).manual_seed(8)
    old32 = torch.randn(P, generator=g, device=dev)
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(old32).to(torch.bfloat16) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(8).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    out = torch.empty(P, dtype=torch.float64, device=dev)
    v = torch.empty(P, dtype=torch.float64, device=dev)
    m32 = torch.empty(P, dtype=torch.float32, device=dev)
    r1 = lambda: ops.fedopt_step(old32, ups, ns, Ns, first=True, final=True, m_out=m32, v_out=v, out=out)  # noqa: E731
    ms1, _ = timed(r1, reps=10, warm=2)
    c1 = sha(out[:1 << 20], m32[:1 << 20], v[:1 << 20])
    old64, m64, v64 = out.clone(), m32.double(), v.clone()
    mo, vo, o2 = torch.empty_like(m64), torch.empty_like(v64), torch.empty_like(old64)
    r2 = lambda: ops.fedopt_step(old64, ups, ns, Ns, first=True, final=True, m_in=m64, m_out=mo, v_in=v64,  # noqa: E731
                                 v_out=vo, out=o2)
    ms2, _ = timed(r2, reps=10, warm=2)
    c2 = sha(o2[:1 << 20], mo[:1 << 20], vo[:1 << 20])
    pg = torch.empty(P, dtype=torch.float32, device=dev)
    w = lambda: ops.fedopt_step(old32, ups[:8], ns[:8], Ns[:8], first=False, final=False, pg=pg)  # noqa: E731
    ops.fedopt_step(old32, ups[:8], ns[:8], Ns[:8], first=True, final=False, pg=pg)
    msw, _ = timed(w, reps=10, warm=2)
    for name, ms, b, c in (("round1", ms1, K * P * 2 + P * 4 + P * 20, c1), ("steady", ms2, P * (2 * K + 48), c2),
                           ("wave8_nonfinal", msw, 8 * P * 2 + P * 4 + P * 8, sha(pg[:1 << 20]))):
        print(json.dumps({"phase": name, "ms": ms, "GBps": b / ms / 1e6, "frac": b / ms / 1e6 / 8000.0, "checksum": c}),
              flush=True)


if __name__ == "__main__":
    main()
