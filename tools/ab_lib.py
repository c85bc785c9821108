"""A/B one libfedagg build against another (FEDN_AMD_LIB selects the library): median fold
time for fp32 K=64 / fp32 K=8 / bf16 K=64 over 100 M params, plus a SHA-256 of each result so
the two builds can be checked bit-identical. One JSON line per workload."""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from tools.microbench import timed  # noqa: E402


def main():
    _abi.use_probe()
    torch.cuda.set_device(0)
    P = 100_000_000
    lib = os.path.basename(os.environ.get("FEDN_AMD_LIB", "libfedagg.so"))
    g = torch.Generator(device="cuda").manual_seed(0)
    base = torch.randn(P, generator=g, device="cuda")
    ups32 = [torch.randn(P, generator=g, device="cuda").mul_(0.01).add_(base) for _ in range(64)]
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, 64)]
    Ns = [int(v) for v in np.cumsum(ns)]
    out = torch.empty(P, device="cuda")
    for name, ups, K, by in (("f32_k64", ups32, 64, 64 * P * 4 + P * 4), ("f32_k8", ups32[:8], 8, 8 * P * 4 + P * 4)):
        med, best = timed(lambda: ops.fedavg_fold(out, ups, ns[:K], Ns[:K], init=True), reps=20)
        h = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
        print(json.dumps({"lib": lib, "workload": name, "ms": med, "GBps": by / med / 1e6, "best_GBps": by / best / 1e6,
                          "sha": h}), flush=True)
    ups16 = [u.to(torch.bfloat16) for u in ups32]
    del ups32
    by = 64 * P * 2 + P * 4
    med, best = timed(lambda: ops.fedavg_fold(out, ups16, ns, Ns, init=True), reps=20)
    h = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": lib, "workload": "bf16_k64", "ms": med, "GBps": by / med / 1e6, "best_GBps": by / best / 1e6,
                      "sha": h}), flush=True)


if __name__ == "__main__":
    main()
