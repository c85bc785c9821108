"""configs[4] wave finish A/B (GPU box): 1 B bf16 params x 128 FedYogi updates from 8 pooled pinned
host buffers (as bench.py's fedopt_waves), WaveFedOpt with the separate K = 0 server step vs the
server step fused into the last wave's launch, at waves of 8 and 16. Per variant: round wall time,
per-kind kernel time / algorithmic bytes / HBM fraction, and a sha256 of the result (all variants
must agree bit for bit).

    python tools/wave_probe.py [--params 1000000000] [--reps 2]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd.waves import WaveFedOpt  # noqa: E402

PER_EL = {"first": lambda k: 2 * k + 16, "mid": lambda k: 2 * k + 24, "final": lambda k: 40,
          "mid_final": lambda k: 2 * k + 40, "first_final": lambda k: 2 * k + 32}
HBM = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=1_000_000_000)
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    P, K, pool = a.params, a.clients, 8
    g = torch.Generator(device=dev).manual_seed(5)
    base = torch.randn(P, generator=g, device=dev)
    host = []
    for _ in range(pool):
        h = torch.empty(P, dtype=torch.bfloat16, pin_memory=True)
        h.copy_((base + 0.01 * torch.randn(P, generator=g, device=dev)).to(torch.bfloat16))
        host.append(h)
    ups = [host[k % pool] for k in range(K)]
    ns = [int(v) for v in np.random.default_rng(5).integers(1, 5001, K)]
    params = {"serveropt": "yogi"}
    old = WaveFedOpt([dev], P).slices(base.double())
    del base
    WaveFedOpt([dev], P, wave=8).round(ups[:8], ns[:8], old, params)       # warm-up
    shas = set()
    for rep in range(a.reps):
        for W, fuse in ((8, False), (8, True), (16, False), (16, True)):
            wf = WaveFedOpt([dev], P, wave=W, fuse_final=fuse)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            outs = wf.round(ups, ns, old, params)
            t = time.perf_counter() - t0
            spans = {}
            outs2 = WaveFedOpt([dev], P, wave=W, fuse_final=fuse).round(ups, ns, old, params, kernel_times=spans)
            sha = hashlib.sha256(outs[0].cpu().numpy().tobytes()).hexdigest()[:16]
            same = bool(torch.equal(outs[0], outs2[0]))
            shas.add(sha)
            kern = {}
            for kind, rows in spans.items():
                ms = sum(r[3] for r in rows)
                b = sum(r[1] * PER_EL[kind](r[2]) for r in rows)
                kern[kind] = {"launches": len(rows), "ms_total": round(ms, 3),
                              "frac": round(b / (ms / 1e3) / 1e9 / HBM, 4)}
            ktot = sum(v["ms_total"] for v in kern.values())
            print(json.dumps({"rep": rep, "W": W, "fuse_final": fuse, "round_s": round(t, 4),
                              "kernel_ms_total": round(ktot, 2), "kernels": kern, "sha": sha, "repeat_same": same}),
                  flush=True)
            del outs, outs2, wf
            torch.cuda.empty_cache()
    print(json.dumps({"variants_bit_identical": len(shas) == 1, "shas": sorted(shas)}), flush=True)


if __name__ == "__main__":
    main()
