"""Why a 64-client fold over a short chunk (1.56 M params and below: a rank's round at N = 8, R >= 8,
tools/rank_fold_time.py) runs at ~0.4 of peak: every wave of such a launch is resident at once, so
the launch takes one wave's latency chain through the 64 clients — how many client loads it keeps in
flight sets the time, not bandwidth. Probe library geometries (fa_tune): 1 strip per lane with 4
(product), 8 or 16 clients loaded ahead; 2 strips x 4 / 8; the pipelined 4-strip kernel. fp32,
K = 64, P = 0.39 M ... 12.5 M; HIP-event median per launch, fraction of the 8 TB/s peak; results
checked bit-identical to the product kernel.

Run on the GPU box:  python tools/small_chunk_probe.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from tools.microbench import timed  # noqa: E402

K = 64
STRIPS, UNROLL, AUTO_GEOM = 0, 1, 20
GEOMS = {"product": None, "s1_u4": (1, 4), "s1_u8": (1, 8), "s1_u16": (1, 16), "s2_u4": (2, 4), "s2_u8": (2, 8),
         "pipe_s4": (4, 0)}


def main():
    _abi.load()
    probe = _abi.load_probe()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    ns = [int(v) for v in np.random.default_rng(2).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    Pmax = 12_500_992
    base = torch.randn(Pmax, generator=g, device=dev)
    ups = [torch.randn(Pmax, generator=g, device=dev).mul_(0.01).add_(base) for _ in range(K)]
    for P in (390_656, 781_312, 1_562_624, 3_125_248, 6_250_496, 12_500_992):
        views = [u[:P] for u in ups]
        want = torch.empty(P, device=dev)
        ops.fedavg_fold(want, views, ns, Ns, init=True)
        row = {"P": P, "K": K}
        for name, geom in GEOMS.items():
            agg = torch.empty(P, device=dev)
            with _abi.use_probe():
                if geom is None:
                    probe.fa_tune(AUTO_GEOM, 1)
                    probe.fa_tune(STRIPS, 4)
                    probe.fa_tune(UNROLL, 0)
                else:
                    probe.fa_tune(AUTO_GEOM, 0)
                    probe.fa_tune(STRIPS, geom[0])
                    probe.fa_tune(UNROLL, geom[1])
                ms, _ = timed(lambda: ops.fedavg_fold(agg, views, ns, Ns, init=True), reps=20, warm=3)
                probe.fa_tune(AUTO_GEOM, 1)
                probe.fa_tune(STRIPS, 4)
                probe.fa_tune(UNROLL, 0)
            same = bool(torch.equal(agg.view(torch.int32), want.view(torch.int32)))
            row[name] = {"ms": round(ms, 4), "frac": round((K * P * 4 + P * 4) / ms / 8e9, 3), "bit_identical": same}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
