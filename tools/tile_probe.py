"""Mid-size models: the fold's tile size against the number of workgroups (libfedagg_probe.so).
One tile per workgroup and every workgroup folds all K clients, so at P = 1-20 M the grid is only
a few times the ~1,024 resident workgroups and the last partial wave of workgroups decides the
time. Sweeps P and the strips per lane (tile = 256 lanes x strips x 16 B) for fp32 and bf16,
K = 64 and 8; median of interleaved repeats; aggregates must be bit-identical across settings."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from tools.microbench import timed  # noqa: E402

PEAK = 8000.0
SEL = os.environ.get("SEL", "s4,s2,s1u4,s1u8,s1u16,s2u4,s2u8,s4u2,s4_wide_bf16").split(",")
SETTINGS = [("s4", dict(strips=4, unroll=0, narrow=1)), ("s2", dict(strips=2, unroll=0, narrow=1)),
            ("s1u4", dict(strips=1, unroll=4, narrow=1)), ("s1u8", dict(strips=1, unroll=8, narrow=1)),
            ("s1u16", dict(strips=1, unroll=16, narrow=1)), ("s2u4", dict(strips=2, unroll=4, narrow=1)),
            ("s2u8", dict(strips=2, unroll=8, narrow=1)), ("s4u2", dict(strips=4, unroll=2, narrow=1)),
            ("s4_wide_bf16", dict(strips=4, unroll=0, narrow=0))]


def main():
    _abi.use_probe()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    rng = np.random.default_rng(3)
    Pmax = int(os.environ.get("PMAX", "100000000"))
    base = torch.randn(Pmax, generator=g, device=dev)
    ups32 = [torch.randn(Pmax, generator=g, device=dev).mul_(0.01).add_(base) for _ in range(64)]
    ups16 = [u.to(torch.bfloat16) for u in ups32]
    for P in [int(x) for x in os.environ.get("PS", "10000000,40000000,100000000").split(",")]:
        for dt, ups in (("f32", ups32), ("bf16", ups16)):
            for K in [int(x) for x in os.environ.get("KS", "64,8").split(",")]:
                ns = [int(v) for v in rng.integers(1, 5001, K)]
                Ns = [int(v) for v in np.cumsum(ns)]
                agg = torch.empty(P, device=dev)
                views = [u[:P] for u in ups[:K]]
                ref = None
                res = {name: [] for name, _ in SETTINGS if name in SEL}
                for _ in range(3):
                    for name, kw in [st for st in SETTINGS if st[0] in SEL]:
                        if name == "s4_wide_bf16" and dt != "bf16":
                            continue
                        ops.tune(auto_geom=0, **kw)
                        ms, _b = timed(lambda: ops.fedavg_fold(agg, views, ns, Ns, init=True), reps=10, warm=2)
                        res[name].append(ms)
                        if ref is None:
                            ref = agg.clone()
                        elif not torch.equal(agg.view(torch.int32), ref.view(torch.int32)):
                            raise SystemExit(f"{name} P={P} {dt}: differs")
                b = K * P * (4 if dt == "f32" else 2) + P * 4
                for name, ts in res.items():
                    if not ts:
                        continue
                    ms = float(np.median(ts))
                    print(json.dumps({"dtype": dt, "K": K, "P": P, "setting": name, "ms": ms, "frac": b / ms / 1e6 / PEAK}),
                          flush=True)
    ops.tune(strips=4, unroll=0, narrow=1, auto_geom=1)


if __name__ == "__main__":
    main()
