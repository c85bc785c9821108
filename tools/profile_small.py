"""cProfile of the plug-in's host work on a small model (configs[0]'s mnist-pytorch shapes): where the
per-round and per-update microseconds go in combine_models. Run on the GPU box:
    python tools/profile_small.py [--clients K] [--kind fedavg|fedopt]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi  # noqa: E402
from fedn_amd.aggregators import get_aggregator  # noqa: E402
from fedn_amd.updatehandler import MemoryUpdateHandler  # noqa: E402

MNIST = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--kind", default="fedavg")
    ap.add_argument("--rounds", type=int, default=30)
    a = ap.parse_args()
    _abi.load()
    rng = np.random.default_rng(0)
    base = [rng.standard_normal(s).astype(np.float32) for s in MNIST]
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(a.clients)]
    ns = [int(v) for v in rng.integers(1, 5001, a.clients)]
    uh = MemoryUpdateHandler()
    agg = get_aggregator(a.kind, uh)
    gid = uh.put_global_model(base, "g0")
    params = {"serveropt": "adam"} if a.kind == "fedopt" else None

    def one_round():
        for u, n in zip(ups, ns):
            uh.submit(u, n, model_id=gid)
        t0 = time.perf_counter()
        agg.combine_models(helper=None, parameters=params)
        return time.perf_counter() - t0

    for _ in range(5):
        one_round()
    ts = sorted(one_round() for _ in range(a.rounds))
    print(f"{a.kind} mnist K={a.clients}: median round {ts[len(ts) // 2] * 1e3:.3f} ms (min {ts[0] * 1e3:.3f})")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.rounds):
        one_round()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
    print(s.getvalue())


if __name__ == "__main__":
    main()
