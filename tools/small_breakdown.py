"""Where the fixed cost of a small-model round goes (configs[0]'s mnist shapes, K host updates):
wall time of each phase of combine_models, per round, median over rounds (no profiler overhead).
Run on the GPU box: python tools/small_breakdown.py [--clients K]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, staging  # noqa: E402
from fedn_amd.aggregators import fedavg as fedavg_mod  # noqa: E402
from fedn_amd.aggregators import get_aggregator  # noqa: E402
from fedn_amd.updatehandler import MemoryUpdateHandler  # noqa: E402

MNIST = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]
T = {}


def timed(owner, name, label):
    f = getattr(owner, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[label] = T.get(label, 0.0) + time.perf_counter() - t0
    setattr(owner, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--kind", default="fedavg", choices=["fedavg", "fedopt"])
    a = ap.parse_args()
    _abi.load()
    rng = np.random.default_rng(0)
    base = [rng.standard_normal(s).astype(np.float32) for s in MNIST]
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(a.clients)]
    ns = [int(v) for v in rng.integers(1, 5001, a.clients)]
    timed(fedavg_mod, "make_fedavg_pipeline", "make_pipeline")
    cls = staging.FedAvgPipeline if a.kind == "fedavg" else staging.FedOptPipeline
    for name in ("__init__", "add", "result", "server_step", "timings", "release", "upload_arena", "_fold_group",
                 "_fold_then_d2h", "put_small", "_h2d_old", "_fold_pg"):
        if name in vars(cls) or hasattr(cls, name):
            timed(cls, name, name)
    uh = MemoryUpdateHandler()
    agg = get_aggregator(a.kind, uh)
    gid = uh.put_global_model(base, "g0")
    params = {"serveropt": "adam"} if a.kind == "fedopt" else None
    rows = []
    for r in range(a.rounds + 5):
        for u, n in zip(ups, ns):
            uh.submit(u, n, model_id=gid)
        T.clear()
        t0 = time.perf_counter()
        agg.combine_models(helper=None, parameters=params)
        T["total"] = time.perf_counter() - t0
        if r >= 5:
            rows.append(dict(T))
    keys = sorted({k for r in rows for k in r})
    med = {k: round(float(np.median([r.get(k, 0.0) for r in rows]) * 1e3), 4) for k in keys}
    print(json.dumps({"kind": a.kind, "clients": a.clients, "median_ms": med}), flush=True)


if __name__ == "__main__":
    main()
