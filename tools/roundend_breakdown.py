"""Where the round-end FedAvg time goes (tools/bench_roundend.py's batched config, 64 x 100 M fp32
device-resident): wall time of each plug-in phase per combine_models call, by wrapping the pipeline
methods with timers. Diagnostic only."""
import functools
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_roundend import DeviceResidentHandler, staged_updates  # noqa: E402
from fedn_amd import _abi, staging  # noqa: E402
from fedn_amd.aggregators import fedavg as fedavg_mod  # noqa: E402
from fedn_amd.aggregators import get_aggregator  # noqa: E402

T = {}


def timed(owner, name, label):
    f = getattr(owner, name)

    @functools.wraps(f)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[label] = T.get(label, 0.0) + time.perf_counter() - t0
    setattr(owner, name, w)


def main():
    _abi.load()
    torch.cuda.set_device(0)
    K, P = 64, 100_000_000
    ups = staged_updates(K, P, 1)
    ns = [int(v) for v in np.random.default_rng(1).integers(1, 5001, K)]
    timed(fedavg_mod, "make_fedavg_pipeline", "make_pipeline")
    for name in ("add", "result", "timings", "release", "_flush", "_to_host"):
        if hasattr(staging.FedAvgPipeline, name):
            timed(staging.FedAvgPipeline, name, name)
    uh = DeviceResidentHandler()
    agg = get_aggregator("fedavg", uh)              # one aggregator: a session's rounds
    for rep in range(6):
        for i, (s, n) in enumerate(zip(ups, ns)):
            uh.submit(s, n, i)
        torch.cuda.synchronize()
        T.clear()
        t0 = time.perf_counter()
        model, data = agg.combine_models(helper=None)
        T["total"] = time.perf_counter() - t0
        print(json.dumps({"rep": rep, **{k: round(v * 1e3, 3) for k, v in T.items()},
                          "time_kernel_ms": round(data["time_kernel"] * 1e3, 3),
                          "time_d2h_ms": round(data["time_d2h"] * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
