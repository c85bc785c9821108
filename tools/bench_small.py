"""Round latency of the plug-ins for SMALL models (BASELINE configs[0]'s mnist-pytorch shapes and a
mid-size CNN), host-resident numpy updates through the real combine_models call — the regime most
FEDn deployments run in, where FEDn's numpy loop is already fast and the GPU path must not add
latency. Beside it, the numpy restatement of the same rounds (oracle/, bit-equal to FEDn) timed on
one host core. Every GPU round is checked bit-identical to the oracle.

Run on the GPU box:  python tools/bench_small.py
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi  # noqa: E402
from fedn_amd.aggregators import get_aggregator  # noqa: E402
from fedn_amd.updatehandler import MemoryUpdateHandler  # noqa: E402
from oracle import numpy_ref as ref  # noqa: E402  (the checker and the CPU baseline only)

MNIST = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]          # examples/mnist-pytorch model.py:18-32
CNN = [(64, 3, 3, 3), (64,), (128, 64, 3, 3), (128,), (256, 128, 3, 3), (256,), (512, 256, 3, 3), (512,),
       (4096, 512), (4096,), (10, 4096), (10,)]                        # ~3.7 M params, 12 tensors
PARAMS = {"serveropt": "adam", "learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}


def models(rng, shapes, K):
    base = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    return base, ups, ns


def same(a, b):
    return len(a) == len(b) and all(x.dtype == y.dtype and np.array_equal(x.view(np.uint8), y.view(np.uint8))
                                    for x, y in zip(a, b))


def run(kind, shapes, K, rounds=20, warm=3):
    rng = np.random.default_rng(K)
    base, ups, ns = models(rng, shapes, K)
    uh = MemoryUpdateHandler()
    agg = get_aggregator(kind, uh)
    gid = uh.put_global_model(base, "g0")
    st = ref.FedOptState()
    old = base
    times, ok = [], True
    cpu = []
    for r in range(warm + rounds):
        for a, n in zip(ups, ns):
            uh.submit(a, n, model_id=gid)
        t0 = time.perf_counter()
        model, data = agg.combine_models(helper=None, delete_models=True,
                                         parameters=PARAMS if kind == "fedopt" else None)
        t = time.perf_counter() - t0
        t1 = time.perf_counter()
        if kind == "fedavg":
            want, _ = ref.fedavg_combine(list(zip(ups, ns)))
        else:
            want, _ = ref.fedopt_combine(st, list(zip(ups, ns)), old, PARAMS)
        tc = time.perf_counter() - t1
        ok &= same(model, want)
        if kind == "fedopt":                     # the next round starts from the new global model
            old = want
            gid = uh.put_global_model(model, f"g{r + 1}")
        if r >= warm:
            times.append(t)
            cpu.append(tc)
    P = sum(int(np.prod(s)) for s in shapes)
    gpu_ms, cpu_ms = float(np.median(times)) * 1e3, float(np.median(cpu)) * 1e3
    return {"aggregator": kind, "params": P, "tensors": len(shapes), "clients": K,
            "round_ms_gpu_plugin": gpu_ms, "round_ms_numpy_oracle_1core": cpu_ms, "speedup": cpu_ms / gpu_ms,
            "bit_exact_all_rounds": bool(ok), "rounds": rounds}


def main():
    _abi.load()
    for kind in ("fedavg", "fedopt"):
        for shapes, K in ((MNIST, 2), (MNIST, 10), (MNIST, 64), (CNN, 10), (CNN, 64)):
            print(json.dumps(run(kind, shapes, K)), flush=True)


if __name__ == "__main__":
    main()
