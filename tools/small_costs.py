"""Per-call host costs inside configs[0]'s K = 2 plug-in round (mnist shapes), each timed alone,
median over many calls: which pieces of the ~50 µs of Python around the GPU round trip are worth
removing (tools/small_floor.py measures the round and its floor). Run on the GPU box:
python tools/small_costs.py
"""
import json
import logging
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops, staging  # noqa: E402
from fedn_amd.aggregators import fedavg as fedavg_mod  # noqa: E402
from fedn_amd.aggregators.aggregatorbase import queued_updates  # noqa: E402
from fedn_amd.layout import Layout  # noqa: E402
from fedn_amd.updatehandler import MemoryUpdateHandler  # noqa: E402

MNIST = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]


def med(f, n=2000, warm=50):
    for _ in range(warm):
        f()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 2)


def main():
    _abi.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rng = np.random.default_rng(0)
    ups = [[rng.standard_normal(s).astype(np.float32) for s in MNIST] for _ in range(2)]
    P = sum(int(np.prod(s)) for s in MNIST)
    out = {}
    out["torch.device"] = med(lambda: torch.device(dev))
    out["current_stream"] = med(lambda: torch.cuda.current_stream(dev))
    out["default_device"] = med(fedavg_mod.default_device)
    out["Layout.of"] = med(lambda: Layout.of(ups[0]))
    out["pinned_empty_210KB"] = med(lambda: torch.empty(P, dtype=torch.float32, pin_memory=True))
    blk = torch.empty(P, dtype=torch.float32, pin_memory=True)
    out["host_device_ptr"] = med(lambda: ops.host_device_ptr(blk.data_ptr(), dev))
    out["torch_dtype+fold_result_dtype"] = med(lambda: ops.fold_result_dtype(ops.torch_dtype(np.dtype(np.float32)),
                                                                            torch.float32))
    st = torch.cuda.current_stream(dev)
    pb = ops.host_device_ptr(blk.data_ptr(), dev)
    arena = torch.empty(3 * P, dtype=torch.float32, pin_memory=True)
    pa = ops.host_device_ptr(arena.data_ptr(), dev)
    out["fedavg_fold_raw_call"] = med(lambda: ops.fedavg_fold_raw(pb, torch.float32, P, [pa, pa + 4 * P, pa + 8 * P],
                                                                  torch.float32, [0.0, 7.0, 9.0], [1.0, 7.0, 16.0],
                                                                  True, st, dev), n=500)
    st.synchronize()
    lay = Layout.of(ups[0])
    outl = [None] * 6
    out["unpack_group"] = med(lambda: lay.unpack_group(blk.numpy(), np.dtype(np.float32), outl, copy=False))
    cache = staging.StagingCache()
    box = {}

    def make():
        p = staging.FedAvgPipeline(dev, ups[0], cache=cache)
        box["p"] = p
        return p

    def make_release():
        p = make()
        p.quiesce()
        p.release()
    out["FedAvgPipeline_init+release"] = med(make_release, n=1000)
    uh = MemoryUpdateHandler()

    def submit2():
        for u in ups:
            uh.submit(u, 10)
        for mu, load in queued_updates(uh, None, size_box=[None, 1e-6]):
            load()
    out["submit2+drain2"] = med(submit2, n=1000)
    log = logging.getLogger("fedn")
    out["logger.info"] = med(lambda: log.info("AGGREGATOR(fedavg): Aggregating model updates... "))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
