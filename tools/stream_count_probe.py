"""Where the fold traversal loses against a pure streaming read (profiles/r01_store_probe.log).

For K client buffers holding ~25.6 GB in total: stream_sum (the FedAvg traversal with one add)
with its normal store, with the store suppressed (reads only), and with streaming
(non-temporal) or write-through (sc1) stores; then the real fp32 fold with each store mode.
Plain = store mode 0; the library default is 1 (nt).
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from tools.microbench import timed  # noqa: E402

_abi.use_probe()
torch.cuda.set_device(0)
src = torch.empty(8 << 30, dtype=torch.uint8, device="cuda").random_()
sink = ops.stream_read_sink(src)
ops.tune(read=16)
med, best = timed(lambda: ops.stream_read(src, sink))
print(json.dumps({"kernel": "stream_read x16/lane", "GBps": (8 << 30) / med / 1e6}), flush=True)
del src, sink
TOTAL = 6_400_000_000
for K in (8, 64):
    P = TOTAL // K // 4096 * 4096
    bufs = [torch.empty(P, device="cuda").uniform_() for _ in range(K)]
    out = torch.empty(P, device="cuda")
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    by = K * P * 4 + P * 4
    ref = None
    for name, knobs, fn in (
            ("stream_sum", {"nt_store": 0}, lambda: ops.stream_sum(out, bufs)),
            ("stream_sum no-store", {"sum_nostore": 1}, lambda: ops.stream_sum(out, bufs)),
            ("stream_sum nt-store", {"nt_store": 1}, lambda: ops.stream_sum(out, bufs)),
            ("stream_sum sc1-store", {"nt_store": 2}, lambda: ops.stream_sum(out, bufs)),
            ("fold", {"nt_store": 0}, lambda: ops.fedavg_fold(out, bufs, ns, Ns, init=True)),
            ("fold nt-store", {"nt_store": 1}, lambda: ops.fedavg_fold(out, bufs, ns, Ns, init=True)),
            ("fold sc1-store", {"nt_store": 2}, lambda: ops.fedavg_fold(out, bufs, ns, Ns, init=True)),
            ("fold", {"nt_store": 0}, lambda: ops.fedavg_fold(out, bufs, ns, Ns, init=True))):
        ops.tune(**knobs)
        med, best = timed(fn, reps=20)
        ops.tune(sum_nostore=0, nt_store=1)      # library defaults
        same = None
        if name.startswith("fold"):
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            same = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
        nb = K * P * 4 if "no-store" in name else by
        print(json.dumps({"K": K, "P": P, "kernel": name, "ms": med, "GBps": nb / med / 1e6, "best_GBps": nb / best / 1e6,
                          "identical": same}), flush=True)
    del bufs, out
    torch.cuda.empty_cache()
