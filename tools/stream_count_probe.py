"""Does the fold traversal get faster with fewer concurrently read client buffers?
stream_sum (the FedAvg traversal with one add) over K buffers holding 25.6 GB in total."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from tools.microbench import timed  # noqa: E402

_abi.load()
torch.cuda.set_device(0)
src = torch.empty(8 << 30, dtype=torch.uint8, device="cuda").random_()
sink = ops.stream_read_sink(src)
ops.tune(read=16)
med, best = timed(lambda: ops.stream_read(src, sink))
print(json.dumps({"kernel": "stream_read x16/lane", "GBps": (8 << 30) / med / 1e6}), flush=True)
del src, sink
TOTAL = 6_400_000_000          # fp32 elements across all buffers (25.6 GB)
for K in (8, 32, 64):
    P = TOTAL // K // 4096 * 4096
    bufs = [torch.empty(P, device="cuda").uniform_() for _ in range(K)]
    out = torch.empty(P, device="cuda")
    med, best = timed(lambda: ops.stream_sum(out, bufs))
    by = K * P * 4 + P * 4
    print(json.dumps({"K": K, "P": P, "ms": med, "GBps": by / med / 1e6, "best_GBps": by / best / 1e6,
                      "read_GBps": K * P * 4 / med / 1e6}), flush=True)
    ops.tune(sum_nostore=1)            # same traversal, store suppressed: reads only
    med, best = timed(lambda: ops.stream_sum(out, bufs))
    ops.tune(sum_nostore=0)
    print(json.dumps({"K": K, "P": P, "store": False, "ms": med, "read_GBps": K * P * 4 / med / 1e6,
                      "best_read_GBps": K * P * 4 / best / 1e6}), flush=True)
    del bufs, out
    torch.cuda.empty_cache()
