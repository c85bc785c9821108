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
TOTAL = 6_400_000_000          # fp32 elements across all buffers (25.6 GB)
for K in (2, 4, 8, 16, 32, 64):
    P = TOTAL // K // 4096 * 4096
    bufs = [torch.empty(P, device="cuda").uniform_() for _ in range(K)]
    out = torch.empty(P, device="cuda")
    med, best = timed(lambda: ops.stream_sum(out, bufs))
    by = K * P * 4 + P * 4
    print(json.dumps({"K": K, "P": P, "ms": med, "GBps": by / med / 1e6, "best_GBps": by / best / 1e6,
                      "read_GBps": K * P * 4 / med / 1e6}), flush=True)
    del bufs, out
    torch.cuda.empty_cache()
