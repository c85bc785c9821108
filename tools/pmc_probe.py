"""One workload per process, for rocprofv3 --pmc passes (tools/gpu_session.sh pmcprobe).

  read     k_stream_read over one 6.4 GB buffer (16 x 16 B per lane)
  sum8     the fold traversal, store suppressed, 8 buffers x 800 M fp32
  sum64    the same, 64 buffers x 100 M fp32
  fold64   the real fp32 fold, 64 x 100 M (the BASELINE workload)
Each runs 3 launches; the counters are averaged per dispatch by tools/pmc_probe_report.py.
"""
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402

TOTAL = 6_400_000_000


def main(which):
    _abi.use_probe()
    torch.cuda.set_device(0)
    if which == "read":
        src = torch.empty(TOTAL, dtype=torch.uint8, device="cuda").random_()
        sink = ops.stream_read_sink(src)
        ops.tune(read=16)
        for _ in range(3):
            ops.stream_read(src, sink)
    else:
        K = {"sum8": 8, "sum64": 64, "fold64": 64}[which]
        P = TOTAL // K // 4096 * 4096
        bufs = [torch.empty(P, device="cuda").uniform_() for _ in range(K)]
        out = torch.empty(P, device="cuda")
        ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
        Ns = [int(v) for v in np.cumsum(ns)]
        for _ in range(3):
            if which == "fold64":
                ops.fedavg_fold(out, bufs, ns, Ns, init=True)
            else:
                ops.tune(sum_nostore=1)
                ops.stream_sum(out, bufs)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(sys.argv[1])
