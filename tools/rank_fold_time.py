"""Time one rank's share of bench.py --gpus N's step on ONE GPU: the R fold launches of 64 clients x C
fp32 params (sharded.CyclicShardedFedAvg's block-cyclic geometry, the same launches
tools/pmc_rank_fold.py replays for PMC) — issued as the step issues them (client table as device
addresses, CyclicShardedFedAvg.round_folder) and, for comparison, through 64 tensor slices per
launch — for N = 2, 4, 8 and every round count R the warm-up may pick, plus a fa_push of each folded round into N - 1 other buffers of this GPU (the push kernel's own
cost when the links are not the limit). What the fold contributes to the N-GPU step; the gather over
xGMI is the node's to measure.

Run on the GPU box:  python tools/rank_fold_time.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fedn_amd import _abi, ops  # noqa: E402
from pmc_rank_fold import rank_geometry  # noqa: E402

P, K, STEPS = 100_000_000, 64, 10


def timed(fn, steps, stream):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(stream)
    for _ in range(steps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def main():
    _abi.load()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    g = torch.Generator(device=dev).manual_seed(1)
    for world in (2, 4, 8):
        L_max = max(rank_geometry(P, world, R)[2] for R in (1, 2, 4, 8, 16))
        base = torch.randn(L_max, generator=g, device=dev)
        ups = [torch.randn(L_max, generator=g, device=dev).mul_(0.01).add_(base) for _ in range(K)]
        agg = torch.empty(L_max, device=dev)
        peers = [torch.empty(L_max, device=dev) for _ in range(world - 1)]
        for R in (1, 2, 4, 8, 16):
            C, rounds, L = rank_geometry(P, world, R)

            bases = [u.data_ptr() for u in ups]

            def fold():                         # CyclicShardedFedAvg.round_folder's launches
                for i in range(rounds):
                    ops.fedavg_fold_ptrs(agg[i * C:(i + 1) * C], [b + i * C * 4 for b in bases], torch.float32,
                                         ns, Ns, init=True, stream=stream)

            def fold_sliced():                  # the same launches through 64 tensor slices each
                for i in range(rounds):
                    sl = slice(i * C, (i + 1) * C)
                    ops.fedavg_fold(agg[sl], [u[sl] for u in ups], ns, Ns, init=True, stream=stream)

            def push():
                for i in range(rounds):
                    sl = slice(i * C, (i + 1) * C)
                    ops.push([p[sl].data_ptr() for p in peers], agg[sl], C * 4, stream)

            fms = timed(fold, STEPS, stream)
            sms = timed(fold_sliced, STEPS, stream)
            pms = timed(push, STEPS, stream)
            alg = K * L * 4 + L * 4
            print(json.dumps({"world": world, "rounds": rounds, "chunk": C, "local_len": L,
                              "fold_ms_per_step": round(fms, 4), "fold_frac_of_peak": round(alg / fms / 8e9, 4),
                              "fold_sliced_ms_per_step": round(sms, 4),
                              "push_local_ms_per_step": round(pms, 4),
                              "push_note": f"fa_push of every round into {world - 1} buffers of this GPU "
                                           "(HBM-local: the kernel's own cost, not the links')"}), flush=True)
        del base, ups, agg, peers
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
