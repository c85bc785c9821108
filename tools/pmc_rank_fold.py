"""One rank's fold at N > 1, on one GPU, for rocprofv3 PMC passes (tools/gpu_session.sh pmcrank):
bench.py --gpus N deals the 100 M-param model block-cyclically over N ranks in R rounds
(sharded.CyclicShardedFedAvg) and each rank folds R chunks of C params per step, one launch each.
This replays exactly those launches (64 clients x C fp32, R per step) so the per-launch HBM traffic
of the rank's fold can be measured on a one-GPU box; tools/pmc_traffic.py --rank-session turns it
into profiles/pmc_traffic.json entries under bench.py's N > 1 workload keys."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from fedn_amd.sharded import ALIGN_ELEMS  # noqa: E402


def rank_geometry(P, world, rounds_wanted, align=ALIGN_ELEMS):
    """(C, rounds, local_len) as CyclicShardedFedAvg computes them for bench.py's chunk choice."""
    chunk = -(-P // (world * rounds_wanted))
    C = max(align, -(-chunk // align) * align)
    nchunks = max(1, -(-P // C))
    rounds = -(-nchunks // world)
    return C, rounds, rounds * C


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--ag-rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    _abi.load()
    dev = torch.device("cuda", 0)
    C, rounds, L = rank_geometry(a.params, a.world, a.ag_rounds)
    g = torch.Generator(device=dev).manual_seed(1)
    base = torch.randn(C, generator=g, device=dev)
    ups = [torch.randn(C, generator=g, device=dev).mul_(0.01).add_(base) for _ in range(a.clients)]
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, a.clients)]
    Ns = [int(v) for v in np.cumsum(ns)]
    agg = torch.empty(C, device=dev)
    for _ in range(a.steps * rounds):
        ops.fedavg_fold(agg, ups, ns, Ns, init=True)
    torch.cuda.synchronize()
    print(json.dumps({"world": a.world, "chunk": C, "rounds": rounds, "local_len": L,
                      "workload": f"fedavg_k{a.clients}_p{L}_r{rounds}_f32_rank_of_{a.world}"}), flush=True)


if __name__ == "__main__":
    main()
