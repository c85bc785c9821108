"""End-to-end (host-resident) FedAvg rate: client updates start in HOST memory, as they do
in a FEDn combiner (UpdateHandler.load_model_update returns numpy arrays), and must cross
PCIe before the fold. Recorded in DESIGN.md; never bench.py's ``value``.

Modes (one JSON line each):
  plugin   fedn_amd.aggregators.fedavg.Aggregator.combine_models over a MemoryUpdateHandler
           holding K numpy updates: pack into pinned slots (threaded), async H2D on a copy
           stream, fold on arrival on the compute stream, D2H of the result.
  pinned   updates already in pinned host buffers (an ingest that lands bytes in pinned
           memory): ring of device slots, H2D(k+1) overlapped with fold(k). PCIe-bound.
  h2d      the same H2D copies alone (the link's achievable rate on this box).
Each mode's result is checked bit-for-bit against the device-resident fold.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=5, help="plugin mode: timed rounds after the first")
    a = ap.parse_args()
    _abi.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K, P = a.clients, a.params
    g = torch.Generator(device=dev).manual_seed(0)
    base = torch.randn(P, generator=g, device=dev)
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    pinned = []
    for _ in range(K):
        u = torch.randn(P, generator=g, device=dev).mul_(0.01).add_(base)
        h = torch.empty(P, dtype=torch.float32, pin_memory=True)
        h.copy_(u)
        pinned.append(h)
    del base, u
    gb = K * P * 4 / 1e9

    # --- h2d only ----------------------------------------------------------------------
    slots = [torch.empty(P, device=dev) for _ in range(a.slots)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        slots[k % a.slots].copy_(pinned[k], non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(json.dumps({"mode": "h2d", "clients": K, "params": P, "s": t, "GBps": gb / t}), flush=True)

    # --- pinned: overlapped H2D + fold ----------------------------------------------------
    comp = torch.cuda.current_stream(dev)
    copy = torch.cuda.Stream(dev)
    h2d_done = [torch.cuda.Event() for _ in range(a.slots)]
    used = [torch.cuda.Event() for _ in range(a.slots)]
    agg = torch.empty(P, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        s = k % a.slots
        if k >= a.slots:
            copy.wait_event(used[s])
        with torch.cuda.stream(copy):
            slots[s].copy_(pinned[k], non_blocking=True)
            h2d_done[s].record(copy)
        comp.wait_event(h2d_done[s])
        if k == 0:
            agg.copy_(slots[s])                         # model = model_next
        else:
            ops.fedavg_fold(agg, [slots[s]], [ns[k]], [Ns[k]], init=False, stream=comp)
        used[s].record(comp)
    out = torch.empty(P, dtype=torch.float32, pin_memory=True)
    out.copy_(agg, non_blocking=True)
    comp.synchronize()
    t = time.perf_counter() - t0
    ref_host = out.clone()
    print(json.dumps({"mode": "pinned", "clients": K, "params": P, "s": t, "params_per_s": K * P / t,
                      "GBps_in": gb / t, "includes": "H2D of every update + fold + D2H of the result"}), flush=True)
    del slots, agg
    torch.cuda.empty_cache()

    # --- plugin: numpy updates through the FEDn-contract aggregator ------------------------
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    uh = MemoryUpdateHandler()
    host_np = [p.numpy() for p in pinned]   # plain numpy views (the plug-in re-packs them)
    for k in range(K):
        uh.submit([host_np[k]], ns[k])
    agg_plugin = get_aggregator("fedavg", uh)
    model, data = agg_plugin.combine_models(helper=None)      # round 1: pinned pool warm-up
    times, rounds = [], []
    for r in range(a.rounds):            # a session's later rounds; the first ones run while the GPU ramps up
        for k in range(K):
            uh.submit([host_np[k]], ns[k])
        t0 = time.perf_counter()
        model, data = agg_plugin.combine_models(helper=None)
        times.append(time.perf_counter() - t0)
        rounds.append({k: v for k, v in data.items() if isinstance(v, (int, float))})
    exact = bool(np.array_equal(model[0].view(np.uint32), ref_host.numpy().view(np.uint32)))
    i = int(np.argsort(times)[len(times) // 2])
    t = times[i]
    print(json.dumps({"mode": "plugin", "clients": K, "params": P, "s": t, "params_per_s": K * P / t,
                      "GBps_in": gb / t, "bit_exact_vs_pinned": exact, "rounds_s": [round(x, 4) for x in times],
                      "note": f"median of rounds 2..{a.rounds + 1} of one session", "data": rounds[i]}), flush=True)


if __name__ == "__main__":
    main()
