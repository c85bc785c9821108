"""Host-resident FedAvg rounds through the plug-in on D device entries (one process, multidev.py),
the H2D source of each update's large tensors in four modes:

  pack            pageable arrays packed into pinned slots (the default for pageable memory)
  register        pageable arrays page-locked in place (multidev.INPLACE_REGISTER), the SAME arrays
                  every round (a caller reusing its buffers: pages re-registered cheaply)
  register_fresh  as register, each round's updates new arrays (as FEDn decodes them): first-time
                  page-locking, and the unregistration at round end
  pinned_fresh    each round's updates new arrays in page-locked memory from helper.pinned_empty
                  (what fedn_amd.helper.load decodes large members into), DMA'd in place; the copy
                  into them stands in for the decode and is outside the timed round

Same updates, same session shape as bench.py's host_resident field; median of rounds 2..; bit-exact
on a sample against the oracle.

On a one-GPU box the D entries share ONE PCIe link, so the rate there is link-bound whatever the
host does; what the A/B shows is the host-side cost per update that an N-link node would expose
(``stage_ms``: the calling thread's time in multidev._stage per update).

    python tools/bench_hostres.py [--devices 2 4 8] [--clients 16] [--params 100000000] [--modes ...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, multidev  # noqa: E402
from fedn_amd.aggregators.fedavg import Aggregator  # noqa: E402
from fedn_amd.updatehandler import MemoryUpdateHandler  # noqa: E402
from oracle import numpy_ref as ref  # noqa: E402  (the sample checker only)


def run(devs, host, ns, rounds, mode):
    from fedn_amd.helper import pinned_empty
    multidev.INPLACE_MIN_BYTES = 0 if mode == "pack" else (8 << 20)
    multidev.INPLACE_REGISTER = mode.startswith("register")
    stage_t = [0.0, 0]
    real = multidev._ShardedStaging._stage

    def timed(self, arrays):
        t0 = time.perf_counter()
        try:
            return real(self, arrays)
        finally:
            stage_t[0] += time.perf_counter() - t0
            stage_t[1] += 1
    multidev._ShardedStaging._stage = timed
    phase = {}
    wrapped = []
    for cls, name in ((multidev.ShardedFedAvgPipeline, "result"), (multidev._ShardedStaging, "quiesce"),
                      (multidev._ShardedStaging, "_unregister_retired")):
        f = getattr(cls, name)

        def w(self, *a, _f=f, _n=name, **k):
            t0 = time.perf_counter()
            try:
                return _f(self, *a, **k)
            finally:
                phase[_n] = phase.get(_n, 0.0) + time.perf_counter() - t0
        setattr(cls, name, w)
        wrapped.append((cls, name, f))
    try:
        uh = MemoryUpdateHandler()
        agg = Aggregator(uh, devices=list(devs))
        times, model, data = [], None, None
        for r in range(rounds + 1):
            if mode == "register_fresh":
                ups = [h.copy() for h in host]
            elif mode == "pinned_fresh":
                ups = []
                for h in host:
                    p = pinned_empty(h.shape, h.dtype)
                    p[...] = h
                    ups.append(p)
            else:
                ups = host
            for k, h in enumerate(ups):
                uh.submit([h], ns[k])
            del ups
            stage_t[:] = [0.0, 0]
            phase.clear()
            t0 = time.perf_counter()
            model, data = agg.combine_models(helper=None)
            if r:
                times.append(time.perf_counter() - t0)
    finally:
        multidev._ShardedStaging._stage = real
        for cls, name, f in wrapped:
            setattr(cls, name, f)
    S = 1_000_000
    want = ref.fedavg_flat([h[:S] for h in host], ns)
    exact = bool(np.array_equal(model[0][:S].view(np.uint32), want.view(np.uint32)))
    t = sorted(times)[len(times) // 2]
    P = host[0].size
    return {"devices": len(devs), "mode": mode, "round_s": round(t, 4),
            "GBps_in": round(len(host) * P * 4 / t / 1e9, 2), "rounds_s": [round(x, 4) for x in times],
            "stage_ms_per_update": round(stage_t[0] / max(1, stage_t[1]) * 1e3, 3) if stage_t[1] else None,
            "stage_host_ms_per_update": round(data.get("time_stage_host", 0.0) / max(1, stage_t[1]) * 1e3, 3),
            "stage_wait_ms_per_update": round(data.get("time_stage_wait", 0.0) / max(1, stage_t[1]) * 1e3, 3),
            "bytes_h2d_in_place": data.get("bytes_h2d_in_place"), "bytes_h2d_packed": data.get("bytes_h2d_packed"),
            "bit_exact_on_sample": exact, "last_round_phase_ms": {k: round(v * 1e3, 2) for k, v in phase.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--modes", nargs="+", default=["pack", "register", "register_fresh", "pinned_fresh"])
    a = ap.parse_args()
    _abi.load()
    from fedn_amd import layout
    layout.MULTIDEV_MIN_BYTES = 0
    g = torch.Generator(device="cuda:0").manual_seed(11)
    base = torch.randn(a.params, generator=g, device="cuda:0")
    host = [torch.randn(a.params, generator=g, device="cuda:0").mul_(0.01).add_(base).cpu().numpy()
            for _ in range(a.clients)]
    del base
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, a.clients)]
    for D in a.devices:
        devs = [torch.device("cuda", 0)] * D
        for mode in a.modes:
            print(json.dumps(run(devs, host, ns, a.rounds, mode)), flush=True)


if __name__ == "__main__":
    main()
