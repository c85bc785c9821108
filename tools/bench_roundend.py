"""Round-end latency of the plug-ins when the round's updates are ALREADY in HBM.

With the streaming ingest (ingest.StagingUpdateHandler) every update is decoded and copied to
the device as it arrives, so what is left when FEDn calls ``combine_models`` at round end is
the device work plus the D2H of the new model. This times exactly that, through the real
plug-ins, on synthetic device-resident updates (StagedModel objects served by a minimal
UpdateHandler), and compares:

  batched   staging.BATCH = 64 (default): pending updates fold in one multi-client launch,
            the final launch chunked with each chunk's D2H overlapped
  per-update  staging.BATCH = 1: one launch per update as it is loaded (the previous behaviour)

Results are checked bit-identical between the two. Configs: FedAvg 64 x 100 M fp32 (the
BASELINE workload) and FedOpt (adam, steady state round 2) 32 x 350 M fp32 (configs[3]).
"""
import argparse
import json
import os
import queue
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, staging  # noqa: E402
from fedn_amd.aggregators import get_aggregator  # noqa: E402
from fedn_amd.ingest import StagedModel  # noqa: E402
from fedn_amd.layout import Layout  # noqa: E402


class _MU:
    def __init__(self, i, model_id):
        self.model_update_id = f"u{i}"
        self.model_id = model_id


class DeviceResidentHandler:
    """The UpdateHandler surface the plug-ins use (updatehandler.py:31-163), serving updates
    that are already StagedModels in HBM, as ingest.StagingUpdateHandler leaves them. Like that
    handler it declares ``stages_on_arrival``: the plug-in drains it one update at a time, with no
    read-ahead thread (aggregatorbase.queued_updates), the path the product handler takes."""

    stages_on_arrival = True

    def __init__(self):
        self.model_updates = queue.Queue()
        self.staged = {}
        self.globals = {}

    def submit(self, staged, n, i, model_id="g"):
        mu = _MU(i, model_id)
        self.staged[mu.model_update_id] = (staged, n)
        self.model_updates.put(mu)

    def next_model_update(self):
        return self.model_updates.get(block=False)

    def load_model_update(self, mu, helper):
        s, n = self.staged[mu.model_update_id]
        return s, {"num_examples": n}

    def load_model(self, helper, model_id):
        return self.globals[model_id]

    def delete_model(self, mu):
        pass


def staged_updates(K, P, seed, base=None):
    dev = torch.device("cuda", 0)
    layout = Layout.of([np.empty(P, np.float32)])
    g = torch.Generator(device=dev).manual_seed(seed)
    if base is None:
        base = torch.randn(P, generator=g, device=dev)
    out = []
    for _ in range(K):
        buf = torch.empty(layout.nbytes, dtype=torch.uint8, device=dev)
        buf[:P * 4].view(torch.float32).copy_(torch.randn(P, generator=g, device=dev).mul_(0.01).add_(base))
        ev = torch.cuda.Event()
        ev.record()
        out.append(StagedModel(layout, buf, ev, None))
    torch.cuda.synchronize()
    return out


WARM = 2


def run_fedavg(K, P, reps):
    ups = staged_updates(K, P, 1)
    ns = [int(v) for v in np.random.default_rng(1).integers(1, 5001, K)]
    res = {}
    for mode, batch in (("batched", 64), ("per-update", 1), ("batched", 64)):
        staging.BATCH = batch
        ts = []
        uh = DeviceResidentHandler()
        agg = get_aggregator("fedavg", uh)          # one aggregator across reps: a session's rounds
        for rep in range(WARM + reps):       # the first rounds ramp the GPU clocks and pin result blocks
            for i, (s, n) in enumerate(zip(ups, ns)):
                uh.submit(s, n, i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            model, data = agg.combine_models(helper=None)
            if rep >= WARM:
                ts.append(time.perf_counter() - t0)
        res.setdefault(mode, []).append((sorted(ts)[len(ts) // 2], model[0], data))
    staging.BATCH = 64
    same = all(np.array_equal(r[1].view(np.uint32), res["batched"][0][1].view(np.uint32))
               for v in res.values() for r in v)
    for mode in ("batched", "per-update"):
        t, _, data = min(res[mode], key=lambda r: r[0])
        print(json.dumps({"config": f"fedavg {K} x {P} fp32, device-resident at round end", "mode": mode,
                          "combine_models_s": t, "params_per_s": K * P / t,
                          "d2h_floor_s": P * 4 / 57e9, "time_kernel": data.get("time_kernel"),
                          "time_d2h": data.get("time_d2h"), "bit_identical": same}), flush=True)


def run_fedopt(K, P, reps):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    old32 = torch.randn(P, generator=g, device=dev)
    ups = staged_updates(K, P, 4, base=old32)
    ns = [int(v) for v in np.random.default_rng(4).integers(1, 5001, K)]
    old_host = [old32.cpu().numpy()]
    res = {}
    for mode, batch in (("batched", 64), ("per-update", 1), ("batched", 64)):
        staging.BATCH = batch
        ts = []
        for _ in range(reps):
            uh = DeviceResidentHandler()
            agg = get_aggregator("fedopt", uh)
            params = {"serveropt": "adam"}
            # round 1 (untimed) makes m / v / the old model fp64, as in a running session
            uh.globals["g0"] = old_host
            for i, (s, n) in enumerate(zip(ups, ns)):
                uh.submit(s, n, i, "g0")
            m1, _ = agg.combine_models(helper=None, parameters=params)
            uh.globals["g1"] = m1
            for i, (s, n) in enumerate(zip(ups, ns)):
                uh.submit(s, n, i, "g1")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            model, data = agg.combine_models(helper=None, parameters=params)
            ts.append(time.perf_counter() - t0)
            del m1
        res.setdefault(mode, []).append((sorted(ts)[len(ts) // 2], model[0], data))
    staging.BATCH = 64
    same = all(np.array_equal(r[1].view(np.uint64), res["batched"][0][1].view(np.uint64))
               for v in res.values() for r in v)
    for mode in ("batched", "per-update"):
        t, _, data = min(res[mode], key=lambda r: r[0])
        print(json.dumps({"config": f"fedopt adam round 2, {K} x {P} fp32 updates, fp64 state, device-resident",
                          "mode": mode, "combine_models_s": t, "params_per_s": K * P / t,
                          "note": "includes the H2D of the fp64 global model (load_model returns host arrays) "
                                  "and the D2H of the fp64 result",
                          "time_kernel": data.get("time_kernel"), "time_d2h": data.get("time_d2h"),
                          "bit_identical": same}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="fedavg,fedopt")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    _abi.load()
    torch.cuda.set_device(0)
    if "fedavg" in a.which:
        run_fedavg(64, 100_000_000, a.reps)
        torch.cuda.empty_cache()
    if "fedopt" in a.which:
        run_fedopt(32, 350_000_000, a.reps)


if __name__ == "__main__":
    main()
