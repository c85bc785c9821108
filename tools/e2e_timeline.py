"""Timeline of the host-resident FedAvg round through the plug-in (tools/bench_e2e.py's ``plugin``
mode): per update, the wall time its pack starts / ends and the GPU time its H2D starts / ends
(HIP events, relative to the first H2D), so DMA idle gaps can be attributed. Diagnostic only."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, staging  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--slots", type=int, nargs="+", default=[3])
    ap.add_argument("--pageable", action="store_true", help="updates in pageable numpy memory (FEDn's np.load)")
    a = ap.parse_args()
    _abi.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K, P = a.clients, a.params
    rng = np.random.default_rng(0)
    base = rng.standard_normal(P, dtype=np.float32)
    ups = []
    for _ in range(K):
        if a.pageable:
            ups.append(base + np.float32(0.01) * rng.standard_normal(P, dtype=np.float32))
        else:
            h = torch.empty(P, dtype=torch.float32, pin_memory=True)
            h.numpy()[:] = base + np.float32(0.01) * rng.standard_normal(P, dtype=np.float32)
            ups.append(h.numpy())
    ns = [int(v) for v in rng.integers(1, 5001, K)]

    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    marks = []
    real_stage = staging._Pipeline.stage

    def stage(self, arrays):
        t0 = time.perf_counter()
        s = real_stage(self, arrays)
        marks.append((t0, time.perf_counter(), self._h2d[-1]))
        return s

    staging._Pipeline.stage = stage
    for nslots in a.slots:
        orig_init = staging.FedAvgPipeline.__init__

        def init(self, device, first_arrays, nslots_=3, slots=None, streams=None, _n=nslots):
            orig_init(self, device, first_arrays, _n, slots, streams)

        staging.FedAvgPipeline.__init__ = init
        uh = MemoryUpdateHandler()
        agg = Aggregator(uh, device=dev)
        for rnd in range(2):                      # round 1 warms the pinned pool
            for k in range(K):
                uh.submit([ups[k]], ns[k])
            marks.clear()
            t0 = time.perf_counter()
            model, data = agg.combine_models(helper=None)
            t = time.perf_counter() - t0
        staging.FedAvgPipeline.__init__ = orig_init
        torch.cuda.synchronize()
        e0 = marks[0][2][0]
        rows = []
        for w0, w1, (hs, he) in marks:
            rows.append({"pack_start_ms": round((w0 - t0) * 1e3, 2), "pack_end_ms": round((w1 - t0) * 1e3, 2),
                         "h2d_start_ms": round(e0.elapsed_time(hs), 2), "h2d_end_ms": round(e0.elapsed_time(he), 2)})
        gaps = [round(rows[i + 1]["h2d_start_ms"] - rows[i]["h2d_end_ms"], 2) for i in range(len(rows) - 1)]
        print(json.dumps({"slots": nslots, "pageable": a.pageable, "round_s": round(t, 4),
                          "h2d_busy_ms": round(sum(r["h2d_end_ms"] - r["h2d_start_ms"] for r in rows), 2),
                          "gaps_ms": gaps, "first_pack_end_ms": rows[0]["pack_end_ms"],
                          "last_h2d_end_ms": rows[-1]["h2d_end_ms"],
                          "data": {k: round(v, 4) for k, v in data.items() if isinstance(v, float)},
                          "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
