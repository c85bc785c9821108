"""The chip-wide store windows beside other GPU work.

k_fedavg_pipe_win (the BASELINE workload: 64 x 100 M fp32, first launch) and k_fedopt_cw (configs[3]:
FedAdam, 32 x 350 M fp32, round 1 and steady state) hold every wave's stores until a common window of
the GPU's 100 MHz clock: premised on all of the chip's stores being bunched, they gain 4-7 % alone.
Here each is timed against its unwindowed twin (fa_tune AVG_WIN_PERIOD / OPT_WIN_PERIOD = -1 on the
probe library: the same body, stores whenever ready) in three settings:

  alone     nothing else on the GPU
  h2d       a 4 GiB pinned-host -> HBM copy running on another stream (a pipeline's staging)
  fold2     a second FedAvg fold (8 x 100 M fp32, no window) queued on another stream, so two
            sessions' kernels share the CUs

Kernel time = HIP events on the measured kernel's own stream; windowed and unwindowed interleaved,
median of --reps. Every windowed result is compared bit for bit with its twin's.

  python tools/window_concurrent.py [--reps 7]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--avg-params", type=int, default=100_000_000)
    ap.add_argument("--opt-params", type=int, default=350_000_000)
    ap.add_argument("--h2d-gib", type=float, default=4.0)
    a = ap.parse_args()
    _abi.use_probe()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    main_st = torch.cuda.Stream(dev)
    bg = torch.cuda.Stream(dev)
    g = torch.Generator(device=dev).manual_seed(6)

    # background work
    host = torch.empty(int(a.h2d_gib * (1 << 30)), dtype=torch.uint8, pin_memory=True)
    host_dst = torch.empty_like(host, device=dev)
    P2 = 100_000_000
    bg_ups = [torch.randn(P2, generator=g, device=dev) for _ in range(8)]
    bg_agg = torch.empty(P2, device=dev)
    bg_ns = [int(v) for v in np.random.default_rng(2).integers(1, 5001, 8)]
    bg_Ns = [int(v) for v in np.cumsum(bg_ns)]

    def background(kind):
        if kind == "h2d":
            with torch.cuda.stream(bg):
                host_dst.copy_(host, non_blocking=True)        # ~70 ms at PCIe rate: spans the kernel
        elif kind == "fold2":
            for _ in range(24):                                # ~15 ms of folds queued ahead
                ops.fedavg_fold(bg_agg, bg_ups, bg_ns, bg_Ns, init=True, stream=bg)

    # the measured kernels
    P = a.avg_params
    ups = [torch.randn(P, generator=g, device=dev) for _ in range(64)]
    agg = torch.empty(P, device=dev)
    ns = [int(v) for v in np.random.default_rng(64).integers(1, 5001, 64)]
    Ns = [int(v) for v in np.cumsum(ns)]
    Po, K = a.opt_params, 32
    old32 = torch.randn(Po, generator=g, device=dev)
    oups = [torch.randn(Po, generator=g, device=dev).mul_(0.01).add_(old32) for _ in range(K)]
    ons = [int(v) for v in np.random.default_rng(32).integers(1, 5001, K)]
    oNs = [int(v) for v in np.cumsum(ons)]
    kw = {"learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4, "serveropt": "adam"}
    out1 = torch.empty(Po, dtype=torch.float64, device=dev)
    m32 = torch.empty(Po, dtype=torch.float32, device=dev)
    v1 = torch.empty(Po, dtype=torch.float64, device=dev)
    old64 = torch.randn(Po, generator=g, device=dev, dtype=torch.float64)
    m64 = torch.randn(Po, generator=g, device=dev, dtype=torch.float64).mul_(1e-3)
    v64 = torch.rand(Po, generator=g, device=dev, dtype=torch.float64).mul_(1e-6)
    m_o, v_o, out2 = (torch.empty(Po, dtype=torch.float64, device=dev) for _ in range(3))

    work = {
        "fedavg_k64_100M": (lambda s: ops.fedavg_fold(agg, ups, ns, Ns, init=True, stream=s), "avg_win_period",
                            [agg], 64 * P * 4 + P * 4),
        "fedadam_round1_k32_350M": (lambda s: ops.fedopt_step(old32, oups, ons, oNs, first=True, final=True, m_out=m32,
                                                              v_out=v1, out=out1, stream=s, **kw),
                                    "opt_win_period", [out1, m32, v1], K * Po * 4 + Po * 24),
        "fedadam_steady_k32_350M": (lambda s: ops.fedopt_step(old64, oups, ons, oNs, first=True, final=True, m_in=m64,
                                                              m_out=m_o, v_in=v64, v_out=v_o, out=out2, stream=s, **kw),
                                    "opt_win_period", [out2, m_o, v_o], Po * (4 * K + 48)),
    }
    res = {"params": {"reps": a.reps, "h2d_gib": a.h2d_gib, "fold2": "8 x 100 M fp32 folds, 24 queued"}}
    for name, (fn, knob, outs, alg) in work.items():
        # bit-identity and which kernel each setting ran
        ran, bits = {}, {}
        for var, period in (("window", 0), ("no_window", -1)):
            ops.tune(**{knob: period})
            fn(main_st)
            main_st.synchronize()
            ran[var] = ops.last_kernel()
            bits[var] = [o.clone() for o in outs]
        exact = all(torch.equal(x.view(torch.uint8), y.view(torch.uint8)) for x, y in zip(bits["window"], bits["no_window"]))
        del bits
        row = {"kernel": ran, "bit_identical": exact, "alg_bytes": alg}
        for setting in ("alone", "h2d", "fold2"):
            times = {"window": [], "no_window": []}
            for _ in range(a.reps):
                for var, period in (("window", 0), ("no_window", -1)):
                    ops.tune(**{knob: period})
                    torch.cuda.synchronize()
                    background(setting)
                    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s_.record(main_st)
                    fn(main_st)
                    e_.record(main_st)
                    torch.cuda.synchronize()
                    times[var].append(s_.elapsed_time(e_))
            med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
            row[setting] = {"window_ms": round(med["window"], 4), "no_window_ms": round(med["no_window"], 4),
                            "window_gain": round(1 - med["window"] / med["no_window"], 4),
                            "window_tbs": round(alg / med["window"] / 1e9, 3)}
            print(json.dumps({"workload": name, "setting": setting, **row[setting]}), flush=True)
        ops.tune(**{knob: 0})
        res[name] = row
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
