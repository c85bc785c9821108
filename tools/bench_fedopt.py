"""FedOpt benchmarks (BASELINE.json configs[3] and configs[4]); results go to DESIGN.md.

config4  350 M fp32 params, 32 device-resident client updates, FedAdam. One fused launch
         (pseudo-gradient fold + server step). Round 1 (old fp32, m/v None) and steady state
         (old/m/v fp64, the dtype flow fedopt.py produces), bytes P*(4K+48) per step.
config5  1 B bf16 params, 128 client updates streamed from pinned host memory in waves of W,
         FedYogi, H2D of wave i+1 overlapped with the fold of wave i (fa_fedopt_step without
         FINAL keeps the running pseudo-gradient in HBM), then the server step. The host pool
         holds `pool` distinct pinned updates reused cyclically (256 GB of distinct bf16
         updates does not fit the box's host memory); every update still crosses PCIe.
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

PEAK = 8000.0


def timed(fn, reps=5, warm=2):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return sorted(s.elapsed_time(e) for s, e in ev)[reps // 2]


def config4(P, K, opt):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(4)
    old32 = torch.randn(P, generator=g, device=dev)
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(old32) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(4).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    out = torch.empty(P, dtype=torch.float64, device=dev)
    v = torch.empty(P, dtype=torch.float64, device=dev)
    m32 = torch.empty(P, dtype=torch.float32, device=dev)
    # round 1: old fp32, m/v None -> m fp32, v fp64
    r1 = lambda: ops.fedopt_step(old32, ups, ns, Ns, first=True, final=True, m_out=m32, v_out=v, out=out,  # noqa: E731
                                 serveropt=opt)
    ms1 = timed(r1)
    b1 = K * P * 4 + P * 4 + P * (4 + 8 + 8)
    old64 = out.clone()
    m64 = m32.double()
    r2 = lambda: ops.fedopt_step(old64, ups, ns, Ns, first=True, final=True, m_in=m64, m_out=m64, v_in=v, v_out=v,  # noqa: E731
                                 out=out, serveropt=opt)
    ms2 = timed(r2)
    b2 = P * (4 * K + 48)
    for name, ms, b in (("round1", ms1, b1), ("steady", ms2, b2)):
        print(json.dumps({"config": "config4", "opt": opt, "phase": name, "params": P, "clients": K, "ms": ms,
                          "params_per_s": K * P / ms * 1e3, "GBps": b / ms / 1e6, "frac_hbm": b / ms / 1e6 / PEAK,
                          "alg_bytes": b}), flush=True)


def config4_ab(P, K, opts, settings):
    """Kernel A/B on configs[3]: fp64 division knob (fastdiv64 0 = IEEE, 1 = RN64(1/N) + Markstein),
    round 1 and steady state, outputs checked bit-identical to the first setting's."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(4)
    old32 = torch.randn(P, generator=g, device=dev)
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(old32) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(4).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    out = torch.empty(P, dtype=torch.float64, device=dev)
    v = torch.empty(P, dtype=torch.float64, device=dev)
    m32 = torch.empty(P, dtype=torch.float32, device=dev)
    m64o = torch.empty(P, dtype=torch.float64, device=dev)
    v2 = torch.empty(P, dtype=torch.float64, device=dev)
    out2 = torch.empty(P, dtype=torch.float64, device=dev)
    for opt in opts:
        ref = None
        # fixed steady-state inputs (old/m/v fp64) from one round-1 step with the default knobs
        ops.tune(fastdiv64=0)
        ops.fedopt_step(old32, ups, ns, Ns, first=True, final=True, m_out=m32, v_out=v, out=out, serveropt=opt)
        old64, m64, v64 = out.clone(), m32.double(), v.clone()
        for fd in settings:
            ops.tune(fastdiv64=fd)
            r1 = lambda: ops.fedopt_step(old32, ups, ns, Ns, first=True, final=True, m_out=m32, v_out=v,  # noqa: E731
                                         out=out, serveropt=opt)
            ms1 = timed(r1)
            r2 = lambda: ops.fedopt_step(old64, ups, ns, Ns, first=True, final=True, m_in=m64, m_out=m64o,  # noqa: E731
                                         v_in=v64, v_out=v2, out=out2, serveropt=opt)
            ms2 = timed(r2)
            got = [t.clone() for t in (out, m32, v, out2, m64o, v2)]
            if ref is None:
                ref = got
            same = all(torch.equal(a.view(torch.int32) if a.dtype == torch.float32 else a.view(torch.int64),
                                   b.view(torch.int32) if b.dtype == torch.float32 else b.view(torch.int64))
                       for a, b in zip(got, ref))
            b1 = K * P * 4 + P * 4 + P * (4 + 8 + 8)
            b2 = P * (4 * K + 48)
            print(json.dumps({"config": "config4", "opt": opt, "fastdiv64": fd,
                              "round1_ms": ms1, "round1_GBps": b1 / ms1 / 1e6, "steady_ms": ms2,
                              "steady_GBps": b2 / ms2 / 1e6, "steady_frac": b2 / ms2 / 1e6 / PEAK,
                              "bit_identical_to_first": same}), flush=True)
            del got
    ops.tune(fastdiv64=1)


def config5(P, K, W, pool, opt, ndev=1, check=True):
    """BASELINE configs[4]: K bf16 updates of P params streamed from pinned host memory in waves of
    W (fedn_amd.waves.WaveFedOpt), FedYogi, parameter-sliced over ``ndev`` devices (each copies only
    its slice of every update over its own PCIe link). Reports per-link H2D GB/s and a checksum of
    the result; with ``check`` the result is compared bit-for-bit with a one-device run."""
    import hashlib

    from fedn_amd.waves import WaveFedOpt
    ngpu = torch.cuda.device_count()
    devs = [torch.device("cuda", d % ngpu) for d in range(ndev)]
    g = torch.Generator(device="cuda:0").manual_seed(5)
    old = torch.randn(P, generator=g, device="cuda:0", dtype=torch.float64)
    host = []
    for _ in range(pool):
        h = torch.empty(P, dtype=torch.bfloat16, pin_memory=True)
        h.copy_((old + 0.01 * torch.randn(P, generator=g, device="cuda:0", dtype=torch.float64)).to(torch.bfloat16))
        host.append(h)
    ups = [host[k % pool] for k in range(K)]
    ns = [int(v) for v in np.random.default_rng(5).integers(1, 5001, K)]
    params = {"serveropt": opt}
    old_h = old.cpu()

    def run(devices):
        wf = WaveFedOpt(devices, P, wave=W)
        old_d = wf.slices(old_h)
        for dv in devices:
            torch.cuda.synchronize(dv)
        t0 = time.perf_counter()
        outs = wf.round(ups, ns, old_d, params)
        t = time.perf_counter() - t0
        return wf.gather(outs), t, wf

    out, t, wf = run(devs)
    digest = hashlib.sha256(out.numpy().tobytes()).hexdigest()[:16]
    line = {"config": "config5", "opt": opt, "params": P, "clients": K, "wave": W, "devices": len(devs),
            "distinct_gpus": len({str(d) for d in devs}), "s": t, "params_per_s": K * P / t,
            "h2d_GBps_total": K * P * 2 / t / 1e9,
            "h2d_GBps_per_link": [K * (hi - lo) * 2 / t / 1e9 for lo, hi in wf.bounds],
            "checksum_sha256_16": digest,
            "note": f"{pool} distinct pinned bf16 updates reused cyclically; every update still crosses PCIe"}
    if check and len(devs) > 1:
        ref_out, t1, _ = run([devs[0]])
        line["bit_identical_to_1_device"] = bool(torch.equal(out.view(torch.int64), ref_out.view(torch.int64)))
        line["s_1_device"] = t1
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="4,5")
    ap.add_argument("--p4", type=int, default=350_000_000)
    ap.add_argument("--k4", type=int, default=32)
    ap.add_argument("--p5", type=int, default=1_000_000_000)
    ap.add_argument("--k5", type=int, default=128)
    ap.add_argument("--wave", type=int, default=8)
    ap.add_argument("--pool", type=int, default=16)
    ap.add_argument("--devices", type=int, default=1, help="config5: parameter slices over this many devices")
    ap.add_argument("--ab", action="store_true", help="A/B the FedOpt traversal and fp64 division knobs")
    a = ap.parse_args()
    _abi.load()
    torch.cuda.set_device(0)
    if a.ab:
        _abi.use_probe()          # fa_tune (fastdiv64 A/B) lives in libfedagg_probe.so
        config4_ab(a.p4, a.k4, ("adam", "yogi", "adagrad"), [0, 1, 0, 1])
        return
    if "4" in a.which:
        for opt in ("adam", "yogi", "adagrad"):
            config4(a.p4, a.k4, opt)
            torch.cuda.empty_cache()
    if "5" in a.which:
        config5(a.p5, a.k5, a.wave, a.pool, "yogi", a.devices)


if __name__ == "__main__":
    main()
