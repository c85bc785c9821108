"""FedOpt pipeline waves (BASELINE configs[4] shape: W bf16 updates over an fp64 model, pg in fp64)
with and without the chip-wide store window on their pg stores (k_fedopt_cwp vs k_fedopt_c;
fa_tune OPT_WIN_PERIOD -1 / 0 = none — the product's waves take no window, this probe's result —,
> 0 with OPT_WIN_PROD = 1 = explicit period / window): the first and a middle launch, bit-for-bit against the unwindowed wave,
interleaved repeats, median ms. Probe library.

  python tools/wave_window_probe.py [--params N] [--wave 8] [--win period:w,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402

PEAK = 8000.0


def median_ms(fn, n=5):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for s_, e_ in ev:
        s_.record()
        fn()
        e_.record()
    torch.cuda.synchronize()
    return sorted(s_.elapsed_time(e_) for s_, e_ in ev)[n // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=250_000_000)
    ap.add_argument("--wave", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--win", default="400:100,700:160,1000:230,1500:350,2500:580")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    P, W = a.params, a.wave
    g = torch.Generator(device=dev).manual_seed(1)
    old = torch.randn(P, generator=g, device=dev, dtype=torch.float64)
    ups = [(old.float() + 0.01 * torch.randn(P, generator=g, device=dev)).to(torch.bfloat16) for _ in range(W)]
    ns = [float(i + 1) for i in range(W)]
    Ns = [float(sum(ns[: i + 1])) for i in range(W)]
    pg_in = torch.empty(P, dtype=torch.float64, device=dev)
    ops.fedopt_step(old, ups, ns, Ns, first=True, final=False, pg=pg_in)
    pg = torch.empty_like(pg_in)
    variants = [("none", -1, 0), ("model", 0, 0)] + [
        (f"{p}:{w}", int(p), int(w)) for p, w in (x.split(":") for x in a.win.split(",") if x)]
    rows = []
    with _abi.use_probe():
        try:
            for phase in ("first", "mid"):
                bytes_ = P * (2 * W + 8 + (0 if phase == "first" else 8) + 8)
                res, ref = {}, None
                for _ in range(a.reps):
                    for name, per, w in variants:
                        ops.tune(opt_win_period=per, opt_win_w=max(w, 1) if per > 0 else 0, opt_win_prod=1 if per > 0 else 0)
                        first = phase == "first"

                        def step():
                            ops.fedopt_step(old, ups, ns, Ns, first=first, final=False, pg=pg)
                        pg.copy_(pg_in)
                        step()
                        torch.cuda.synchronize()
                        out = pg.clone()
                        if ref is None:
                            ref = out
                        exact = bool(torch.equal(ref.view(torch.uint8), out.view(torch.uint8)))
                        ms = median_ms(step)             # a middle wave keeps folding into pg: timing only
                        res.setdefault(name, []).append((ms, exact))
                for name, v in res.items():
                    ms = sorted(m for m, _ in v)[len(v) // 2]
                    row = {"phase": phase, "variant": name, "ms": round(ms, 4),
                           "frac": round(bytes_ / ms / 1e6 / PEAK, 4), "bit_exact": all(e for _, e in v)}
                    rows.append(row)
                    print(json.dumps(row), flush=True)
                none = [r for r in rows if r["phase"] == phase and r["variant"] == "none"][0]["ms"]
                best = min((r for r in rows if r["phase"] == phase), key=lambda r: r["ms"])
                print(json.dumps({"phase": phase, "none_ms": none, "best": best["variant"],
                                  "best_vs_none": round(best["ms"] / none - 1, 4)}), flush=True)
        finally:
            ops.tune(opt_win_period=0, opt_win_prod=0)


if __name__ == "__main__":
    main()
