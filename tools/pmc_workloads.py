"""One bench.py kernel workload per process, for rocprofv3 PMC passes whose kernels must not share a
template instantiation with another workload of the same run (tools/gpu_session.sh step "pmcx";
tools/pmc_traffic.py --x-session turns the passes into profiles/pmc_traffic.json entries).

  f32state   configs[3] steady state in the fp32-state mode: 32 fp32 updates x 350 M, f32 old / m / v,
             k_fedopt_c<float, float, CF32, FIRST, FINAL> (the same instantiation as round 1)
  waves      configs[4]'s three wave kernels on one device (1 B bf16 params, waves of 8, FedYogi,
             round 1 of a session as bench.py's fedopt_waves times them): FIRST wave, a later wave,
             the K = 0 FINAL server step, the last wave with FINAL fused (the same instantiation as
             the K = 0 step: its dispatches come after those) — device-resident here (the PCIe copies
             are not measured)
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402

Q, K3 = 350_000_000, 32
PW, W = 1_000_000_000, 8


def f32state(steps):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(4)
    old = torch.randn(Q, generator=g, device=dev)
    ups = [torch.randn(Q, generator=g, device=dev).mul_(0.01).add_(old) for _ in range(K3)]
    ns = [int(v) for v in np.random.default_rng(4).integers(1, 5001, K3)]
    Ns = [int(v) for v in np.cumsum(ns)]
    m = torch.randn(Q, generator=g, device=dev).mul_(0.001)
    v = torch.rand(Q, generator=g, device=dev).mul_(1e-4)
    mo, vo, out = (torch.empty(Q, device=dev) for _ in range(3))
    for _ in range(steps):
        ops.fedopt_step(old, ups, ns, Ns, first=True, final=True, m_in=m, m_out=mo, v_in=v, v_out=vo, out=out)
    torch.cuda.synchronize()


def waves(steps):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    old = torch.randn(PW, generator=g, device=dev, dtype=torch.float64)
    ups = [(old + 0.01 * torch.randn(PW, generator=g, device=dev, dtype=torch.float64)).to(torch.bfloat16)
           for _ in range(W)]
    ns = [int(v) for v in np.random.default_rng(5).integers(1, 5001, W)]
    Ns = [int(v) for v in np.cumsum(ns)]
    pg = torch.empty(PW, dtype=torch.float64, device=dev)
    m, v, out = (torch.empty(PW, dtype=torch.float64, device=dev) for _ in range(3))
    for _ in range(steps):
        ops.fedopt_step(old, ups, ns, Ns, first=True, final=False, pg=pg)
    for _ in range(steps):
        ops.fedopt_step(old, ups, ns, [N + Ns[-1] for N in Ns], first=False, final=False, pg=pg)
    for _ in range(steps):
        ops.fedopt_step(old, [], [], [], first=False, final=True, pg=pg, m_out=m, v_out=v, out=out,
                        serveropt="yogi", upd_dtype=torch.bfloat16)
    for _ in range(steps):     # the last wave with the server step fused (the same instantiation, K = 8)
        ops.fedopt_step(old, ups, ns, [N + Ns[-1] for N in Ns], first=False, final=True, pg=pg, m_out=m, v_out=v,
                        out=out, serveropt="yogi")
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=["f32state", "waves"])
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    _abi.load()
    torch.cuda.set_device(0)
    {"f32state": f32state, "waves": waves}[a.workload](a.steps)
    print(f"pmc_workloads {a.workload}: {a.steps} launches each", flush=True)


if __name__ == "__main__":
    main()
