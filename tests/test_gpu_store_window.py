"""The chip-wide store window (fedagg.hip avg_store_window / opt_store_window) moves
stores in time only: the windowed kernels (k_fedavg_pipe_win, k_fedopt_cw) return the unwindowed
kernels' bits. Compared through the probe library, whose fa_tune knobs switch the window off (-1) or
leave the product's own choice (0), at sizes where the product picks a window (>= 2^24 elements; FedOpt
steady state from 32 clients)."""
import numpy as np
import pytest
import torch

from fedn_amd import _abi, ops

pytestmark = pytest.mark.gpu

P = (1 << 24) + 4096 * 3 + 1000          # a window, and a ragged last tile


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _same(a, b):
    return torch.equal(a.view(torch.uint8), b.view(torch.uint8))


@pytest.mark.parametrize("K", [8, 64])
def test_fedavg_window_is_bit_identical(dev, K):
    g = torch.Generator(device=dev).manual_seed(K)
    base = torch.randn(P, generator=g, device=dev)
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(base) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(K).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    out = {}
    with _abi.use_probe():
        try:
            for mode in (-1, 0, 7000):
                ops.tune(avg_win_period=mode, avg_win_w=700)
                agg = torch.empty(P, device=dev)
                ops.fedavg_fold(agg, ups, ns, Ns, True)
                torch.cuda.synchronize()
                out[mode] = agg
        finally:
            ops.tune(avg_win_period=0)
    assert _same(out[-1], out[0]) and _same(out[-1], out[7000])


@pytest.mark.parametrize("phase", ["round1", "steady"])
def test_fedopt_window_is_bit_identical(dev, phase):
    K = 32
    g = torch.Generator(device=dev).manual_seed(7)
    old32 = torch.randn(P, generator=g, device=dev)
    ups = [torch.randn(P, generator=g, device=dev).mul_(0.01).add_(old32) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(3).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    res = {}
    with _abi.use_probe():
        try:
            for mode in (-1, 0):
                ops.tune(opt_win_period=mode, opt_win_prod=0)
                out = torch.empty(P, dtype=torch.float64, device=dev)
                v = torch.empty(P, dtype=torch.float64, device=dev)
                m = torch.empty(P, dtype=torch.float32, device=dev)
                ops.fedopt_step(old32, ups, ns, Ns, first=True, final=True, m_out=m, v_out=v, out=out)
                if phase == "steady":
                    old64, m64, v64 = out.clone(), m.double(), v.clone()
                    m = torch.empty(P, dtype=torch.float64, device=dev)
                    v = torch.empty(P, dtype=torch.float64, device=dev)
                    out = torch.empty(P, dtype=torch.float64, device=dev)
                    ops.fedopt_step(old64, ups, ns, Ns, first=True, final=True, m_in=m64, m_out=m, v_in=v64, v_out=v,
                                    out=out)
                torch.cuda.synchronize()
                res[mode] = (out, m, v)
        finally:
            ops.tune(opt_win_period=0)
    assert all(_same(a, b) for a, b in zip(res[-1], res[0]))


@pytest.mark.parametrize("first", [True, False])
def test_pipeline_wave_window_is_bit_identical(dev, first):
    """k_fedopt_cwp (probe: a pipeline wave's pg stores in the window) vs k_fedopt_c: bf16 updates, fp64 pg."""
    W = 8
    g = torch.Generator(device=dev).manual_seed(11)
    old = torch.randn(P, generator=g, device=dev, dtype=torch.float64)
    ups = [(old.float() + 0.01 * torch.randn(P, generator=g, device=dev)).to(torch.bfloat16) for _ in range(W)]
    ns = [float(v) for v in np.random.default_rng(5).integers(1, 5001, W)]
    Ns = [float(v) for v in np.cumsum(ns)]
    pg0 = torch.empty(P, dtype=torch.float64, device=dev)
    ops.fedopt_step(old, ups, ns, Ns, first=True, final=False, pg=pg0)
    res = {}
    with _abi.use_probe():
        try:
            for mode, w in ((-1, 0), (0, 0), (600, 150)):
                ops.tune(opt_win_period=mode, opt_win_w=w if mode > 0 else 0, opt_win_prod=1 if mode > 0 else 0)
                pg = pg0.clone()
                ops.fedopt_step(old, ups, ns, Ns, first=first, final=False, pg=pg)
                torch.cuda.synchronize()
                res[mode] = pg
        finally:
            ops.tune(opt_win_period=0, opt_win_prod=0)
    assert _same(res[-1], res[0]) and _same(res[-1], res[600])
