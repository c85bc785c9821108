"""fa_elementwise IFOLD: numpyhelper.increment_average (numpyhelper.py:32) on integer arrays with a
python-float num_examples — the integer difference wraps, then float64 multiply / divide / add —
bit-exact against numpy itself on random, extreme (wrapping) and large-|d| values."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.mark.parametrize("dtype", [np.int32, np.int64])
@pytest.mark.parametrize("n,N", [(2.5, 7.5), (1e-3, 3.0), (3.0e15, 3.0e15 + 2), (-0.0, 1.0), (7.0, 10)])
def test_ifold_matches_numpy(dtype, n, N):
    from fedn_amd import ops
    info = np.iinfo(dtype)
    rng = np.random.default_rng(5)
    P = 100_003
    x = rng.integers(info.min, info.max, P, dtype=dtype, endpoint=True)
    y = rng.integers(info.min, info.max, P, dtype=dtype, endpoint=True)
    x[:6] = [info.max, info.min, 0, -1, info.max, 1 << 20]
    y[:6] = [info.min, info.max, 0, 1, info.max - 1, (1 << 20) + 3]
    x[6:1006] = rng.integers(-1000, 1000, 1000)
    y[6:1006] = x[6:1006] + rng.integers(-50, 50, 1000)
    with np.errstate(over="ignore"):
        want = np.add(x, np.true_divide(np.multiply(n, np.subtract(y, x)), N))
    assert want.dtype == np.float64
    out = torch.empty(P, dtype=torch.float64, device=DEV)
    ops.elementwise("ifold", out, torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV), float(n), float(N))
    got = out.cpu().numpy()
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_ifold_rejects_float_inputs():
    from fedn_amd import _abi, ops
    x = torch.zeros(8, dtype=torch.float32, device=DEV)
    with pytest.raises(_abi.FedAggError):
        ops.elementwise("ifold", torch.empty(8, dtype=torch.float64, device=DEV), x, x, 2.5, 3.0)


def test_int_first_fold_rejects_float_n():
    """fa_fedavg_fold folds the first integer difference in the integer dtype, which is numpy's rule
    for an int num_examples only: a non-integral n is refused (the plug-ins route it to IFOLD)."""
    from fedn_amd import _abi, ops
    x = torch.arange(16, dtype=torch.int64, device=DEV)
    out = torch.empty(16, dtype=torch.float64, device=DEV)
    with pytest.raises(_abi.FedAggError):
        ops.fedavg_fold(out, [x, x + 3], [0, 2.5], [1, 3.5], init=True)
    ops.fedavg_fold(out, [x, x + 3], [0, 2.0], [1, 3.0], init=True)      # integral: the int path
    want = np.add(np.arange(16), 2 * (np.arange(16) + 3 - np.arange(16)) / 3.0)
    assert np.array_equal(out.cpu().numpy(), want)
