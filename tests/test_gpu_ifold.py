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


NARROW = [np.int8, np.int16, np.uint8, np.uint16, np.uint32, np.uint64, np.int32, np.int64]


def _rand_ints(rng, dtype, P):
    info = np.iinfo(dtype)
    x = rng.integers(info.min, info.max, P, dtype=dtype, endpoint=True)
    x[:4] = [info.max, info.min, 0, info.max - 1]
    return x


@pytest.mark.parametrize("dtype", NARROW)
@pytest.mark.parametrize("n,N", [(3, 7), (100, 3000), (1, 2), (0, 5)])
def test_nfold_matches_numpy(dtype, n, N):
    """NFOLD: a python-int num_examples multiplies the wrapped difference in the array's dtype
    (numpy's weak int scalar), then true_divide by N and add x in float64."""
    from fedn_amd import ops
    rng = np.random.default_rng(int(np.dtype(dtype).num) * 31 + n)
    P = 65_537
    x, y = _rand_ints(rng, dtype, P), _rand_ints(rng, dtype, P)
    y[:4] = [np.iinfo(dtype).min, np.iinfo(dtype).max, 1, 0]
    with np.errstate(over="ignore"):
        want = np.add(x, np.true_divide(np.multiply(n, np.subtract(y, x)), N))
    assert want.dtype == np.float64
    out = torch.empty(P, dtype=torch.float64, device=DEV)
    ops.elementwise("nfold", out, torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV), float(n), float(N))
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want.view(np.uint64))


@pytest.mark.parametrize("dtype", NARROW)
def test_ifold_narrow_matches_numpy(dtype):
    from fedn_amd import ops
    rng = np.random.default_rng(int(np.dtype(dtype).num))
    P = 65_537
    x, y = _rand_ints(rng, dtype, P), _rand_ints(rng, dtype, P)
    n, N = 2.5, 7.25
    with np.errstate(over="ignore"):
        want = np.add(x, np.true_divide(np.multiply(n, np.subtract(y, x)), N))
    out = torch.empty(P, dtype=torch.float64, device=DEV)
    ops.elementwise("ifold", out, torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV), n, N)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want.view(np.uint64))


_SAFE = [np.int16, np.int32, np.int64, np.uint16, np.uint32, np.uint64, np.float16, np.float32, np.float64]


@pytest.mark.parametrize("src", [np.int8, np.int16, np.uint8, np.uint16, np.uint32, np.uint64])
def test_cast_narrow_matches_numpy(src):
    """fa_cast from narrow / unsigned integers to each dtype numpy casts them to safely, plus a
    broadcast (1,) -> (n,) and (3, 1) -> (3, 4); unsafe targets are refused."""
    from fedn_amd import _abi, ops
    rng = np.random.default_rng(int(np.dtype(src).num) + 100)
    x = _rand_ints(rng, src, 4099)
    for dst in _SAFE + [src]:
        if not np.can_cast(src, dst, "safe"):
            with pytest.raises(_abi.FedAggError):
                ops.cast(torch.empty(4099, dtype=ops.torch_dtype(dst), device=DEV), torch.from_numpy(x).to(DEV))
            continue
        out = torch.empty(4099, dtype=ops.torch_dtype(dst), device=DEV)
        ops.cast(out, torch.from_numpy(x).to(DEV))
        want = x.astype(dst)
        got = out.cpu().numpy()
        assert got.dtype == want.dtype and np.array_equal(got.view(np.uint8), want.view(np.uint8)), dst
    b = torch.from_numpy(x[:3].reshape(3, 1).copy()).to(DEV)
    out = torch.empty((3, 4), dtype=torch.float64, device=DEV)
    ops.cast(out, b)
    assert np.array_equal(out.cpu().numpy(), np.broadcast_to(x[:3].reshape(3, 1), (3, 4)).astype(np.float64))


def test_nfold_rejects_huge_n():
    from fedn_amd import _abi, ops
    x = torch.zeros(8, dtype=torch.uint64, device=DEV)
    with pytest.raises(_abi.FedAggError):
        ops.elementwise("nfold", torch.empty(8, dtype=torch.float64, device=DEV), x, x, float(1 << 60), 3.0)


@pytest.mark.parametrize("dtypes,n,N", [((np.int8, np.uint16), 37, 1234), ((np.uint32, np.int16), 2.5, 9.0),
                                       ((np.uint64, np.int8), 5, 11)])
def test_helper_increment_average_narrow(dtypes, n, N):
    """fednamdhelper.increment_average (the stock fedavg.py loop's fold) on narrow / unsigned tensors,
    against the oracle's numpyhelper.increment_average."""
    from golden_io import assert_lists_identical
    from oracle import numpy_ref as ref
    from fedn_amd.helper import Helper
    rng = np.random.default_rng(77)
    m1 = [_rand_ints(rng, dt, 1000 + 7 * i).reshape(-1) for i, dt in enumerate(dtypes)]
    m2 = [_rand_ints(rng, dt, 1000 + 7 * i).reshape(-1) for i, dt in enumerate(dtypes)]
    with np.errstate(over="ignore"):
        want = ref.increment_average(m1, m2, n, N)
    assert_lists_identical(Helper().increment_average(m1, m2, n, N), want, str(dtypes))
