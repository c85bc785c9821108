"""fednamdhelper primitives (numpyhelper.py:34-142) on float16 and 8 / 16 / 32 / 64-bit integer
tensors, against numpy itself — the reference helper's arithmetic (numpyhelper.py:44-141 call numpy
directly). No golden fixture covers these dtypes: parity here is pinned to numpy on the same
inputs, bit for bit for every float result (float16 pow with a general exponent and the norm of a
float16 tensor aside: numpy's own half loops, 1e-3 relative)."""
import numpy as np
import pytest

from fedn_amd._abi import FedAggError
from fedn_amd.helper import Helper

pytestmark = pytest.mark.gpu

INTS = [np.int8, np.int16, np.int32, np.int64, np.uint8, np.uint16, np.uint32, np.uint64]


def _data(dt, shape=(37, 29), seed=0):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dt)
    if dt.kind == "f":
        return (rng.standard_normal(shape) * 3).astype(dt)
    info = np.iinfo(dt)
    lo, hi = max(info.min, -1000), min(info.max, 1000)
    return rng.integers(lo, hi, size=shape, endpoint=True).astype(dt)


def _same(g, w, what):
    g, w = np.asarray(g), np.asarray(w)
    assert g.dtype == w.dtype and g.shape == w.shape, f"{what}: {g.dtype}{g.shape} vs {w.dtype}{w.shape}"
    if w.dtype.kind == "f":
        assert np.array_equal(np.isnan(g), np.isnan(w)), what
        ok = ~np.isnan(w)
        assert np.array_equal(g[ok].view(np.uint8), w[ok].view(np.uint8)), what
    else:
        assert np.array_equal(g, w), what


@pytest.mark.parametrize("dt", INTS)
@pytest.mark.parametrize("e", [0, 1, 2, 3, 7])
def test_int_power_wraps_like_numpy(dt, e):
    x = _data(dt)
    _same(Helper().power([x], e)[0], np.power(x, e), f"{np.dtype(dt)} ** {e}")


@pytest.mark.parametrize("dt", INTS + [np.float16])
def test_norm_narrow_and_half(dt):
    x2, x1 = _data(dt, (40, 31), 1), _data(dt, (513,), 2)
    got = Helper().norm([x2, x1])
    want = 0.0
    for x in (x2, x1):
        want += np.linalg.norm(x, 1)
    assert type(got) is type(want)
    if np.dtype(dt) == np.float16:
        assert abs(float(got) - float(want)) <= 1e-3 * abs(float(want))
    else:
        assert got == want


@pytest.mark.parametrize("dt", [np.float16] + INTS)
def test_single_ops_half_and_int(dt):
    """multiply / divide by arrays and python scalars, sqrt, sign, ones: numpy's result dtype and
    bits (integer results — integer multiply, sign — are refused, not computed on the host)."""
    h = Helper()
    x, y = _data(dt, seed=3), _data(dt, seed=4)
    y = np.where(y == 0, np.ones_like(y), y)
    with np.errstate(all="ignore"):
        cases = {"div_arr": (lambda: h.divide([x], [y]), lambda: np.divide(x, y)),
                 "mul_scalar": (lambda: h.multiply([x], [0.37]), lambda: np.multiply(x, 0.37)),
                 "div_scalar": (lambda: h.divide([x], [3.1]), lambda: np.divide(x, 3.1)),
                 "sqrt": (lambda: h.sqrt([np.abs(x) if np.dtype(dt).kind != "u" else x]),
                          lambda: np.sqrt(np.abs(x) if np.dtype(dt).kind != "u" else x)),
                 "ones": (lambda: h.ones([x], 0.25), lambda: np.ones(x.shape) * 0.25),
                 "mul_arr": (lambda: h.multiply([x], [y]), lambda: np.multiply(x, y)),
                 "sign": (lambda: h.sign([x]), lambda: np.sign(x))}
        for name, (g, w) in cases.items():
            want = w()
            if want.dtype.kind != "f":
                with pytest.raises(FedAggError):
                    g()
                continue
            _same(g()[0], want, f"{np.dtype(dt)} {name}")


@pytest.mark.parametrize("pair", [(np.float16, np.float16), (np.float16, np.float32), (np.float32, np.float16),
                                  (np.int8, np.int8), (np.int32, np.float32), (np.uint16, np.float16),
                                  (np.int64, np.int64), (np.float16, np.float64)])
def test_add_subtract_mixed(pair):
    """numpyhelper.add / subtract = x*a + y*b (numpyhelper.py:34-56): each product in its own dtype,
    the sum in the promoted one."""
    h = Helper()
    x, y = _data(pair[0], seed=5), _data(pair[1], seed=6)
    with np.errstate(all="ignore"):
        _same(h.add([x], [y], 0.9, 0.1)[0], x * 0.9 + y * 0.1, f"add {pair}")
        _same(h.subtract([x], [y], 1.0, 1.0)[0], x * 1.0 + y * -1.0, f"subtract {pair}")


def test_half_power_square_exact():
    x = _data(np.float16, seed=7)
    _same(Helper().power([x], 2.0)[0], np.power(x, 2.0), "f16 ** 2.0")
    g = Helper().power([np.abs(x)], 0.5)[0]
    w = np.power(np.abs(x), 0.5)
    assert g.dtype == w.dtype == np.float16
    assert np.allclose(g.astype(np.float64), w.astype(np.float64), rtol=1e-3, atol=0)
