"""CPU tests of the native small-update admission (fedn_amd/csrc/fastpack.c via
layout.fast_admission): it must admit exactly what staging._Pipeline.fast_host admits, pack the
same bytes as Layout.pack, and leave anything else to the general path (-1)."""
import numpy as np
import pytest

from fedn_amd import layout as L
from fedn_amd.layout import Layout, fast_admission, wait_pack_jobs

pytest.importorskip("fedn_amd._fastpack")

MNIST = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]


def _model(rng, shapes, dtypes):
    return [rng.standard_normal(s).astype(d) for s, d in zip(shapes, dtypes)]


def _packed(lay, arrays):
    out = np.zeros(lay.nbytes, np.uint8)
    lay.pack(arrays, out)
    return out


@pytest.mark.parametrize("shapes,dtypes", [
    (MNIST, ["f4"] * 6),
    ([(3, 5), (0,), (7,), (2, 0, 4), (1,)], ["f4", "f4", "f8", "f8", "f2"]),
    ([(1000,), (17,), (4, 4)], ["f8", "f4", "f8"]),
    ([(0,), (0, 3)], ["f4", "f4"]),
])
def test_admit_packs_like_layout(shapes, dtypes):
    rng = np.random.default_rng(0)
    first = _model(rng, shapes, dtypes)
    lay = Layout.of(first)
    admit = fast_admission(lay)
    assert admit is not None
    for _ in range(3):
        upd = _model(rng, shapes, dtypes)
        buf = np.full(lay.nbytes, 0xAB, np.uint8)
        t = admit(upd, buf.ctypes.data)
        assert t >= 0
        if t:
            wait_pack_jobs(t)
        want = _packed(lay, upd)
        # bytes of the layout's padding are not written; every tensor's bytes are
        for i, off, nb in lay.pack_plan:
            assert np.array_equal(buf[off:off + nb], want[off:off + nb]), i
    assert fast_admission(lay) is admit                     # cached per layout


def test_admit_refuses_other_layouts():
    rng = np.random.default_rng(1)
    m = _model(rng, MNIST, ["f4"] * 6)
    lay = Layout.of(m)
    admit = fast_admission(lay)
    buf = np.zeros(lay.nbytes, np.uint8)
    before = buf.copy()

    class Sub(np.ndarray):
        pass

    bad = [
        m[:5],                                               # fewer tensors
        m + [m[0]],                                          # more tensors
        tuple(m),                                            # not a list
        [m[0].astype(np.float64)] + m[1:],                   # dtype
        [m[0].astype(">f4")] + m[1:],                        # byte order
        [m[0].T.copy()] + m[1:],                             # shape
        [m[0].reshape(-1)] + m[1:],                          # ndim
        [np.asfortranarray(m[0])] + m[1:],                   # not C-contiguous
        [m[0][::-1]] + m[1:],                                # negative strides
        [m[0].view(Sub)] + m[1:],                            # a subclass (fast_host refuses it too)
        [m[0].tolist()] + m[1:],                             # not an array
    ]
    for arrays in bad:
        assert admit(arrays, buf.ctypes.data) == -1
    assert np.array_equal(buf, before)                       # nothing queued, nothing written


def test_admission_missing_extension(monkeypatch):
    """Without the extension the pipelines keep the Python admission (same bytes, slower)."""
    monkeypatch.setattr(L, "_FAST", False)
    lay = Layout.of([np.ones(4, np.float32), np.ones(2, np.float32)])
    monkeypatch.delattr(lay, "_fast_admit", raising=False)
    assert fast_admission(lay) is None
    monkeypatch.delattr(lay, "_fast_admit")                # the next test sees the extension again
