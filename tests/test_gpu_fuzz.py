"""Seeded random rounds through the plug-ins vs the oracle (itself pinned to FEDn's own outputs by
tests/golden): random layouts — 1-7 tensors of rank 0-3, empty and one-element tensors, odd sizes,
now and then a tensor large enough for the multi-strip tiles — in float32 / float64 / float16, K = 1-24
clients, now and then a client whose tensor differs in dtype (numpy promotion, the per-tensor path),
each round through the host path (small rounds: native admission, arena, zero-copy), through the
streaming ingest (updates staged into HBM on arrival), as npz bytes inflated by the native codec
into the ingest, and sliced over two device entries in one process (multidev.py; this box's GPU
listed twice), from the host or staged on arrival as parameter slices. FedAvg one round, FedOpt (adam / yogi /
adagrad, random hyper-parameters) three rounds with m / v carried. Bar: bit-exact values and dtypes,
every update counted — the same bar as the golden fixtures, on cases no fixture spells out."""
import os

import numpy as np
import pytest
import torch

from golden_io import assert_lists_identical
from oracle import numpy_ref as ref

pytestmark = pytest.mark.gpu

# extended runs: FEDN_AMD_FUZZ_BASE shifts every seed range, FEDN_AMD_FUZZ_SCALE multiplies its length
_BASE = int(os.environ.get("FEDN_AMD_FUZZ_BASE", "0"))
_SCALE = float(os.environ.get("FEDN_AMD_FUZZ_SCALE", "1"))


def _seeds(n):
    return range(_BASE, _BASE + max(1, int(n * _SCALE)))


DEV = "cuda:0"
DTYPES = [np.float32, np.float64, np.float16]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fedn_amd import _abi
    _abi.load()


def _layout(rng):
    T = int(rng.integers(1, 8))
    shapes = []
    for _ in range(T):
        r = rng.random()
        if r < 0.1:
            shapes.append(())                                   # a scalar tensor
        elif r < 0.2:
            shapes.append((0,) if rng.random() < 0.5 else (3, 0))   # empty
        elif r < 0.3:
            shapes.append((int(rng.integers(20_000, 90_000)),))     # crosses several tiles
        else:
            nd = int(rng.integers(1, 4))
            shapes.append(tuple(int(rng.integers(1, 41)) for _ in range(nd)))
    one = DTYPES[int(rng.integers(0, 3))]
    dtypes = [one if rng.random() < 0.7 else DTYPES[int(rng.integers(0, 3))] for _ in shapes]
    return shapes, dtypes


def _values(rng, shape, dtype, base=None, scale=1.0):
    x = rng.standard_normal(shape) * scale
    if base is not None:
        x = base.astype(np.float64) + 0.01 * x
    x = np.asarray(x).astype(dtype)
    if x.size and rng.random() < 0.3:                          # exact zeros and a signed zero
        x.reshape(-1)[:: max(1, x.size // 5)] = 0
        x.reshape(-1)[0] = -0.0
    return x


def _clients(rng, shapes, dtypes, K, base, mixed):
    ups = []
    for k in range(K):
        u = [_values(rng, s, d, b) for s, d, b in zip(shapes, dtypes, base)]
        if mixed and k > 0 and rng.random() < 0.15 and u:       # a client whose tensor differs in dtype
            i = int(rng.integers(0, len(u)))
            u[i] = u[i].astype(DTYPES[(DTYPES.index(u[i].dtype.type) + 1) % 3])
        ups.append(u)
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    return ups, ns


ROUTES = ["host", "staged", "npz", "sliced", "staged_sliced"]


def _submit_all(route, uh, st, ups, ns, model_id="global"):
    import io
    for a, n in zip(ups, ns):
        if route == "npz":
            b = io.BytesIO()
            np.savez_compressed(b, **{str(i): t for i, t in enumerate(a)})
            uh.submit_bytes(b.getvalue(), n, model_id=model_id, via=st)
        else:
            uh.submit(a, n, model_id=model_id, via=st if route in ("staged", "staged_sliced") else None)


def _handlers(route):
    from fedn_amd.helper import Helper
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    uh = MemoryUpdateHandler()
    st = None
    if route == "staged":
        st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=2)
    elif route == "npz":
        st = StagingUpdateHandler(uh, helper=Helper(), device=DEV, workers=2, native_decode=True)
    elif route == "staged_sliced":           # staged on arrival as parameter slices over two device entries
        st = StagingUpdateHandler(uh, helper=None, devices=[DEV, DEV], workers=2)
    return uh, st


def _aggregator(kind, route, uh, st, monkeypatch):
    from fedn_amd.aggregators import fedavg, fedopt
    mod = fedavg if kind == "fedavg" else fedopt
    if route in ("sliced", "staged_sliced"):
        from fedn_amd import layout
        monkeypatch.setattr(layout, "MULTIDEV_MIN_BYTES", 0)     # slice even these small models
        return mod.Aggregator(st or uh, devices=[DEV, DEV])
    return mod.Aggregator(st or uh)


def _helper(route):
    from fedn_amd.helper import Helper
    return Helper() if route == "npz" else None


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("seed", _seeds(48))
def test_fuzz_fedavg(seed, route, monkeypatch):
    rng = np.random.default_rng(1000 + seed)
    shapes, dtypes = _layout(rng)
    K = int(rng.integers(1, 25))
    base = [_values(rng, s, d) for s, d in zip(shapes, dtypes)]
    ups, ns = _clients(rng, shapes, dtypes, K, base, mixed=seed % 3 == 0)
    want, nr = ref.fedavg_combine(list(zip(ups, ns)))
    uh, st = _handlers(route)
    try:
        agg = _aggregator("fedavg", route, uh, st, monkeypatch)      # (the slicing rule set before staging)
        _submit_all(route, uh, st, ups, ns)
        model, data = agg.combine_models(helper=_helper(route), delete_models=True)
    finally:
        if st is not None:
            st.close()
    assert data["nr_aggregated_models"] == nr == K
    assert_lists_identical(model, want, f"seed {seed} {route} shapes {shapes} dtypes {dtypes} K {K}")


@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("seed", _seeds(30))
def test_fuzz_fedopt(seed, route, monkeypatch):
    rng = np.random.default_rng(2000 + seed)
    shapes, dtypes = _layout(rng)
    opt = ["adam", "yogi", "adagrad"][seed % 3]
    params = {"serveropt": opt, "learning_rate": float(10 ** rng.uniform(-4, -1)),
              "beta1": float(rng.uniform(0.5, 0.99)), "beta2": float(rng.uniform(0.9, 0.9999)),
              "tau": float(10 ** rng.uniform(-6, -2))}
    old = [_values(rng, s, d) for s, d in zip(shapes, dtypes)]
    uh, st = _handlers(route)
    agg = _aggregator("fedopt", route, uh, st, monkeypatch)
    state = ref.FedOptState()
    try:
        for r in range(3):
            K = int(rng.integers(1, 17))
            ups, ns = _clients(rng, shapes, dtypes, K, old, mixed=seed % 4 == 1)
            gid = uh.put_global_model(old, f"g{r}")
            _submit_all(route, uh, st, ups, ns, model_id=gid)
            model, data = agg.combine_models(helper=_helper(route), delete_models=True, parameters=params)
            want, nr = ref.fedopt_combine(state, list(zip(ups, ns)), old, params)
            what = f"seed {seed} {route} {opt} round {r} shapes {shapes} dtypes {dtypes} K {K}"
            assert data["nr_aggregated_models"] == nr == K, what
            assert_lists_identical(model, want, what)
            assert_lists_identical(agg.m, state.m, what + " m")
            assert_lists_identical(agg.v, state.v, what + " v")
            old = model
    finally:
        if st is not None:
            st.close()
