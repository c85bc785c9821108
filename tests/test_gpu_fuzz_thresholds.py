"""The fuzz rounds of test_gpu_fuzz.py with the staging pipeline's size thresholds shrunk to the
fuzz's model sizes, so that random layouts of a few KB to a few hundred KB take the paths that in
production only models of 4 MB to GBs take: piecewise pack + H2D with one fold launch per piece
(STAGE_PIECES_MIN / STAGE_PIECE, piece boundaries at odd byte offsets that split elements), the
result's chunked D2H (MIN_CHUNK_BYTES), arenas holding one or two updates with partial uploads
(ARENA_BYTES / ARENA_UPLOAD_EVERY), zero-copy folds of the arena on or off (ZERO_COPY_BYTES),
small update batches per launch (BATCH), FedOpt's pinned ring for the global model (RING_BYTES), the host pack inline or on the native
gather's threads (layout.PACK_MIN_PARALLEL / PACK_CHUNK) and the large / small split itself
(SMALL_UPDATE_BYTES). Every threshold is read by staging.py at call time; the values are drawn per
seed. Bar: bit-exact values and dtypes against the oracle, every update counted."""
import numpy as np
import pytest
import torch

from golden_io import assert_lists_identical
from oracle import numpy_ref as ref
from test_gpu_fuzz import _aggregator, _clients, _handlers, _helper, _layout, _seeds, _submit_all, _values


ROUTES = ["host", "staged", "npz", "sliced", "staged_sliced"]


@pytest.fixture
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fedn_amd import _abi
    _abi.load()


def _thresholds(seed, monkeypatch):
    from fedn_amd import staging
    rng = np.random.default_rng(5000 + seed)
    pick = lambda *v: v[int(rng.integers(0, len(v)))]   # noqa: E731
    t = {"SMALL_UPDATE_BYTES": pick(1024, 16 << 10, 4 << 20),
         "STAGE_PIECES_MIN": pick(8 << 10, 64 << 10),
         "STAGE_PIECE": pick(4096, 6000, 12_345, 65_536),
         "MIN_CHUNK_BYTES": pick(4096, 8 << 20),
         "ARENA_BYTES": pick(8 << 10, 64 << 20),
         "ARENA_UPLOAD_EVERY": pick(1, 2, 16),
         "ZERO_COPY_BYTES": pick(0, 1 << 30),
         "BATCH": pick(1, 3, 64)}
    for k, v in t.items():
        monkeypatch.setattr(staging, k, v)
    # FedOpt's global model streams through a ring of pinned pieces (HostStreamer, RING_BYTES bound
    # as its default argument)
    t["RING_BYTES"] = pick(4096, 6000, 64 << 20)
    monkeypatch.setattr(staging.HostStreamer.__init__, "__defaults__", (3, t["RING_BYTES"]))
    # the host pack: inline vs the native gather's threads, and the parallel copy's piece size
    from fedn_amd import layout
    t["PACK_MIN_PARALLEL"] = pick(0, 1 << 20)
    t["PACK_CHUNK"] = pick(4096, 16 << 20)
    monkeypatch.setattr(layout, "PACK_MIN_PARALLEL", t["PACK_MIN_PARALLEL"])
    monkeypatch.setattr(layout, "PACK_CHUNK", t["PACK_CHUNK"])
    return t


def _big_layout(rng):
    """test_gpu_fuzz's layouts, and in 2 of 3 cases one more tensor of 3 k - 60 k elements, so that
    most updates cross the shrunk thresholds."""
    shapes, dtypes = _layout(rng)
    if rng.random() < 2 / 3:
        shapes.append((int(rng.integers(3_000, 60_000)),))
        dtypes.append(dtypes[0])
    return shapes, dtypes


def _nbytes(shapes, dtypes):
    return sum(int(np.prod(s)) * np.dtype(d).itemsize for s, d in zip(shapes, dtypes))


def test_fuzz_thresholds_reach_the_paths():
    """(CPU) the drawn cases do reach the piecewise path and the small (arena) path."""
    pieces = small = 0
    for seed in range(40):
        from fedn_amd import staging
        mp = pytest.MonkeyPatch()
        try:
            t = _thresholds(seed, mp)
            nb = _nbytes(*_big_layout(np.random.default_rng(3000 + seed)))
            pieces += nb > t["SMALL_UPDATE_BYTES"] and nb >= t["STAGE_PIECES_MIN"] and nb > t["STAGE_PIECE"]
            small += nb <= t["SMALL_UPDATE_BYTES"]
        finally:
            mp.undo()
        assert staging.BATCH == 64
    assert pieces >= 10 and small >= 5, (pieces, small)


@pytest.mark.gpu
@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("seed", _seeds(40))
def test_fuzz_thresholds_fedavg(seed, route, monkeypatch, _gpu):
    t = _thresholds(seed, monkeypatch)
    rng = np.random.default_rng(3000 + seed)
    shapes, dtypes = _big_layout(rng)
    K = int(rng.integers(1, 25))
    base = [_values(rng, s, d) for s, d in zip(shapes, dtypes)]
    ups, ns = _clients(rng, shapes, dtypes, K, base, mixed=seed % 4 == 0)
    want, nr = ref.fedavg_combine(list(zip(ups, ns)))
    uh, st = _handlers(route)
    try:
        agg = _aggregator("fedavg", route, uh, st, monkeypatch)
        _submit_all(route, uh, st, ups, ns)
        model, data = agg.combine_models(helper=_helper(route), delete_models=True)
    finally:
        if st is not None:
            st.close()
    assert data["nr_aggregated_models"] == nr == K
    assert_lists_identical(model, want, f"seed {seed} {route} {t} shapes {shapes} dtypes {dtypes} K {K}")


@pytest.mark.gpu
@pytest.mark.parametrize("route", ROUTES)
@pytest.mark.parametrize("seed", _seeds(24))
def test_fuzz_thresholds_fedopt(seed, route, monkeypatch, _gpu):
    t = _thresholds(100 + seed, monkeypatch)
    rng = np.random.default_rng(4000 + seed)
    shapes, dtypes = _big_layout(rng)
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
            ups, ns = _clients(rng, shapes, dtypes, K, old, mixed=seed % 5 == 2)
            gid = uh.put_global_model(old, f"g{r}")
            _submit_all(route, uh, st, ups, ns, model_id=gid)
            model, data = agg.combine_models(helper=_helper(route), delete_models=True, parameters=params)
            want, nr = ref.fedopt_combine(state, list(zip(ups, ns)), old, params)
            what = f"seed {seed} {route} {opt} round {r} {t} shapes {shapes} dtypes {dtypes} K {K}"
            assert data["nr_aggregated_models"] == nr == K, what
            assert_lists_identical(model, want, what)
            assert_lists_identical(agg.m, state.m, what + " m")
            assert_lists_identical(agg.v, state.v, what + " v")
            old = model
    finally:
        if st is not None:
            st.close()
