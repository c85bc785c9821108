"""configs[0]'s one-call round (fedn_amd/smallround.py) against the oracle, bit for bit: the mnist-pytorch
model (examples/mnist-pytorch model.py:18-32) and other small float models through the FedAvg plug-in
(fedavg.py:45-83), and every way a round leaves that path for the general pipeline — an update of
another dtype or shape, one too many for the arena, a failed launch — with the admitted updates
replayed in FIFO order. Also: a model a caller still holds is never overwritten by a later round
(pooled result blocks are reused only once nothing views them)."""
import numpy as np
import pytest
import torch

from oracle import numpy_ref as ref

pytestmark = pytest.mark.gpu

MNIST = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fedn_amd import _abi
    _abi.load()


def _models(rng, shapes, K, dtype=np.float32):
    base = [rng.standard_normal(s).astype(dtype) for s in shapes]
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(dtype) for b in base] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    return list(zip(ups, ns))


def _same(got, want):
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g.dtype == w.dtype and g.shape == w.shape
        assert np.array_equal(g.view(np.uint8), w.view(np.uint8))


def _agg():
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    uh = MemoryUpdateHandler()
    return uh, get_aggregator("fedavg", uh)


def _round(uh, agg, updates):
    for arrays, n in updates:
        uh.submit(arrays, n)
    return agg.combine_models(helper=None)


def _spy(agg, monkeypatch):
    """Counts of rounds that took the one-call path and rounds handed to the general pipeline."""
    from fedn_amd import smallround
    seen = {"small": 0, "general": 0}
    real_result, real_general = smallround.SmallRound.result, smallround.SmallRound.general

    def result(self):
        seen["small"] += 1
        return real_result(self)

    def general(self, make):
        seen["general"] += 1
        return real_general(self, make)
    monkeypatch.setattr(smallround.SmallRound, "result", result)
    monkeypatch.setattr(smallround.SmallRound, "general", general)
    return seen


@pytest.mark.parametrize("K", [1, 2, 3, 10, 19])
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.float16])
def test_small_round_is_the_oracle(K, dtype, monkeypatch):
    rng = np.random.default_rng(K * 7 + np.dtype(dtype).itemsize)
    updates = _models(rng, MNIST, K, dtype)
    uh, agg = _agg()
    seen = _spy(agg, monkeypatch)
    from fedn_amd import staging
    cap = staging.ZERO_COPY_BYTES // sum(int(np.prod(s)) * np.dtype(dtype).itemsize for s in MNIST)
    for _ in range(3):                       # a session: the arena, plans and blocks are reused
        model, data = _round(uh, agg, updates)
        want, nr = ref.fedavg_combine(updates)
        assert data["nr_aggregated_models"] == nr == K
        _same(model, want)
        assert uh.model_updates.qsize() == 0 and not uh.store.models    # every folded update deleted
    if K <= min(cap, 64):
        assert seen == {"small": 3, "general": 0}
    else:                                    # the queue showed a round larger than the arena
        assert seen == {"small": 0, "general": 0}
    if K == 1:
        assert model[0] is updates[0][0][0]  # the first update itself (fedavg.py:65-66)


def test_a_held_model_is_never_overwritten():
    """The arrays a round returns view a pooled pinned block: the next rounds must take another block
    while those arrays live, and may reuse it once they are dropped."""
    rng = np.random.default_rng(3)
    uh, agg = _agg()
    rounds = [_models(rng, MNIST, 2) for _ in range(8)]
    held = []
    for ups in rounds:
        model, _ = _round(uh, agg, ups)
        held.append((model, [a.copy() for a in model], ups))
    for model, copy, ups in held:           # every model still as its round left it
        _same(model, copy)
        _same(model, ref.fedavg_combine(ups)[0])
    base_ptrs = {m[0].__array_interface__["data"][0] for m, _, _ in held}
    assert len(base_ptrs) == 8               # eight live models, eight blocks
    del held, model
    ptrs = []
    for ups in rounds[:3]:                   # models dropped at once: a pooled block comes back
        model, _ = _round(uh, agg, ups)
        _same(model, ref.fedavg_combine(ups)[0])
        ptrs.append(model[0].__array_interface__["data"][0])
        del model
    assert len(set(ptrs)) == 1


def test_other_dtype_or_shape_goes_general_in_fifo_order(monkeypatch):
    rng = np.random.default_rng(5)
    ups = _models(rng, MNIST, 5)
    uh, agg = _agg()
    seen = _spy(agg, monkeypatch)
    mixed = list(ups)
    mixed[3] = ([a.astype(np.float64) for a in ups[3][0]], ups[3][1])      # numpy promotes from here on
    model, data = _round(uh, agg, mixed)
    want, nr = ref.fedavg_combine(mixed)
    assert data["nr_aggregated_models"] == nr == 5
    _same(model, want)
    assert seen["general"] == 1
    bad = list(ups)
    bad[2] = ([a[:, :2] if a.ndim == 2 else a for a in ups[2][0]], ups[2][1])     # not broadcastable: skipped
    model, data = _round(uh, agg, bad)
    want, nr = ref.fedavg_combine(bad)
    assert data["nr_aggregated_models"] == nr == 4
    _same(model, want)
    assert list(uh.store.models) != []               # the skipped update stays in storage (fedavg.py:71-78)


@pytest.mark.parametrize("queue_visible", [True, False])
def test_more_updates_than_the_arena_goes_general(monkeypatch, queue_visible):
    """A round the queue shows to be larger than the arena goes the general way from its first update;
    one whose updates outgrow the arena unseen (they arrived during the round) is handed over part-way,
    its admitted updates replayed in order."""
    from fedn_amd import staging
    monkeypatch.setattr(staging, "ZERO_COPY_BYTES", 3 * 210_688)      # a 3-update arena for mnist
    rng = np.random.default_rng(6)
    ups = _models(rng, MNIST, 7)
    uh, agg = _agg()
    seen = _spy(agg, monkeypatch)
    if not queue_visible:
        monkeypatch.setattr(agg, "_queued", lambda: 0)
    model, data = _round(uh, agg, ups)
    want, nr = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == nr == 7
    _same(model, want)
    assert seen == ({"small": 0, "general": 0} if queue_visible else {"small": 0, "general": 1})


def test_failed_launch_recovers_through_the_general_path(monkeypatch):
    from fedn_amd import ops, smallround
    rng = np.random.default_rng(8)
    ups = _models(rng, MNIST, 4)
    uh, agg = _agg()

    def boom(self, *a, **k):
        raise ops.FedAggError(3, "injected launch failure")
    monkeypatch.setattr(smallround.SmallSession, "fold", boom)
    model, data = _round(uh, agg, ups)
    want, nr = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == nr == 4
    _same(model, want)
    assert uh.model_updates.qsize() == 0


def test_fold_host_refuses_pageable_memory():
    from fedn_amd import _abi
    import ctypes
    lib = _abi.load()
    a = np.zeros(1024, np.float32)
    b = np.ones(1024, np.float32)
    ptrs = (ctypes.c_void_p * 2)(a.ctypes.data, b.ctypes.data)
    n = (ctypes.c_double * 2)(0.0, 1.0)
    N = (ctypes.c_double * 2)(1.0, 2.0)
    rc = lib.fa_fedavg_fold_host(a.ctypes.data, _abi.FA_F32, ptrs, _abi.FA_F32, n, N, 2, 1024, 1, None)
    assert rc == _abi.FA_EINVAL and b"page-locked" in lib.fa_last_error()


# ---------------------------------------------------------------- FedOpt (fedopt.py:74-121, 151-258)
def _opt_agg():
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    uh = MemoryUpdateHandler()
    return uh, get_aggregator("fedopt", uh)


def _opt_spy(monkeypatch):
    from fedn_amd import smallround
    seen = {"small": 0, "general": 0}
    real_step, real_general = smallround.SmallFedOptRound.server_step, smallround.SmallFedOptRound.general

    def step(self, state, params):
        seen["small"] += 1
        return real_step(self, state, params)

    def general(self):
        seen["general"] += 1
        return real_general(self)
    monkeypatch.setattr(smallround.SmallFedOptRound, "server_step", step)
    monkeypatch.setattr(smallround.SmallFedOptRound, "general", general)
    return seen


@pytest.mark.parametrize("opt", ["adam", "yogi", "adagrad"])
@pytest.mark.parametrize("K", [1, 2, 5, 19])
def test_small_fedopt_round_is_the_oracle(K, opt, monkeypatch):
    """Three rounds of a session: fp32 clients over the fp32 global model, then over the float64 model
    the previous round returned (FEDn stores FedOpt's float64 output as the next global model); m / v
    carried in HBM, every round and the state bit-exact to the oracle."""
    rng = np.random.default_rng(90 + K)
    base = [rng.standard_normal(s).astype(np.float32) for s in MNIST]
    params = {"serveropt": opt, "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
    uh, agg = _opt_agg()
    seen = _opt_spy(monkeypatch)
    st, old = ref.FedOptState(), base
    for r in range(3):
        ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 5001, K)]
        gid = uh.put_global_model(old, f"g{r}")
        for a, n in zip(ups, ns):
            uh.submit(a, n, model_id=gid)
        model, data = agg.combine_models(helper=None, parameters=params)
        want, nr = ref.fedopt_combine(st, list(zip(ups, ns)), old, params)
        assert data["nr_aggregated_models"] == nr == K
        _same(model, want)
        _same(agg.m, st.m)
        _same(agg.v, st.v)
        assert uh.model_updates.qsize() == 0 and all(k.startswith("g") for k in uh.store.models)   # updates deleted
        old = model                          # held by the caller: its block must not be reused
    assert seen == {"small": 3, "general": 0}


def test_small_fedopt_goes_general_on_another_layout(monkeypatch):
    rng = np.random.default_rng(95)
    base = [rng.standard_normal(s).astype(np.float32) for s in MNIST]
    uh, agg = _opt_agg()
    seen = _opt_spy(monkeypatch)
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(4)]
    ups[2] = [a.astype(np.float64) for a in ups[2]]               # numpy promotes from here on
    ns = [int(v) for v in rng.integers(1, 5001, 4)]
    gid = uh.put_global_model(base, "g0")
    for a, n in zip(ups, ns):
        uh.submit(a, n, model_id=gid)
    model, data = agg.combine_models(helper=None)
    st = ref.FedOptState()
    want, nr = ref.fedopt_combine(st, list(zip(ups, ns)), base)
    assert data["nr_aggregated_models"] == nr == 4
    _same(model, want)
    _same(agg.m, st.m)
    assert seen["general"] == 1


def test_fedopt_step_host_refuses_pageable_memory():
    from fedn_amd import _abi
    import ctypes
    lib = _abi.load()
    old = np.zeros(256, np.float32)
    upd = np.ones(256, np.float32)
    out = np.zeros(256, np.float64)
    m = torch.empty(256, dtype=torch.float64, device="cuda:0")
    v = torch.empty(256, dtype=torch.float64, device="cuda:0")
    ptrs = (ctypes.c_void_p * 1)(upd.ctypes.data)
    n = (ctypes.c_double * 1)(1.0)
    rc = lib.fa_fedopt_step_host(old.ctypes.data, _abi.FA_F32, ptrs, _abi.FA_F32, n, n, 1, None, _abi.FA_NONE,
                                 m.data_ptr(), _abi.FA_F64, None, _abi.FA_F64, v.data_ptr(), out.ctypes.data,
                                 _abi.FA_F64, _abi.FA_ADAM, 1e-3, 0.9, 0.99, 1e-4, 256, None)
    assert rc == _abi.FA_EINVAL and b"page-locked" in lib.fa_last_error()


@pytest.mark.parametrize("shapes", [[(0,), (3, 0)], [(0,), (64,), (0, 5), (10,)]], ids=["all_empty", "some_empty"])
def test_empty_tensors_fedavg_and_fedopt(shapes, monkeypatch):
    """Zero-size tensors through the one-call way: a model of only empty tensors (a 0-element fold, the
    layout's 256-B minimum arena slot) and one with empty tensors among others, FedAvg and FedOpt, two
    rounds each: the oracle's bits, shapes and dtypes."""
    rng = np.random.default_rng(11)
    seen = _spy(None, monkeypatch)
    uh, agg = _agg()
    for _ in range(2):
        updates = _models(rng, shapes, 3)
        model, data = _round(uh, agg, updates)
        want, nr = ref.fedavg_combine(updates)
        assert data["nr_aggregated_models"] == nr == 3
        _same(model, want)
    assert seen == {"small": 2, "general": 0}
    oseen = _opt_spy(monkeypatch)
    uh, agg = _opt_agg()
    st = ref.FedOptState()
    old = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    for r in range(2):
        ups = _models(rng, shapes, 3)
        gid = uh.put_global_model(old, f"g{r}")
        for a, n in ups:
            uh.submit(a, n, model_id=gid)
        model, data = agg.combine_models(helper=None)
        want, nr = ref.fedopt_combine(st, ups, old)
        assert data["nr_aggregated_models"] == nr == 3
        _same(model, want)
        _same(agg.m, st.m)
        _same(agg.v, st.v)
        old = model
    assert oseen == {"small": 2, "general": 0}
