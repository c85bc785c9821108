"""Per-update failure isolation in batched rounds (fedavg.py:75-78, fedopt.py:103-106).

The plug-ins fold small host updates, and every update the ingest staged in HBM, in multi-client
launches (one per <= 64 updates), and a small round in ONE zero-copy launch. FEDn folds one update at
a time: an update whose fold raises is logged and skipped, its examples stay counted, and the round
goes on. Here, a batch whose launch fails is refolded one update at a time from its staged copies
(arena, slot or HBM); only the updates whose own fold fails are skipped, uncounted, and kept in
storage (FEDn deletes an update only after its fold, fedavg.py:71-74).

A "poisoned" update is simulated at the C-ABI wrapper: every launch whose client table holds its
(num_examples, running total) pair raises FedAggError before anything is enqueued, as a failing
status would. The expected model is the oracle's with that update's fold raising.
"""
import inspect

import numpy as np
import pytest
import torch

from golden_io import assert_lists_identical
from oracle import numpy_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
FOLD_OPS = ("fedavg_fold", "fedavg_fold_ptrs", "fedavg_fold_raw", "fedavg_fold_host", "fedopt_step", "fedopt_step_raw",
            "fedopt_step_host")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fedn_amd import _abi
    _abi.load()


def _poison(monkeypatch, pairs):
    """Every fold launch whose (n, N) lists contain one of ``pairs`` raises FedAggError."""
    from fedn_amd import _abi, ops
    hits = []
    for name in FOLD_OPS:
        real = getattr(ops, name)
        sig = inspect.signature(real)

        def wrapper(*a, _real=real, _sig=sig, _name=name, **kw):
            b = _sig.bind(*a, **kw)
            ns, Ns = b.arguments["n"], b.arguments["N"]
            if any((float(x), float(y)) in pairs for x, y in zip(ns, Ns)):
                hits.append((_name, len(ns)))
                raise _abi.FedAggError(_abi.FA_EHIP, f"{_name}: injected failure (poisoned update in the table)")
            return _real(*a, **kw)

        monkeypatch.setattr(ops, name, wrapper)
    return hits


def _clients(rng, shapes, K, base):
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
    ns = [int(v) for v in rng.choice(np.arange(1, 5001), K, replace=False)]
    return ups, ns


SMALL = [(30, 7), (5,), (64,)]                # packed well under staging.SMALL_UPDATE_BYTES: arena batches
LARGE = [(1100, 1000), (333,)]                # > 4 MiB: staged updates, chunked result launch


def _handlers(route):
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    uh = MemoryUpdateHandler()
    st = None
    if route.startswith("staged_sliced"):
        st = StagingUpdateHandler(uh, helper=None, devices=[DEV, DEV], workers=2)
    elif route.startswith("staged"):
        st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=2)
    return uh, st


def _setup(route, monkeypatch):
    from fedn_amd import layout, staging
    if "sliced" in route:
        monkeypatch.setattr(layout, "MULTIDEV_MIN_BYTES", 0)
    if route == "host_nozc":
        monkeypatch.setattr(staging, "ZERO_COPY_BYTES", 0)
    if route == "host_flush":                # batches flushed by add() (3 updates per launch)
        monkeypatch.setattr(staging, "BATCH", 3)
        monkeypatch.setattr(staging, "ZERO_COPY_BYTES", 0)


CASES = [("host", SMALL, 6, [2]), ("host_nozc", SMALL, 6, [3]), ("host_flush", SMALL, 8, [1, 5]),
         ("staged", SMALL, 6, [4]), ("staged_large", LARGE, 5, [2]), ("staged_sliced", SMALL, 6, [1]),
         ("staged_k70", SMALL, 70, [10, 66]), ("staged_k70_large", LARGE, 70, [3, 67]),
         ("host", SMALL, 3, [1, 2]), ("staged", SMALL, 4, [0])]


@pytest.mark.parametrize("route,shapes,K,bad", CASES, ids=[f"{c[0]}-K{c[2]}-bad{'_'.join(map(str, c[3]))}"
                                                           for c in CASES])
def test_fedavg_batched_failure_skips_only_the_failing_update(route, shapes, K, bad, monkeypatch):
    from fedn_amd.aggregators.fedavg import Aggregator
    _setup(route, monkeypatch)
    rng = np.random.default_rng(K * 31 + bad[0])
    base = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ups, ns = _clients(rng, shapes, K, base)
    Ns = np.cumsum(ns)
    uh, st = _handlers(route)
    try:
        agg = Aggregator(st or uh, devices=[DEV, DEV]) if "sliced" in route else Aggregator(st or uh, device=DEV)
        mus = [uh.submit(u, n, via=st) for u, n in zip(ups, ns)]
        hits = _poison(monkeypatch, {(float(ns[p]), float(Ns[p])) for p in bad if p > 0})
        model, data = agg.combine_models(helper=None)
    finally:
        if st is not None:
            st.close()
    skipped = [p for p in bad if p > 0]       # the first update is the model itself: it never folds

    def increment(m1, m2, n, N):              # the reference fold raising on a poisoned update
        if any(m2 is ups[p] for p in skipped):
            raise RuntimeError("fold failed")
        return ref.increment_average(m1, m2, n, N)

    want, nr = ref.fedavg_combine(list(zip(ups, ns)), increment)
    assert nr == data["nr_aggregated_models"] == K - len(skipped)
    assert_lists_identical(model, want, f"fedavg {route} K {K} skipping {skipped}")
    assert uh.model_updates.qsize() == 0
    kept = {mu.model_update_id for p, mu in enumerate(mus) if p in skipped}
    assert set(uh.store.models) == kept, "skipped updates stay in storage, folded ones are deleted"
    if skipped:
        assert hits, "the poisoned launch was never issued"


OPT_CASES = [("host", SMALL, 6, [2]), ("host_nozc", SMALL, 6, [0]), ("host_flush", SMALL, 8, [1, 6]),
             ("staged", SMALL, 6, [3]), ("staged_large", LARGE, 5, [4]), ("staged_sliced", SMALL, 6, [2]),
             ("staged_k70", SMALL, 70, [5, 65])]


@pytest.mark.parametrize("route,shapes,K,bad", OPT_CASES, ids=[f"{c[0]}-K{c[2]}-bad{'_'.join(map(str, c[3]))}"
                                                               for c in OPT_CASES])
def test_fedopt_batched_failure_skips_only_the_failing_update(route, shapes, K, bad, monkeypatch):
    """Round 2 of a 3-round adam session has poisoned updates: they are skipped (their examples
    counted), the server step runs on the others; m / v and round 3 continue exactly as the oracle."""
    from fedn_amd.aggregators.fedopt import Aggregator
    _setup(route, monkeypatch)
    rng = np.random.default_rng(K * 37 + bad[0])
    old = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    uh, st = _handlers(route)
    state = ref.FedOptState()
    poisoned = [np.zeros((13, 17, 19), np.float32)]   # subtract() raises in the oracle: a skipped update
    try:
        agg = Aggregator(st or uh, devices=[DEV, DEV]) if "sliced" in route else Aggregator(st or uh, device=DEV)
        for r in range(3):
            ups, ns = _clients(rng, shapes, K, old)
            Ns = np.cumsum(ns)
            gid = uh.put_global_model(old, f"g{r}")
            mus = [uh.submit(u, n, model_id=gid, via=st) for u, n in zip(ups, ns)]
            undo = None
            if r == 1:
                undo = monkeypatch.context()
                mp = undo.__enter__()
                _poison(mp, {(float(ns[p]), float(Ns[p])) for p in bad})
            try:
                model, data = agg.combine_models(helper=None)
            finally:
                if undo is not None:
                    undo.__exit__(None, None, None)
            feed = [(poisoned if (r == 1 and k in bad) else ups[k], ns[k]) for k in range(K)]
            want, nr = ref.fedopt_combine(state, feed, old)
            what = f"fedopt {route} round {r} K {K} skipping {bad if r == 1 else []}"
            assert data["nr_aggregated_models"] == nr == K - (len(bad) if r == 1 else 0), what
            assert_lists_identical(model, want, what)
            assert_lists_identical(agg.m, state.m, what + " m")
            assert_lists_identical(agg.v, state.v, what + " v")
            left = {mu.model_update_id for k, mu in enumerate(mus) if r == 1 and k in bad}
            assert {m for m in uh.store.models if not m.startswith("g")} == left, what + " storage"
            for k in sorted(left):
                uh.store.delete(k)
            old = model
    finally:
        if st is not None:
            st.close()


def test_fedopt_server_step_failure_after_batch_refold_returns_none(monkeypatch):
    """The fused launch fails, the refold of its updates succeeds, and the server step alone fails
    too: (None, data) with every update counted (fedopt.py:111-116); the state is round 1's."""
    from fedn_amd import _abi, ops
    from fedn_amd.aggregators.fedopt import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(77)
    old = [rng.standard_normal(s).astype(np.float32) for s in SMALL]
    uh = MemoryUpdateHandler()
    agg = Aggregator(uh, device=DEV)
    state = ref.FedOptState()
    ups, ns = _clients(rng, SMALL, 4, old)
    gid = uh.put_global_model(old, "g0")
    for u, n in zip(ups, ns):
        uh.submit(u, n, model_id=gid)
    model, _ = agg.combine_models(helper=None)
    want, _ = ref.fedopt_combine(state, list(zip(ups, ns)), old)
    assert_lists_identical(model, want, "round 1")
    for name in ("fedopt_step", "fedopt_step_raw", "fedopt_step_host"):
        real = getattr(ops, name)

        def wrapper(*a, _real=real, **kw):
            if kw.get("final"):
                raise _abi.FedAggError(_abi.FA_EHIP, "injected server-step failure")
            return _real(*a, **kw)

        monkeypatch.setattr(ops, name, wrapper)
    ups, ns = _clients(rng, SMALL, 4, want)
    gid = uh.put_global_model(want, "g1")
    for u, n in zip(ups, ns):
        uh.submit(u, n, model_id=gid)
    model, data = agg.combine_models(helper=None)
    assert model is None and data["nr_aggregated_models"] == 4
    assert_lists_identical(agg.m, state.m, "m kept")
    assert_lists_identical(agg.v, state.v, "v kept")


MIXED = [(300, 7), (5,)]                      # + an int64 counter per update: two dtype groups


def _mixed_updates(rng, K):
    base = [rng.standard_normal(s).astype(np.float32) for s in MIXED]
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] +
           [np.array([int(rng.integers(0, 1000))], dtype=np.int64)] for _ in range(K)]
    ns = [int(v) for v in rng.choice(np.arange(1, 5001), K, replace=False)]
    return ups, ns


@pytest.mark.parametrize("route", ["host_flush", "staged"])
def test_snapshot_that_cannot_be_taken_only_matters_on_failure(route, monkeypatch):
    """the all-or-nothing snapshot of a multi-launch fold is taken inside the fold's try,
    and an HBM-full clone (simulated: every snapshot reports staging.NO_SNAPSHOT) does not skip a
    valid update — the folds go ahead and the round is bit-exact; a launch that then fails part-way
    cannot be undone, so the round is lost loudly (combine_models raises) instead of returning a
    model with a half-applied update."""
    from fedn_amd import staging
    from fedn_amd.aggregators.fedavg import Aggregator
    _setup(route, monkeypatch)
    monkeypatch.setattr(staging, "BATCH", 3)   # u1-u3 fold as the init batch, u4-u5 continue it
    real = staging.FedAvgPipeline._snapshot
    taken = []

    def no_room(self, launches):
        snap = real(self, launches)
        if snap is None:
            return None
        taken.append(launches)
        return staging.NO_SNAPSHOT
    monkeypatch.setattr(staging.FedAvgPipeline, "_snapshot", no_room)
    for poisoned in (False, True):
        rng = np.random.default_rng(77)
        ups, ns = _mixed_updates(rng, 6)
        uh, st = _handlers(route)
        try:
            agg = Aggregator(st or uh, device=DEV)
            for u, n in zip(ups, ns):
                uh.submit(u, n, via=st)
            if not poisoned:
                model, data = agg.combine_models(helper=None)
                want, nr = ref.fedavg_combine(list(zip(ups, ns)))
                assert data["nr_aggregated_models"] == nr == 6
                assert_lists_identical(model, want, f"{route} without a snapshot")
                assert taken, "no multi-launch fold ran: the case does not exercise the snapshot"
            else:
                # the update's int64-group launch fails AFTER its float32-group launch ran: that
                # half-applied fold could only be undone from the snapshot it could not take
                from fedn_amd import _abi, ops
                Ns = np.cumsum(ns)
                bad = (float(ns[4]), float(Ns[4]))
                real_fold = ops.fedavg_fold_ptrs

                def fold(acc, ptrs, upd_dt, n, N, *a, **kw):
                    if upd_dt == torch.int64 and any((float(x), float(y)) == bad for x, y in zip(n, N)):
                        raise _abi.FedAggError(_abi.FA_EHIP, "injected failure of the second launch")
                    return real_fold(acc, ptrs, upd_dt, n, N, *a, **kw)
                monkeypatch.setattr(ops, "fedavg_fold_ptrs", fold)
                with pytest.raises(RuntimeError, match="could not be copied aside"):
                    agg.combine_models(helper=None)
        finally:
            if st is not None:
                st.close()
