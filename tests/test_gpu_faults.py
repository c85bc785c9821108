"""the kernel path never kills the round. A libfedagg call that fails (nonzero
status -> FedAggError) is handled by the plug-ins exactly as FEDn handles an update whose fold
raises: the update is logged and skipped with its examples still counted (fedavg.py:75-78,
fedopt.py:103-106) — for batched launches after refolding the batch one update at a time
(tests/test_gpu_batch_faults.py covers every batching route) — and a server step that raises gives
``(None, data)`` (fedopt.py:111-116).
Failures are injected at the C-ABI wrapper (fedn_amd.ops) before anything is enqueued, which
is where a real status code surfaces; every result is checked against the oracle."""
import numpy as np
import pytest
import torch

from golden_io import assert_lists_identical
from oracle import numpy_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _failing(monkeypatch, name, fail_on):
    """Make fedn_amd.ops.<name> raise FedAggError on the calls ``fail_on`` selects."""
    from fedn_amd import _abi, ops
    real = getattr(ops, name)
    calls = []

    def wrapper(*a, **kw):
        calls.append(kw)
        if fail_on(len(calls), kw):
            raise _abi.FedAggError(_abi.FA_EHIP, f"{name}: injected failure (call {len(calls)})")
        return real(*a, **kw)

    monkeypatch.setattr(ops, name, wrapper)
    return calls


def _models(rng, K, shapes):
    base = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    return base, ups, ns


def _poison_update(monkeypatch, n, N):
    """Every fold launch whose client table holds the update (n, N) raises FedAggError: an update
    whose fold fails however it is launched (alone, or in a multi-client batch)."""
    import inspect

    from fedn_amd import _abi, ops
    for name in ("fedavg_fold_ptrs", "fedavg_fold_raw", "fedavg_fold_host"):
        real = getattr(ops, name)
        sig = inspect.signature(real)

        def wrapper(*a, _real=real, _sig=sig, _name=name, **kw):
            b = _sig.bind(*a, **kw)
            if any(float(x) == n and float(y) == N for x, y in zip(b.arguments["n"], b.arguments["N"])):
                raise _abi.FedAggError(_abi.FA_EHIP, f"{_name}: injected failure")
            return _real(*a, **kw)

        monkeypatch.setattr(ops, name, wrapper)


@pytest.mark.parametrize("shapes", [[(1000, 1100), (999,)], [(30, 7), (5,)]], ids=["large", "small_batched"])
def test_fedavg_fold_failure_skips_the_update(monkeypatch, shapes):
    """Update 2's fold fails. Large host updates fold on arrival (one launch per update): the update
    is skipped right there. Small ones are batched (one zero-copy launch for the round, or one launch
    per <= 64 updates): the batch's launch fails, its updates are refolded one at a time from their
    staged copies, and only update 2 — whose own fold fails again — is skipped (fedavg.py:75-78).
    Either way: logged, uncounted, its examples still in every later running total, the model the
    oracle's with update 2's fold raising."""
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(51)
    _, ups, ns = _models(rng, 5, shapes)
    uh = MemoryUpdateHandler()
    agg = Aggregator(uh, device=DEV)
    for u, n in zip(ups, ns):
        uh.submit(u, n)
    _poison_update(monkeypatch, float(ns[2]), float(sum(ns[:3])))
    model, data = agg.combine_models(helper=None)

    def increment(m1, m2, n, N):                      # the reference fold raising on update 2
        if m2 is ups[2]:
            raise RuntimeError("fold failed")
        return ref.increment_average(m1, m2, n, N)

    want, nr = ref.fedavg_combine(list(zip(ups, ns)), increment)
    assert nr == data["nr_aggregated_models"] == 4
    assert_lists_identical(model, want, "fedavg with a failed fold")
    assert uh.model_updates.qsize() == 0


@pytest.mark.parametrize("shapes,at_chunk", [([(700, 900), (333,)], 1), ([(1500, 1500), (333,)], 2)],
                         ids=["first_launch", "second_chunk"])
def test_fedopt_server_step_failure_returns_none_and_keeps_state(monkeypatch, shapes, at_chunk):
    """The fused server step fails in round 2 — at its first launch, or at the second of the chunked
    launches after the first chunk's m / v were written: ``(None, data)``, m / v stay round 1's (the
    step writes new buffers), and round 3 continues from them exactly as if round 2 had not run."""
    from fedn_amd.aggregators.fedopt import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(52)
    uh = MemoryUpdateHandler()
    agg = Aggregator(uh, device=DEV)
    st = ref.FedOptState()
    old = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    fail = [False]
    finals = [0]

    def fail_on(i, kw):
        # the server step fails from its at_chunk-th launch on: the fused launch fails, the batch's
        # updates refold into pg one at a time (no final launch), and the server step alone fails again
        if not kw.get("final") or not fail[0]:
            return False
        finals[0] += 1
        return finals[0] >= at_chunk

    calls = _failing(monkeypatch, "fedopt_step", fail_on)
    for r in range(3):
        fail[0] = r == 1
        finals[0] = 0
        ups = [[(o + 0.01 * rng.standard_normal(o.shape)).astype(o.dtype) for o in old] for _ in range(3)]
        ns = [int(v) for v in rng.integers(1, 5001, 3)]
        gid = uh.put_global_model(old, f"global-{r}")
        for u, n in zip(ups, ns):
            uh.submit(u, n, model_id=gid)
        model, data = agg.combine_models(helper=None)
        assert data["nr_aggregated_models"] == 3
        if r == 1:
            assert model is None
            assert_lists_identical(agg.m, st.m, "m kept")
            assert_lists_identical(agg.v, st.v, "v kept")
            continue
        want, _ = ref.fedopt_combine(st, list(zip(ups, ns)), old)
        assert_lists_identical(model, want, f"round {r}")
        assert_lists_identical(agg.m, st.m, f"m r{r}")
        assert_lists_identical(agg.v, st.v, f"v r{r}")
        old = want
    assert any(kw.get("final") for kw in calls)
    torch.cuda.synchronize()


def test_fedopt_zero_copy_step_failure_keeps_state(monkeypatch):
    """A small round folded zero-copy (the one-call step, smallround.py, then the pipeline's
    fedopt_step_raw launch per group: staging.ZERO_COPY_BYTES) that fails in round 2: ``(None, data)``,
    m / v stay round 1's, round 3 continues from them."""
    from fedn_amd import staging
    from fedn_amd.aggregators.fedopt import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    assert staging.ZERO_COPY_BYTES > 0
    rng = np.random.default_rng(53)
    shapes = [(64, 784), (64,), (10, 64), (10,)]
    uh = MemoryUpdateHandler()
    agg = Aggregator(uh, device=DEV)
    st = ref.FedOptState()
    old = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    fail = [False]
    # the server step fails (the zero-copy FIRST + FINAL launch, then the K = 0 step after the updates
    # refolded into pg one at a time); the pseudo-gradient folds themselves succeed
    calls = _failing(monkeypatch, "fedopt_step_raw", lambda i, kw: fail[0] and kw.get("final"))
    _failing(monkeypatch, "fedopt_step", lambda i, kw: fail[0] and kw.get("final"))
    # since round 6 a small round's first try is the one-call step (smallround.py, fedopt_step_host)
    host_calls = _failing(monkeypatch, "fedopt_step_host", lambda i, kw: fail[0] and kw.get("final"))
    for r in range(3):
        fail[0] = r == 1
        ups = [[(o + 0.01 * rng.standard_normal(o.shape)).astype(o.dtype) for o in old] for _ in range(3)]
        ns = [int(v) for v in rng.integers(1, 5001, 3)]
        gid = uh.put_global_model(old, f"global-{r}")
        for u, n in zip(ups, ns):
            uh.submit(u, n, model_id=gid)
        model, data = agg.combine_models(helper=None)
        assert data["nr_aggregated_models"] == 3
        if r == 1:
            assert model is None
            assert_lists_identical(agg.m, st.m, "m kept")
            assert_lists_identical(agg.v, st.v, "v kept")
            continue
        want, _ = ref.fedopt_combine(st, list(zip(ups, ns)), old)
        assert_lists_identical(model, want, f"round {r}")
        assert_lists_identical(agg.m, st.m, f"m r{r}")
        assert_lists_identical(agg.v, st.v, f"v r{r}")
        old = want
    assert sum(1 for kw in host_calls if kw.get("final")) == 3    # every round took the one-call step first
    assert sum(1 for kw in calls if kw.get("final")) == 1         # round 2 then the general zero-copy step
    torch.cuda.synchronize()
