"""HBM admission control of the staging ingest (budget.py, ingest.StagingUpdateHandler): with a
budget too small for the round, the updates beyond it stay host-side and the aggregator folds them
from the host at their place in the FIFO — bit-exact against the oracle, every client counted
(fedavg.py:47-68, fedopt.py:74-98 fold any number of host updates one at a time)."""
import io

import numpy as np
import pytest
import torch

from fedn_amd.aggregators import get_aggregator
from fedn_amd.budget import HbmBudget, parse_bytes
from fedn_amd.helper import Helper
from fedn_amd.ingest import StagingUpdateHandler
from fedn_amd.layout import Layout
from fedn_amd.updatehandler import MemoryUpdateHandler
from golden_io import assert_lists_identical
from oracle import numpy_ref as ref

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
SHAPES = [(300, 257), (257,), (33, 7)]


def _npz(arrays):
    buf = io.BytesIO()
    np.savez_compressed(buf, **{str(i): a for i, a in enumerate(arrays)})
    return buf.getvalue()


def _round(rng, uh, st, base, K, model_id="global", as_bytes=False):
    ups = []
    for _ in range(K):
        arrays = [(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base]
        n = int(rng.integers(1, 5001))
        if as_bytes:
            uh.submit_bytes(_npz(arrays), n, model_id=model_id, via=st)
        else:
            uh.submit(arrays, n, model_id=model_id, via=st)
        ups.append((arrays, n))
    return ups


@pytest.mark.parametrize("as_bytes", [False, True])
def test_budget_fedavg_k70_two_rounds(as_bytes):
    rng = np.random.default_rng(31)
    base = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    nbytes = Layout.of(base).nbytes
    budget = HbmBudget(limit=3 * nbytes)                 # 3 of the 70 updates fit
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=Helper() if as_bytes else None, device=DEV, workers=3, hbm_budget=budget)
    agg = get_aggregator("fedavg", st)
    for r in range(2):
        ups = _round(rng, uh, st, base, 70, as_bytes=as_bytes)
        model, data = agg.combine_models(helper=Helper() if as_bytes else None)
        want, nr = ref.fedavg_combine(ups)
        assert data["nr_aggregated_models"] == nr == 70
        assert_lists_identical(model, want, f"round {r}")
    assert st.host_side >= 2 * 60                        # most updates stayed host-side
    import gc
    gc.collect()
    assert budget.used(DEV) == 0                         # every staged update returned its bytes
    st.close()


@pytest.mark.parametrize("opt", ["adam", "yogi"])
def test_budget_fedopt_k70_two_rounds(opt):
    rng = np.random.default_rng(32)
    base = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    budget = HbmBudget(limit=5 * Layout.of(base).nbytes)
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=3, hbm_budget=budget)
    agg = get_aggregator("fedopt", st)
    state = ref.FedOptState()
    old = base
    params = {"serveropt": opt}
    for r in range(2):
        gid = uh.put_global_model(old, f"g{r}")
        ups = _round(rng, uh, st, old, 70, model_id=gid)
        model, data = agg.combine_models(helper=None, parameters=params)
        want, nr = ref.fedopt_combine(state, ups, old, params)
        assert data["nr_aggregated_models"] == nr == 70
        assert_lists_identical(model, want, f"{opt} round {r}")
        assert_lists_identical(agg.m, state.m, f"{opt} round {r} m")
        old = want
    assert st.host_side >= 2 * 60
    st.close()


def test_budget_zero_stages_nothing():
    """FEDN_AMD_HBM_BUDGET=0: every update is folded from the host (FEDn's own loop on the GPU)."""
    rng = np.random.default_rng(33)
    base = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, device=DEV, workers=2, hbm_budget=HbmBudget(limit=parse_bytes("0")))
    ups = _round(rng, uh, st, base, 9)
    model, data = get_aggregator("fedavg", st).combine_models(helper=None)
    want, _ = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == 9 and st.host_side == 9
    assert_lists_identical(model, want, "budget 0")
    st.close()


def test_staging_oom_falls_back_to_host(monkeypatch):
    """An HBM allocation that fails inside a staging worker (torch OutOfMemoryError) leaves that
    update host-side instead of turning it into a skipped client."""
    from fedn_amd import ingest
    rng = np.random.default_rng(34)
    base = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    real = ingest.stage_arrays
    calls = [0]

    def flaky(arrays, device, stream):
        calls[0] += 1
        if calls[0] % 3 == 0:
            raise torch.cuda.OutOfMemoryError("HIP out of memory (injected)")
        return real(arrays, device, stream)

    monkeypatch.setattr(ingest, "stage_arrays", flaky)
    uh = MemoryUpdateHandler()
    budget = HbmBudget(limit=1 << 40)
    st = StagingUpdateHandler(uh, device=DEV, workers=1, native_decode=False, hbm_budget=budget)
    ups = _round(rng, uh, st, base, 12)
    model, data = get_aggregator("fedavg", st).combine_models(helper=None)
    want, _ = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == 12 and st.host_side == 4
    assert_lists_identical(model, want, "oom fallback")
    st.close()


def test_budget_streaming_upload_k20():
    """Decode-while-uploading under a budget of ~2.5 updates: uploads the budget cannot hold are not
    decoded into HBM (DeviceSink refuses), stagings beyond it stay host-side; 20 updates, all folded,
    bit-exact; the budget is empty again once the round's objects are gone."""
    import gc

    from fedn_amd.updatehandler import MemoryModelService, upload_requests
    from fedn_amd.upload import StreamingUpload
    rng = np.random.default_rng(35)
    base = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    budget = HbmBudget(limit=int(2.5 * Layout.of(base).nbytes))
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=Helper(), device=DEV, workers=2, hbm_budget=budget)
    svc = StreamingUpload(MemoryModelService(uh.store), st, workers=2, slot=65536, ring=2)
    ups = []
    for k in range(20):
        arrays = [(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base]
        n = int(rng.integers(1, 5001))
        svc.Upload(upload_requests(_npz(arrays), f"B{k}", chunk=40_000), None)
        uh.submit_uploaded(f"B{k}", n, via=st)
        ups.append((arrays, n))
    model, data = get_aggregator("fedavg", st).combine_models(helper=Helper())
    svc.close()
    want, nr = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == nr == 20
    assert_lists_identical(model, want, "upload under budget")
    assert st.host_side > 0 and budget.refused > 0
    del model
    st.close()
    gc.collect()
    assert budget.used(DEV) == 0


def test_decoded_upload_reservation_moves_to_its_staged_copy():
    """an update decoded into HBM while it uploaded (DeviceSink, which reserves its payload
    bytes) hands that reservation to its staged copy instead of both counting against the budget. Under
    a budget of 1.5 updates every update is staged (none left host-side), one after the other, and the
    budget holds exactly the staged bytes while they live, nothing once the round is gone."""
    import gc

    from fedn_amd.updatehandler import MemoryModelService, upload_requests
    from fedn_amd.upload import StreamingUpload
    rng = np.random.default_rng(36)
    base = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    lay = Layout.of(base)
    budget = HbmBudget(limit=int(1.5 * lay.nbytes))
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=Helper(), device=DEV, workers=1, hbm_budget=budget)
    svc = StreamingUpload(MemoryModelService(uh.store), st, workers=1, slot=65536, ring=2)
    ups = []
    for k in range(3):
        arrays = [(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base]
        n = int(rng.integers(1, 5001))
        svc.Upload(upload_requests(_npz(arrays), f"D{k}", chunk=40_000), None)
        mu = uh.submit_uploaded(f"D{k}", n, via=st)
        ups.append((arrays, n))
        staged, _ = st.load_model_update(mu, Helper())          # waits for its staging
        assert hasattr(staged, "layout"), "left host-side: the decode's reservation was counted twice"
        assert budget.used(DEV) == lay.nbytes
        uh.model_updates.get()                                   # consumed here, not by an aggregator
        del staged
        gc.collect()
        assert budget.used(DEV) == 0
    svc.close()
    assert st.host_side == 0 and budget.refused == 0
    st.close()
