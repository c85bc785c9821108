"""Multi-device rounds on host updates DMA the large tensors straight from the caller's arrays,
page-locked in place (multidev.INPLACE_MIN_BYTES), instead of packing every byte into a pinned slot
first (tools/pack_probe.py --inplace). Bit-exact against the oracle; the
registrations are undone once the round is over (the same arrays can be page-locked again)."""
import numpy as np
import pytest
import torch

from golden_io import assert_lists_identical
from oracle import numpy_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
SHAPES = [(3_000_000,), (64, 33), (5,), (2_100_000,)]     # two tensors over 8 MiB, two small ones


@pytest.fixture(autouse=True)
def _slice(monkeypatch):
    from fedn_amd import layout
    monkeypatch.setattr(layout, "MULTIDEV_MIN_BYTES", 0)


def _clients(rng, base, K):
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
    return ups, [int(v) for v in rng.integers(1, 5001, K)]


@pytest.mark.parametrize("ndev", [2, 3])
@pytest.mark.parametrize("share", [False, True], ids=["distinct", "shared_arrays"])
def test_sharded_fedavg_host_updates_in_place(ndev, share):
    """``shared_arrays``: two clients hand over the very same array objects — the second page-lock of
    the same pages fails and that update is packed instead; the model is the same."""
    from fedn_amd import ops
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(90 + ndev)
    base = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    ups, ns = _clients(rng, base, 5)
    if share:
        ups[3] = ups[2]
    uh = MemoryUpdateHandler()
    agg = Aggregator(uh, devices=[DEV] * ndev)
    for u, n in zip(ups, ns):
        uh.submit(u, n)
    model, data = agg.combine_models(helper=None)
    want, nr = ref.fedavg_combine(list(zip(ups, ns)))
    assert data["nr_aggregated_models"] == nr == 5
    assert_lists_identical(model, want, f"in-place H2D over {ndev} slices")
    big = sum(int(np.prod(s)) * 4 for s in SHAPES if int(np.prod(s)) * 4 >= (8 << 20))
    assert data["bytes_h2d_in_place"] >= (4 if share else 5) * big
    assert data["bytes_h2d_packed"] > 0
    for u in ups:                                   # every registration was undone: page-lock again
        for a in u:
            if a.nbytes >= (8 << 20):
                ops.host_register_ptr(a.ctypes.data, a.nbytes)
                ops.host_unregister_ptr(a.ctypes.data)
    torch.cuda.synchronize()


def test_sharded_fedopt_host_updates_in_place():
    from fedn_amd.aggregators.fedopt import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(93)
    old = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    uh = MemoryUpdateHandler()
    agg = Aggregator(uh, devices=[DEV, DEV])
    st = ref.FedOptState()
    for r in range(2):
        ups, ns = _clients(rng, old, 3)
        gid = uh.put_global_model(old, f"g{r}")
        for u, n in zip(ups, ns):
            uh.submit(u, n, model_id=gid)
        model, data = agg.combine_models(helper=None)
        want, _ = ref.fedopt_combine(st, list(zip(ups, ns)), old)
        assert data["nr_aggregated_models"] == 3
        assert_lists_identical(model, want, f"round {r}")
        assert_lists_identical(agg.m, st.m, f"m {r}")
        assert_lists_identical(agg.v, st.v, f"v {r}")
        old = model
