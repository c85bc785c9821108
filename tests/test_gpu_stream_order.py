"""Fresh HBM and torch's stream order (DESIGN round-6 row 3b). torch's caching allocator hands a freed
block to the next allocation in the order of the stream it was allocated on: work the block's previous
owner queued there may still run after the new owner receives it. A buffer written first by ANOTHER
stream (a copy stream's H2D into a new staging slot, a private stream's kernel into new m / v) must
therefore wait for the allocating stream first, or that queued work lands on top of it.

Each test queues a long run of folds on the current stream, then fills blocks of exactly the size the
path will allocate next behind them, frees those blocks, and runs the path: its results must be the
oracle's, not the fills' zeros."""
import numpy as np
import pytest
import torch

from oracle import numpy_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fedn_amd import _abi
    _abi.load()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()             # no other free block of the sizes below in the pool
    yield
    torch.cuda.synchronize()


def _busy_then_zero_fills(nbytes, count=16, folds=200):
    """Queue ~tens of ms of folds on the current stream, then ``count`` blocks of ``nbytes`` (an int or
    a list of sizes, ``count`` of each) zero-filled behind them, and free the blocks (their fills still
    queued)."""
    from fedn_amd import ops
    P = 50_000_000
    ups = [torch.ones(P, device=DEV) for _ in range(8)]
    agg = torch.empty(P, device=DEV)
    for _ in range(folds):
        ops.fedavg_fold(agg, ups, [1] * 8, list(range(1, 9)), init=True)
    sizes = nbytes if isinstance(nbytes, (list, tuple)) else [nbytes]
    blocks = [torch.empty(nb, dtype=torch.uint8, device=DEV) for nb in sizes for _ in range(count)]
    for b in blocks:
        b.zero_()
    del blocks
    return ups, agg                      # kept until the test ends: their folds are still queued too


def _same(got, want, what):
    assert len(got) == len(want), what
    for i, (g, w) in enumerate(zip(got, want)):
        assert g.dtype == w.dtype and g.shape == w.shape, f"{what}[{i}]"
        assert np.array_equal(g.view(np.uint8), w.view(np.uint8)), f"{what}[{i}] differs"


def test_fedopt_one_call_step_after_queued_work_on_its_buffers():
    """The FedOpt one-call step's new m / v (fp32-state mode: P float32 each) come from blocks whose
    zero-fills are still queued on the current stream: the step must run after them."""
    from fedn_amd.aggregators import fedopt_f32state
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(3)
    shapes = [(40, 30), (30,), (7,)]
    P = sum(int(np.prod(s)) for s in shapes)
    old = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ups = [([(w + 0.01 * rng.standard_normal(w.shape)).astype(np.float32) for w in old], int(n))
           for n in rng.integers(1, 5001, 3)]
    uh = MemoryUpdateHandler()
    agg = fedopt_f32state.Aggregator(uh, device=DEV)
    gid = uh.put_global_model(old, "g0")
    for a, n in ups:
        uh.submit(a, n, model_id=gid)
    keep = _busy_then_zero_fills(P * 4)
    model, data = agg.combine_models(helper=None, parameters={"serveropt": "adam", "learning_rate": 1e-2})
    m, v = agg.m, agg.v
    st = ref.FedOptState()
    want, nr = ref.fedopt_combine_f32state(st, ups, old, {"serveropt": "adam", "learning_rate": 1e-2})
    assert data["nr_aggregated_models"] == nr == 3
    _same(model, want, "model")
    _same(m, st.m, "m")
    _same(v, st.v, "v")
    del keep


def test_staging_slot_first_h2d_after_queued_work_on_its_block():
    """The general FedAvg pipeline's first staging slots (allocated on the compute stream, written by the
    copy stream's H2D) come from blocks whose zero-fills are still queued on the compute stream."""
    from fedn_amd import staging
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.layout import Layout
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(5)
    shapes = [(1000, 2000), (2000,)]
    base = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ups = [([(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base], int(n))
           for n in rng.integers(1, 5001, 4)]
    nbytes = Layout.of(ups[0][0]).nbytes
    assert nbytes > staging.SMALL_UPDATE_BYTES and 2 * nbytes > staging.ZERO_COPY_BYTES   # slots, not arenas
    uh = MemoryUpdateHandler()
    agg = get_aggregator("fedavg", uh)
    for a, n in ups:
        uh.submit(a, n)
    keep = _busy_then_zero_fills(nbytes, count=8)
    model, data = agg.combine_models(helper=None)
    want, nr = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == nr == 4
    _same(model, want, "model")
    del keep


def test_multidevice_slots_and_global_model_after_queued_work():
    """The same for the pipelines sliced over several devices (multidev.py, two slices on this GPU):
    FedAvg's per-device slots, then FedOpt's per-device global-model buffers."""
    from fedn_amd.aggregators import fedavg, fedopt
    from fedn_amd.layout import Layout
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(7)
    shapes = [(1000, 2000), (2000,)]
    base = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ups = [([(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base], int(n))
           for n in rng.integers(1, 5001, 4)]
    bounds, _, dev_bytes = Layout.of(ups[0][0]).shard_geometry(2)
    old_bytes = sorted({(hi - lo) * 4 for lo, hi in bounds[np.dtype(np.float32)]})   # FedOpt's float32 global model
    uh = MemoryUpdateHandler()
    agg = fedavg.Aggregator(uh, devices=[DEV, DEV])
    for a, n in ups:
        uh.submit(a, n)
    keep = _busy_then_zero_fills(sorted(set(dev_bytes)), count=8)
    model, data = agg.combine_models(helper=None)
    want, nr = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == nr == 4
    _same(model, want, "fedavg model")
    del keep
    uh = MemoryUpdateHandler()
    agg = fedopt.Aggregator(uh, devices=[DEV, DEV])
    gid = uh.put_global_model(base, "g0")
    for a, n in ups:
        uh.submit(a, n, model_id=gid)
    keep = _busy_then_zero_fills(old_bytes + sorted(set(dev_bytes)), count=8)
    model, data = agg.combine_models(helper=None)
    st = ref.FedOptState()
    want, nr = ref.fedopt_combine(st, ups, base)
    assert data["nr_aggregated_models"] == nr == 4
    _same(model, want, "fedopt model")
    del keep


def test_wave_slots_first_h2d_after_queued_work():
    """configs[4]'s wave slots (allocated on the compute stream, first written by the copy stream)."""
    from fedn_amd.waves import WaveFedOpt
    P, K = 1_000_003, 12
    g = torch.Generator().manual_seed(9)
    base = torch.randn(P, generator=g)
    host = [(base + 0.01 * torch.randn(P, generator=g)).to(torch.bfloat16).pin_memory() for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(9).integers(1, 5001, K)]
    wf = WaveFedOpt([DEV], P, wave=4)
    old = wf.slices(base)
    keep = _busy_then_zero_fills(P * 2, count=12)
    outs = wf.round(host, ns, old, {"serveropt": "yogi"})
    got = wf.gather(outs).numpy()
    want, _ = ref.fedopt_combine(ref.FedOptState(), [([h.float().numpy()], n) for h, n in zip(host, ns)],
                                 [base.numpy()], {"serveropt": "yogi"})
    _same([got], want, "waves")
    del keep
