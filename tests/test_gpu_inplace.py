"""Multi-device rounds on host updates DMA the large tensors that lie in page-locked memory already
(what fedn_amd.helper.load decodes large npz members into) straight from the caller's arrays instead
of packing every byte into a pinned slot first (multidev.INPLACE_MIN_BYTES; VERDICT r3 item 5;
tools/bench_hostres.py). Pageable arrays are packed unless multidev.INPLACE_REGISTER page-locks them
in place (a caller that reuses its buffers); those registrations are undone once the round is over.
Bit-exact against the oracle in every mode."""
import io

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


def _clients(rng, base, K, pinned=False):
    from fedn_amd.helper import pinned_empty
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
    if pinned:
        for u in ups:
            for i, a in enumerate(u):
                p = pinned_empty(a.shape, a.dtype)
                if p is not None:
                    p[...] = a
                    u[i] = p
    return ups, [int(v) for v in rng.integers(1, 5001, K)]


@pytest.mark.parametrize("env", [{"FEDN_AMD_DEVICES": "cuda:0,cuda:0"}, {"FEDN_AMD_DECODE_PINNED": "1"}],
                         ids=["multi_device_combiner", "forced"])
def test_helper_load_decodes_large_members_pinned(env, monkeypatch):
    """fedn_amd.helper.load for a multi-GPU combiner: members of 8 MiB+ land in page-locked memory
    (a device address exists for them), smaller ones in ordinary arrays; values identical to the
    archive's."""
    from fedn_amd import ops
    from fedn_amd.helper import Helper
    monkeypatch.delenv("FEDN_AMD_DECODE_PINNED", raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(7)
    ws = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    h = Helper()
    b = io.BytesIO()
    h.save(ws, b)
    out = h.load(io.BytesIO(b.getvalue()))
    assert_lists_identical(out, ws, "pinned decode")
    for a in out:
        if a.nbytes >= (8 << 20):
            ops.host_device_ptr(a.ctypes.data, torch.device(DEV))
        else:
            with pytest.raises(ops.FedAggError):
                ops.host_device_ptr(a.ctypes.data, torch.device(DEV))


def test_helper_load_one_device_keeps_plain_arrays(monkeypatch):
    """One device packs every update anyway: no pinned decode unless asked for."""
    from fedn_amd import ops
    from fedn_amd.helper import Helper
    monkeypatch.delenv("FEDN_AMD_DEVICES", raising=False)
    monkeypatch.delenv("FEDN_AMD_DECODE_PINNED", raising=False)
    ws = [np.arange(3_000_000, dtype=np.float32)]
    b = io.BytesIO()
    Helper().save(ws, b)
    out = Helper().load(io.BytesIO(b.getvalue()))
    assert_lists_identical(out, ws, "plain decode")
    with pytest.raises(ops.FedAggError):
        ops.host_device_ptr(out[0].ctypes.data, torch.device(DEV))


@pytest.mark.parametrize("ndev", [2, 3])
@pytest.mark.parametrize("mode", ["pinned", "pageable"])
def test_sharded_fedavg_host_updates_pinned(ndev, mode):
    """pinned: every large tensor is DMA'd in place, nothing registered here; pageable (default
    policy): every byte is packed."""
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(80 + ndev)
    base = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    ups, ns = _clients(rng, base, 5, pinned=mode == "pinned")
    uh = MemoryUpdateHandler()
    agg = Aggregator(uh, devices=[DEV] * ndev)
    for u, n in zip(ups, ns):
        uh.submit(u, n)
    model, data = agg.combine_models(helper=None)
    want, nr = ref.fedavg_combine(list(zip(ups, ns)))
    assert data["nr_aggregated_models"] == nr == 5
    assert_lists_identical(model, want, f"{mode} H2D over {ndev} slices")
    big = sum(int(np.prod(s)) * 4 for s in SHAPES if int(np.prod(s)) * 4 >= (8 << 20))
    assert data["bytes_h2d_in_place"] == (5 * big if mode == "pinned" else 0)
    torch.cuda.synchronize()


@pytest.mark.parametrize("ndev", [2, 3])
@pytest.mark.parametrize("share", [False, True], ids=["distinct", "shared_arrays"])
def test_sharded_fedavg_host_updates_in_place(ndev, share, monkeypatch):
    """INPLACE_REGISTER: pageable arrays page-locked in place. ``shared_arrays``: two clients hand
    over the very same array objects — registered once, DMA'd for both; the model is the same."""
    from fedn_amd import multidev, ops
    monkeypatch.setattr(multidev, "INPLACE_REGISTER", True)
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


@pytest.mark.parametrize("pinned", [False, True], ids=["registered", "pinned"])
def test_sharded_fedopt_host_updates_in_place(pinned, monkeypatch):
    from fedn_amd import multidev
    from fedn_amd.aggregators.fedopt import Aggregator
    monkeypatch.setattr(multidev, "INPLACE_REGISTER", not pinned)
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(93)
    old = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    uh = MemoryUpdateHandler()
    agg = Aggregator(uh, devices=[DEV, DEV])
    st = ref.FedOptState()
    for r in range(2):
        ups, ns = _clients(rng, old, 3, pinned=pinned)
        gid = uh.put_global_model(old, f"g{r}")
        for u, n in zip(ups, ns):
            uh.submit(u, n, model_id=gid)
        model, data = agg.combine_models(helper=None)
        want, _ = ref.fedopt_combine(st, list(zip(ups, ns)), old)
        assert data["nr_aggregated_models"] == 3
        assert data["bytes_h2d_in_place"] > 0
        assert_lists_identical(model, want, f"round {r}")
        assert_lists_identical(agg.m, st.m, f"m {r}")
        assert_lists_identical(agg.v, st.v, f"v {r}")
        old = model


def test_fedn_round_on_npz_updates_decodes_pinned_and_dmas_in_place(monkeypatch):
    """The whole FEDn-shaped path on several devices: npz bytes in storage (ModelService.Upload),
    FEDn's load_model_update through the plug-in's helper (members of 8 MiB+ decoded into pinned
    blocks, FEDN_AMD_DEVICES naming two entries), the multi-device FedAvg pipeline DMAing those
    tensors in place — bit-exact against the oracle on the decoded arrays."""
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.helper import Helper
    from fedn_amd.updatehandler import MemoryUpdateHandler
    monkeypatch.setenv("FEDN_AMD_DEVICES", f"{DEV},{DEV}")
    monkeypatch.delenv("FEDN_AMD_DECODE_PINNED", raising=False)
    rng = np.random.default_rng(97)
    base = [rng.standard_normal(s).astype(np.float32) for s in SHAPES]
    ups, ns = _clients(rng, base, 4)
    h = Helper()
    uh = MemoryUpdateHandler()
    for u, n in zip(ups, ns):
        b = io.BytesIO()
        h.save(u, b)
        uh.submit_bytes(b.getvalue(), n)
    agg = Aggregator(uh)
    model, data = agg.combine_models(helper=h)
    want, nr = ref.fedavg_combine(list(zip(ups, ns)))
    assert data["nr_aggregated_models"] == nr == 4
    assert_lists_identical(model, want, "npz -> pinned decode -> in-place H2D")
    big = sum(int(np.prod(s)) * 4 for s in SHAPES if int(np.prod(s)) * 4 >= (8 << 20))
    assert data["bytes_h2d_in_place"] >= 3 * big        # the first update may be staged differently
    torch.cuda.synchronize()
