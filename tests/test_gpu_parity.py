"""GPU parity: libfedagg on an MI355X vs the CPU oracle (itself pinned to the reference).

Bar: bit-exact values AND dtypes (NaN payloads excepted) — the kernels replay numpy's
op order with IEEE rounding (SURVEY.md §0 parity findings 1-3).
"""
import numpy as np
import pytest
import torch

from golden_io import assert_lists_identical, case_names, load_case
from oracle import numpy_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
# clients that differ from the first in dtype / broadcastable shape (numpy promotion, mixed.py)
MIXED_FEDAVG = [n for n in case_names("fedavg") if "_mix_" in n or "_bcast_" in n or "fewer_tensors" in n]
MIXED_FEDOPT = [n for n in case_names("fedopt") if "_mix_" in n or "_bcast_" in n or "layout_change" in n
                or "f64_clients" in n]
_NARROW_KEYS = ("int8", "u8_", "unsigned", "narrow", "bool")
NARROW_FEDAVG = [n for n in case_names("fedavg") if any(k in n for k in _NARROW_KEYS)]
NARROW_FEDOPT = [n for n in case_names("fedopt") if any(k in n for k in _NARROW_KEYS)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fedn_amd import _abi
    _abi.load()


@pytest.fixture(autouse=True)
def _slice_every_model(monkeypatch):
    """The multi-device tests use small models: slice them over the devices anyway (the size rule
    that keeps small models on one GPU, layout.spread, has its own test)."""
    from fedn_amd import layout
    monkeypatch.setattr(layout, "MULTIDEV_MIN_BYTES", 0)


def _plugin(name):
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    uh = MemoryUpdateHandler()
    return uh, get_aggregator(name, uh)


# ------------------------------------------------------------------------- golden, plug-in level
@pytest.mark.parametrize("name", case_names("fedavg"))
def test_fedavg_plugin_golden(name):
    rd = load_case(name)["rounds"][0]
    uh, agg = _plugin("fedavg")
    for arrays, n in rd["updates"]:
        uh.submit(arrays, n)
    model, data = agg.combine_models(helper=None, delete_models=True, parameters=None)
    assert data["nr_aggregated_models"] == rd["nr"]
    assert uh.model_updates.qsize() == rd["qsize"]
    for k in rd["data_keys"]:
        assert k in data
    assert_lists_identical(model, rd["out"], name)


@pytest.mark.parametrize("name", case_names("fedopt"))
def test_fedopt_plugin_golden(name):
    case = load_case(name)
    uh, agg = _plugin("fedopt")
    for r, rd in enumerate(case["rounds"]):
        gid = uh.put_global_model(rd["old"], f"global-{r}")
        for arrays, n in rd["updates"]:
            uh.submit(arrays, n, model_id=gid)
        model, data = agg.combine_models(helper=None, delete_models=True, parameters=case["params"])
        assert_lists_identical(model, rd["out"], f"{name} r{r} out")
        assert data.get("nr_aggregated_models", -1) == rd["nr"]
        assert uh.model_updates.qsize() == rd["qsize"]
        if rd["m"] is not None:
            assert_lists_identical(agg.m, rd["m"], f"{name} r{r} m")
            assert_lists_identical(agg.v, rd["v"], f"{name} r{r} v")
        else:
            assert agg.m is None and agg.v is None


# ------------------------------------------------------------------------- ops level, random
def _updates(rng, K, P, dtype=np.float32, offset=0):
    base = rng.standard_normal(P)
    ups = [(base + 0.01 * rng.standard_normal(P)).astype(dtype) for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    return ups, ns


def _to_dev(a, offset=0):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if offset:
        big = torch.empty(t.numel() + offset, dtype=t.dtype, device=DEV)
        d = big[offset:]
        d.copy_(t.to(DEV))
        return d
    return t.to(DEV)


def _fold_dev(ups_dev, ns, agg_dtype, chunks=None):
    from fedn_amd import ops
    Ns = list(np.cumsum(ns))
    agg = torch.empty(ups_dev[0].numel(), dtype=agg_dtype, device=DEV)
    if chunks is None:
        ops.fedavg_fold(agg, ups_dev, ns, Ns, init=True)
    else:
        k0, first = 0, True
        for c in chunks:
            ops.fedavg_fold(agg, ups_dev[k0:k0 + c], ns[k0:k0 + c], Ns[k0:k0 + c], init=first)
            first = False
            k0 += c
    torch.cuda.synchronize()
    return agg.cpu().numpy()


@pytest.mark.parametrize("K", [2, 3, 8, 9, 63, 64, 65, 130])
@pytest.mark.parametrize("P", [1, 5, 4099, 1 << 16])
def test_fedavg_ops_vs_oracle(K, P):
    rng = np.random.default_rng(K * 1000 + P)
    ups, ns = _updates(rng, K, P)
    want = ref.fedavg_flat(ups, ns)
    got = _fold_dev([_to_dev(u) for u in ups], ns, torch.float32)
    assert_lists_identical([got], [want], f"K={K} P={P}")


@pytest.mark.parametrize("offset", [1, 2, 3])
def test_fedavg_misaligned_scalar_path(offset):
    rng = np.random.default_rng(offset)
    ups, ns = _updates(rng, 5, 1001)
    want = ref.fedavg_flat(ups, ns)
    got = _fold_dev([_to_dev(u, offset) for u in ups], ns, torch.float32)
    assert_lists_identical([got], [want], "misaligned")


def test_fedavg_streaming_chunks_equal_single_pass():
    rng = np.random.default_rng(7)
    ups, ns = _updates(rng, 20, 12345)
    dev = [_to_dev(u) for u in ups]
    a = _fold_dev(dev, ns, torch.float32)
    b = _fold_dev(dev, ns, torch.float32, chunks=[1, 2, 5, 1, 11])
    assert_lists_identical([b], [a], "waves")
    assert_lists_identical([a], [ref.fedavg_flat(ups, ns)], "oracle")


@pytest.mark.parametrize("dt,agg_dt", [(np.float64, torch.float64), (np.float16, torch.float16),
                                        (np.int64, torch.float64), (np.int32, torch.float64)])
def test_fedavg_other_dtypes(dt, agg_dt):
    rng = np.random.default_rng(11)
    if np.dtype(dt).kind == "i":
        ups = [rng.integers(-10**6, 10**6, 3001).astype(dt) for _ in range(6)]
        ns = [int(v) for v in rng.integers(1, 5001, 6)]
    else:
        ups, ns = _updates(rng, 6, 3001, dt)
    want = ref.fedavg_flat(ups, ns)
    got = _fold_dev([_to_dev(u) for u in ups], ns, agg_dt)
    assert_lists_identical([got], [want], str(dt))


def test_fedavg_f32_updates_into_f64_aggregate():
    rng = np.random.default_rng(12)
    ups, ns = _updates(rng, 5, 777)
    first = ups[0].astype(np.float64)
    want = ref.fedavg_flat([first] + ups[1:], ns)
    from fedn_amd import ops
    agg = _to_dev(first)
    ops.fedavg_fold(agg, [_to_dev(u) for u in ups[1:]], ns[1:], list(np.cumsum(ns))[1:], init=False)
    torch.cuda.synchronize()
    assert_lists_identical([agg.cpu().numpy()], [want], "f32->f64")


@pytest.mark.parametrize("K,P", [(9, 10001), (2, 1), (3, 5), (70, 8192 * 3 + 7), (64, 1 << 16), (130, 4099)])
def test_fedavg_bf16_defined_as_fp32_on_upcast(K, P):
    """bf16 has no numpy reference: parity = fp32 oracle on the exactly upcast values. Covers the
    8-strips-of-4 map's whole tiles, its ragged tile, and K > 64 (continuing a stored aggregate)."""
    rng = np.random.default_rng(13 + K + P)
    ups, ns = _updates(rng, K, P)
    bf = [torch.from_numpy(u).to(torch.bfloat16) for u in ups]
    up32 = [b.to(torch.float32).numpy() for b in bf]
    want = ref.fedavg_flat(up32, ns)
    got = _fold_dev([b.to(DEV) for b in bf], ns, torch.float32)
    assert_lists_identical([got], [want], f"bf16 K={K} P={P}")
    if K > 8:
        got_c = _fold_dev([b.to(DEV) for b in bf], ns, torch.float32, chunks=[2, 4, K - 6])
        assert_lists_identical([got_c], [want], "bf16 chunked")


def test_fedavg_bf16_special_values():
    """bf16 zeros, signed zeros, subnormals, extremes, inf and NaN through the f32 fold."""
    vals = np.array([0.0, -0.0, 1e-40, -9.2e-41, 3.3e38, -3.3e38, np.inf, -np.inf, np.nan, 1.0, -2.5, 7.0],
                    dtype=np.float32)
    rng = np.random.default_rng(6)
    bf = [torch.from_numpy(rng.permutation(np.tile(vals, 700)).astype(np.float32)).to(torch.bfloat16) for _ in range(7)]
    ns = [3, 1, 4000, 1, 5, 9, 2]
    with np.errstate(all="ignore"):
        want = ref.fedavg_flat([b.to(torch.float32).numpy() for b in bf], ns)
    got = _fold_dev([b.to(DEV) for b in bf], ns, torch.float32)
    assert_lists_identical([got], [want], "bf16 special")


def test_fedavg_special_values():
    """zeros, signed zeros, denormals, huge values, inf and NaN follow IEEE like numpy."""
    vals = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-40, 3e38, -3e38, np.inf, -np.inf, np.nan, 1.0, -2.5],
                    dtype=np.float32)
    rng = np.random.default_rng(5)
    ups = [rng.permutation(np.tile(vals, 11)).astype(np.float32) for _ in range(7)]
    ns = [3, 1, 4000, 1, 5, 9, 2]
    with np.errstate(all="ignore"):
        want = ref.fedavg_flat(ups, ns)
    got = _fold_dev([_to_dev(u) for u in ups], ns, torch.float32)
    assert_lists_identical([got], [want], "special")


# ------------------------------------------------------------------------- FedOpt ops level
@pytest.mark.parametrize("opt", ["adam", "yogi", "adagrad"])
@pytest.mark.parametrize("K", [1, 4, 70])
@pytest.mark.parametrize("old_dt,upd_dt", [(np.float32, np.float32), (np.float64, np.float32),
                                           (np.float64, np.float64)])
def test_fedopt_ops_two_rounds(opt, K, old_dt, upd_dt):
    from fedn_amd import ops
    rng = np.random.default_rng(K + len(opt))
    P = 2053
    old = rng.standard_normal(P).astype(old_dt)
    params = {"serveropt": opt, "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "tau": 1e-3}
    st = ref.FedOptState()
    m_dev = v_dev = None
    for r in range(2):
        ups = [(old + 0.01 * rng.standard_normal(P)).astype(upd_dt) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 5001, K)]
        want, _ = ref.fedopt_combine(st, [([u], n) for u, n in zip(ups, ns)], [old], params)
        old_d = _to_dev(old)
        pg_dt, m_dt = ops.fedopt_dtypes(ops.torch_dtype(upd_dt), old_d.dtype, None if m_dev is None else m_dev.dtype)
        pg = torch.empty(P, dtype=pg_dt, device=DEV)
        m_out = torch.empty(P, dtype=m_dt, device=DEV)
        v_out = torch.empty(P, dtype=torch.float64, device=DEV)
        out = torch.empty(P, dtype=torch.float64, device=DEV)
        ops.fedopt_step(old_d, [_to_dev(u) for u in ups], ns, list(np.cumsum(ns)), first=True, final=True, pg=pg,
                        m_in=m_dev, m_out=m_out, v_in=v_dev, v_out=v_out, out=out, **params)
        torch.cuda.synchronize()
        assert_lists_identical([out.cpu().numpy()], want, f"r{r} out")
        assert_lists_identical([m_out.cpu().numpy()], st.m, f"r{r} m")
        assert_lists_identical([v_out.cpu().numpy()], st.v, f"r{r} v")
        m_dev, v_dev, old = m_out, v_out, want[0]


def test_fedopt_bf16_updates():
    from fedn_amd import ops
    rng = np.random.default_rng(21)
    P, K = 4099, 5
    old = rng.standard_normal(P).astype(np.float32)
    bf = [torch.from_numpy(old + 0.01 * rng.standard_normal(P).astype(np.float32)).to(torch.bfloat16) for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    st = ref.FedOptState()
    want, _ = ref.fedopt_combine(st, [([b.float().numpy()], n) for b, n in zip(bf, ns)], [old], {"serveropt": "yogi"})
    out = torch.empty(P, dtype=torch.float64, device=DEV)
    m_out = torch.empty(P, dtype=torch.float32, device=DEV)
    v_out = torch.empty(P, dtype=torch.float64, device=DEV)
    ops.fedopt_step(_to_dev(old), [b.to(DEV) for b in bf], ns, list(np.cumsum(ns)), first=True, final=True,
                    m_out=m_out, v_out=v_out, out=out, serveropt="yogi")
    torch.cuda.synchronize()
    assert_lists_identical([out.cpu().numpy()], want, "bf16 fedopt")


# ------------------------------------------------------------------------- full size, sampled
@pytest.mark.slow
def test_fedavg_full_size_sampled():
    """100 M fp32 x 8 clients (BASELINE config 2) on the GPU; the oracle checks 3 slices.
    Elementwise independence makes any slice a complete check of the elements in it."""
    from fedn_amd import ops
    P, K = 100_000_000, 8
    g = torch.Generator(device=DEV).manual_seed(0)
    base = torch.randn(P, generator=g, device=DEV)
    ups = [base + 0.01 * torch.randn(P, generator=g, device=DEV) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
    agg = torch.empty(P, device=DEV)
    ops.fedavg_fold(agg, ups, ns, list(np.cumsum(ns)), init=True)
    torch.cuda.synchronize()
    for lo in (0, P // 2 - 12345, P - 1_000_003):
        sl = slice(lo, lo + 1_000_003)
        want = ref.fedavg_flat([u[sl].cpu().numpy() for u in ups], ns)
        assert_lists_identical([agg[sl].cpu().numpy()], [want], f"slice {lo}")


def test_fedavg_north_star_size_sampled():
    """The metric's workload at full size, 64 x 100 M fp32 (and bf16), folded in one launch; the
    oracle checks 3 slices of 200 K elements plus the last tile."""
    from fedn_amd import ops
    P, K = 100_000_000, 64
    g = torch.Generator(device=DEV).manual_seed(2)
    base = torch.randn(P, generator=g, device=DEV)
    ups = [torch.randn(P, generator=g, device=DEV).mul_(0.01).add_(base) for _ in range(K)]
    del base
    ns = [int(v) for v in np.random.default_rng(2).integers(1, 5001, K)]
    Ns = list(np.cumsum(ns))
    for dt in ("f32", "bf16"):
        if dt == "bf16":
            ups = [u.to(torch.bfloat16) for u in ups]
        agg = torch.empty(P, device=DEV)
        ops.fedavg_fold(agg, ups, ns, Ns, init=True)
        torch.cuda.synchronize()
        for lo in (0, 37_000_001, P - 200_000):
            sl = slice(lo, lo + 200_000)
            want = ref.fedavg_flat([u[sl].float().cpu().numpy() for u in ups], ns)
            assert_lists_identical([agg[sl].cpu().numpy()], [want], f"{dt} slice {lo}")
    del ups, agg
    torch.cuda.empty_cache()


def test_fedopt_configs3_size_sampled():
    """BASELINE configs[3] at full size: 32 x 350 M fp32 FedAdam, round 1 and the fp64 steady
    state, one fused launch each; the oracle checks 3 slices of 100 K elements of out, m and v."""
    from fedn_amd import ops
    P, K = 350_000_000, 32
    g = torch.Generator(device=DEV).manual_seed(3)
    old = torch.randn(P, generator=g, device=DEV)
    ups = [torch.randn(P, generator=g, device=DEV).mul_(0.01).add_(old) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(3).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    params = {"serveropt": "adam", "learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
    kw = {k: params[k] for k in ("learning_rate", "beta1", "beta2", "tau")}
    out = torch.empty(P, dtype=torch.float64, device=DEV)
    v = torch.empty(P, dtype=torch.float64, device=DEV)
    m = torch.empty(P, dtype=torch.float32, device=DEV)
    ops.fedopt_step(old, ups, ns, Ns, first=True, final=True, m_out=m, v_out=v, out=out, serveropt="adam", **kw)
    old64, m64 = out.clone(), m.double()
    del m
    m2 = torch.empty(P, dtype=torch.float64, device=DEV)
    v2 = torch.empty(P, dtype=torch.float64, device=DEV)
    out2 = torch.empty(P, dtype=torch.float64, device=DEV)
    ops.fedopt_step(old64, ups, ns, Ns, first=True, final=True, m_in=m64, m_out=m2, v_in=v, v_out=v2, out=out2,
                    serveropt="adam", **kw)
    torch.cuda.synchronize()
    for lo in (0, 123_456_789, P - 100_000):
        sl = slice(lo, lo + 100_000)
        st = ref.FedOptState()
        upd = [([u[sl].cpu().numpy()], n) for u, n in zip(ups, ns)]
        want1, _ = ref.fedopt_combine(st, upd, [old[sl].cpu().numpy()], params)
        assert_lists_identical([out[sl].cpu().numpy(), v[sl].cpu().numpy()], [want1[0], st.v[0]], f"round 1 {lo}")
        st.m = [st.m[0].astype(np.float64)]       # the steady state takes m in float64 (round >= 3)
        want2, _ = ref.fedopt_combine(st, upd, want1, params)
        assert_lists_identical([out2[sl].cpu().numpy(), m2[sl].cpu().numpy(), v2[sl].cpu().numpy()],
                               [want2[0], st.m[0], st.v[0]], f"steady {lo}")
    del ups, old, old64, m64, m2, v, v2, out, out2
    torch.cuda.empty_cache()


def test_fedopt_waves_1b_sampled():
    """BASELINE configs[4] as defined: 1 B-param bf16 updates, 128 of them, streamed
    from pinned host memory in 16 waves of 8 over 2 parameter slices, FedYogi. 8 distinct pinned
    buffers, each sent 16 times, as bench.py's fedopt_waves does; the oracle checks 3 slices of 100 K
    elements (one straddling the two slices). ~10 s on the box (16 x 8 x 2 GB of H2D)."""
    from fedn_amd.waves import WaveFedOpt
    P, K, pool = 1_000_000_000, 128, 8
    g = torch.Generator(device=DEV).manual_seed(6)
    base = torch.randn(P, generator=g, device=DEV)
    host = []
    for _ in range(pool):
        h = torch.empty(P, dtype=torch.bfloat16, pin_memory=True)
        h.copy_((base + 0.01 * torch.randn(P, generator=g, device=DEV)).to(torch.bfloat16))
        host.append(h)
    base = base.cpu()
    ups = [host[k % pool] for k in range(K)]
    ns = [int(v) for v in np.random.default_rng(6).integers(1, 5001, K)]
    params = {"serveropt": "yogi", "learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
    wf = WaveFedOpt([DEV, DEV], P, wave=8)
    old = wf.slices(base)
    outs = wf.round(ups, ns, old, params)
    lo_hi = wf.bounds
    for lo in (0, 499_999_950, P - 100_000):
        sl = slice(lo, lo + 100_000)
        st = ref.FedOptState()
        upd = [([u[sl].float().numpy()], n) for u, n in zip(ups, ns)]
        want, _ = ref.fedopt_combine(st, upd, [base[sl].numpy()], params)
        got = np.empty(100_000)
        for d, (a, b) in enumerate(lo_hi):      # the slice may straddle the two devices' parts
            s0, s1 = max(lo, a), min(lo + 100_000, b)
            if s1 > s0:
                got[s0 - lo:s1 - lo] = outs[d][s0 - a:s1 - a].cpu().numpy()
        assert_lists_identical([got], [want[0]], f"slice {lo}")
    del host, ups, outs, old, wf
    torch.cuda.empty_cache()


# ------------------------------------------------------------------------- Control.reduce
@pytest.mark.parametrize("workers", [1, 3])
@pytest.mark.parametrize("name", case_names("reduce"))
def test_control_reduce_golden(name, workers):
    from fedn_amd.reduce import reduce_models
    case = load_case(name)
    store = {f"m{c}": m for c, (m, kind) in enumerate(zip(case["models"], case["plan"])) if kind != "missing"}
    deleted = []

    def fetch(mid):
        if mid not in store:
            raise KeyError(mid)
        return store[mid]

    combiners = [{"name": f"c{c}", "model_id": f"m{c}"} for c in range(len(case["plan"]))]
    model, meta = reduce_models(combiners, fetch=fetch, load=lambda d: d, delete=deleted.append, workers=workers)
    assert_lists_identical(model, case["out"], name)
    assert deleted == [c["model_id"] for c in combiners]
    assert set(meta) == {"time_fetch_model", "time_load_model", "time_aggregate_model"}


# ------------------------------------------------------------------------- streaming ingest
@pytest.mark.parametrize("name", ["fedavg_mnist_k2", "fedavg_odd_k17", "fedavg_skipbad_k4", "fedavg_int64_k3",
                                  "fedavg_odd_k1"] + MIXED_FEDAVG + NARROW_FEDAVG)
def test_staging_ingest_fedavg_golden(name):
    """Updates staged into HBM on arrival (ingest.StagingUpdateHandler) give the same result."""
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rd = load_case(name)["rounds"][0]
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=3)
    for arrays, n in rd["updates"]:
        uh.submit(arrays, n, via=st)
    model, data = get_aggregator("fedavg", st).combine_models(helper=None)
    st.close()
    assert data["nr_aggregated_models"] == rd["nr"]
    assert_lists_identical(model, rd["out"], name)


@pytest.mark.parametrize("name", ["fedopt_adam_3r", "fedopt_yogi_lr1e-2_k8"] + MIXED_FEDOPT + NARROW_FEDOPT)
def test_staging_ingest_fedopt_golden(name):
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    case = load_case(name)
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=2)
    agg = get_aggregator("fedopt", st)
    for r, rd in enumerate(case["rounds"]):
        gid = uh.put_global_model(rd["old"], f"global-{r}")
        for arrays, n in rd["updates"]:
            uh.submit(arrays, n, model_id=gid, via=st)
        model, _ = agg.combine_models(helper=None, parameters=case["params"])
        assert_lists_identical(model, rd["out"], f"{name} r{r}")
    st.close()


def _mixed_round(rng, uh, st, shapes, K, host_at, model_id="global", base=None):
    """K updates in FIFO order; those at positions in ``host_at`` bypass the ingest (host
    arrays at combine time), the rest are staged into HBM on arrival (StagedModel)."""
    if base is None:
        base = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ups = []
    for k in range(K):
        arrays = [(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base]
        arrays.append(np.array([int(rng.integers(0, 1000))], dtype=np.int64))   # BatchNorm-like counter
        n = int(rng.integers(1, 5001))
        uh.submit(arrays, n, model_id=model_id, via=None if k in host_at else st)
        ups.append((arrays, n))
    return ups


@pytest.mark.parametrize("K,host_at", [(150, {70, 71, 72, 100}), (64, set()), (65, set()), (3, {0})])
def test_staging_batched_fedavg_mixed(K, host_at):
    """Device-resident updates fold in batched multi-client launches (flush at 64), host
    updates in between on arrival, the last batch chunk by chunk with overlapped D2H:
    bit-identical to the oracle's sequential fold, int64 group included."""
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(K)
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=3)
    ups = _mixed_round(rng, uh, st, [(300, 7), (1029,), (5,)], K, host_at)
    model, data = get_aggregator("fedavg", st).combine_models(helper=None)
    st.close()
    want, nr = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == nr == K
    assert_lists_identical(model, want, f"K={K}")


@pytest.mark.parametrize("K,host_at", [(150, {0, 90}), (70, set()), (20, {5})])
def test_staging_batched_fedopt_mixed(K, host_at):
    """FedOpt with staged updates: pending batches fold into pg (flush at 64) or straight into
    the fused server step; two rounds with m / v carried; == the oracle."""
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(1000 + K)
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=3)
    agg = get_aggregator("fedopt", st)
    shapes = [(64, 33), (17,)]
    old = [rng.standard_normal(s).astype(np.float32) for s in shapes] + [np.array([3], dtype=np.int64)]
    state = ref.FedOptState()
    params = {"serveropt": "yogi", "learning_rate": 1e-2}
    for r in range(2):
        gid = uh.put_global_model(old, f"g{r}")
        ups = _mixed_round(rng, uh, st, shapes, K, host_at, model_id=gid,
                           base=[o.astype(np.float32) for o in old[:2]])
        model, data = agg.combine_models(helper=None, parameters=params)
        want, _ = ref.fedopt_combine(state, ups, old, params)
        assert data["nr_aggregated_models"] == K
        assert_lists_identical(model, want, f"K={K} r{r}")
        assert_lists_identical(agg.m, state.m, f"K={K} r{r} m")
        assert_lists_identical(agg.v, state.v, f"K={K} r{r} v")
        old = want
    st.close()


def test_staging_batched_large_chunked_d2h():
    """A 24 M-element fp32 model (three 32 MiB D2H chunks) from 12 staged updates: the chunked
    fold + overlapped D2H equals one whole-buffer fold on the device."""
    from fedn_amd import ops
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(24)
    P, K = 24_000_000 + 77, 12
    base = rng.standard_normal(P).astype(np.float32)
    ups = [(base + np.float32(0.01) * rng.standard_normal(P).astype(np.float32)) for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=4)
    for u, n in zip(ups, ns):
        uh.submit([u], n, via=st)
    model, _ = get_aggregator("fedavg", st).combine_models(helper=None)
    st.close()
    want = torch.empty(P, dtype=torch.float32, device=DEV)
    ops.fedavg_fold(want, [torch.from_numpy(u).to(DEV) for u in ups], ns, list(np.cumsum(ns)), init=True)
    assert np.array_equal(model[0].view(np.uint32), want.cpu().numpy().view(np.uint32))


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("name", ["fedavg_mnist_k2", "fedavg_odd_k8", "fedavg_int32_k3", "fedavg_skipbad_k4",
                                  "fedavg_mix_f32_f64_k4", "fedavg_bcast_k4", "fedavg_mix_pertensor_k5",
                                  "fedavg_unsigned_k3", "fedavg_narrow_mixed_k3", "fedavg_bool_k3"])
def test_staging_ingest_npz_bytes(name, native):
    """Updates arriving as npz bytes (numpy savez_compressed, as FEDn clients upload them):
    inflated by the native codec straight into pinned memory (native=True) or decoded by
    the helper (native=False), staged into HBM on arrival, folded bit-exactly."""
    import io
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.helper import Helper
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rd = load_case(name)["rounds"][0]
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=Helper(), device=DEV, workers=3, native_decode=native)
    for arrays, n in rd["updates"]:
        b = io.BytesIO()
        np.savez_compressed(b, **{str(i): a for i, a in enumerate(arrays)})
        uh.submit_bytes(b.getvalue(), n, via=st)
    model, data = get_aggregator("fedavg", st).combine_models(helper=Helper())
    st.close()
    assert data["nr_aggregated_models"] == rd["nr"]
    assert_lists_identical(model, rd["out"], name)


@pytest.mark.parametrize("ndev,sink", [(1, "device"), (1, "device-tiny"), (1, "host"), (2, "host")])
@pytest.mark.parametrize("name", ["fedavg_mnist_k2", "fedavg_odd_k8", "fedavg_int32_k3", "fedavg_skipbad_k4",
                                  "fedavg_mix_i64_f32_k3", "fedavg_bcast_k4"])
def test_streaming_upload_ingest(name, ndev, sink):
    """Updates uploaded through ModelService.Upload in 64 KiB chunks are decoded WHILE they
    stream (upload.StreamingUpload), adopted by the staging handler when their ModelUpdate
    arrives and placed in HBM: decoded straight to device blocks through the pinned ring
    (sink "device"; "device-tiny" = 4 KiB slots x 2, so the ring wraps many times inside and
    across tensors), or to pinned host blocks copied tensor by tensor (one device, or as
    parameter slices over two): folded bit-exactly; the stored upload bytes are untouched."""
    import io
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.helper import Helper
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryModelService, MemoryUpdateHandler, upload_requests
    from fedn_amd.upload import StreamingUpload
    rd = load_case(name)["rounds"][0]
    uh = MemoryUpdateHandler()
    devs = [DEV] * ndev
    st = StagingUpdateHandler(uh, helper=Helper(), device=DEV, workers=3, devices=devs if ndev > 1 else None)
    kw = {"host": {"device_decode": False}, "device": {}, "device-tiny": {"slot": 4096, "ring": 2}}[sink]
    svc = StreamingUpload(MemoryModelService(uh.store), st, workers=2, **kw)
    for k, (arrays, n) in enumerate(rd["updates"]):
        b = io.BytesIO()
        np.savez_compressed(b, **{str(i): a for i, a in enumerate(arrays)})
        svc.Upload(upload_requests(b.getvalue(), f"up{k}", chunk=65536), None)
        assert uh.store.get(f"up{k}").data == b.getvalue()
        uh.submit_uploaded(f"up{k}", n, via=st)
    agg = Aggregator(st, devices=devs) if ndev > 1 else Aggregator(st)
    model, data = agg.combine_models(helper=Helper())
    svc.close()
    st.close()
    assert data["nr_aggregated_models"] == rd["nr"]
    assert_lists_identical(model, rd["out"], name)


@pytest.mark.parametrize("name", ["fedopt_adam_3r", "fedopt_yogi_lr1e-2_k8", "fedopt_adagrad_3r",
                                  "fedopt_mix_yogi_3r"])
def test_streaming_upload_fedopt(name):
    """FedOpt over three rounds with every client update decoded into HBM during its upload
    (the global model from load_model, m / v carried): == the reference's fixtures."""
    import io
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.helper import Helper
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryModelService, MemoryUpdateHandler, upload_requests
    from fedn_amd.upload import StreamingUpload
    case = load_case(name)
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=Helper(), device=DEV, workers=2)
    svc = StreamingUpload(MemoryModelService(uh.store), st, workers=2, slot=8192, ring=2)
    agg = get_aggregator("fedopt", st)
    for r, rd in enumerate(case["rounds"]):
        gid = uh.put_global_model(rd["old"], f"global-{r}")
        for k, (arrays, n) in enumerate(rd["updates"]):
            b = io.BytesIO()
            np.savez_compressed(b, **{str(i): a for i, a in enumerate(arrays)})
            svc.Upload(upload_requests(b.getvalue(), f"r{r}u{k}", chunk=5000), None)
            uh.submit_uploaded(f"r{r}u{k}", n, model_id=gid, via=st)
        model, _ = agg.combine_models(helper=Helper(), parameters=case["params"])
        assert_lists_identical(model, rd["out"], f"{name} r{r}")
    svc.close()
    st.close()


def test_streaming_upload_ingest_large_ring():
    """Multi-MiB tensors (fp32 + int64 + fp16) through the device sink with 64 KiB slots x 3,
    the clients' chunks cut at odd sizes: == the oracle's fold of the same arrays."""
    import io
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.helper import Helper
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryModelService, MemoryUpdateHandler, upload_requests
    from fedn_amd.upload import StreamingUpload
    rng = np.random.default_rng(77)
    base = [rng.standard_normal((1031, 997)).astype(np.float32), rng.standard_normal(333_333).astype(np.float16)]
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=Helper(), device=DEV, workers=3)
    svc = StreamingUpload(MemoryModelService(uh.store), st, workers=3, slot=65536, ring=3)
    ups = []
    for k in range(5):
        arrays = [(base[0] + 0.01 * rng.standard_normal(base[0].shape)).astype(np.float32),
                  rng.integers(-9, 9, 4099).astype(np.int64),
                  (base[1] + 0.01 * rng.standard_normal(base[1].shape)).astype(np.float16)]
        n = int(rng.integers(1, 5001))
        b = io.BytesIO()
        np.savez_compressed(b, **{str(i): a for i, a in enumerate(arrays)})
        svc.Upload(upload_requests(b.getvalue(), f"L{k}", chunk=100_003 + 7 * k), None)
        uh.submit_uploaded(f"L{k}", n, via=st)
        ups.append((arrays, n))
    model, data = Aggregator(st).combine_models(helper=Helper())
    svc.close()
    st.close()
    want, nr = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == nr == 5
    assert_lists_identical(model, want, "large ring")


def test_helper_increment_average_gpu():
    """fedn_amd.helper.Helper.increment_average == numpyhelper's (the reference KAT + random)."""
    from fedn_amd.helper import Helper
    c = load_case("kat_int64")["raw"]
    out = Helper().increment_average([c["m1_t0"]], [c["m2_t0"]], int(c["a"]), int(c["W"]))
    assert_lists_identical(out, [c["out_t0"]], "kat")
    rng = np.random.default_rng(9)
    m1 = [rng.standard_normal((7, 3)).astype(np.float32), rng.standard_normal(5).astype(np.float32)]
    m2 = [rng.standard_normal((7, 3)).astype(np.float32), rng.standard_normal(5).astype(np.float32)]
    assert_lists_identical(Helper().increment_average(m1, m2, 37, 1234), ref.increment_average(m1, m2, 37, 1234), "rnd")


# ------------------------------------------------------------------------- one process, several devices
@pytest.mark.parametrize("name", ["fedavg_mnist_k2", "fedavg_odd_k17", "fedavg_int64_k3", "fedavg_skipbad_k4",
                                  "fedavg_odd_k1", "fedavg_flat_k8"] + MIXED_FEDAVG + NARROW_FEDAVG)
@pytest.mark.parametrize("ndev", [2, 3])
def test_multidevice_fedavg_golden(name, ndev):
    """Parameter-slice sharding across devices inside one process (multidev.py); the box has
    one GPU, so the shards are placed on cuda:0 repeatedly — the slicing, per-shard H2D and
    per-shard D2H into the host result are exercised all the same."""
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rd = load_case(name)["rounds"][0]
    uh = MemoryUpdateHandler()
    for arrays, n in rd["updates"]:
        uh.submit(arrays, n)
    model, data = Aggregator(uh, devices=[DEV] * ndev).combine_models(helper=None)
    assert data["nr_aggregated_models"] == rd["nr"]
    assert_lists_identical(model, rd["out"], f"{name} x{ndev}")


@pytest.mark.parametrize("name", case_names("fedopt"))
@pytest.mark.parametrize("ndev", [2, 3])
def test_multidevice_fedopt_golden(name, ndev):
    """FedOpt with old / pg / m / v sharded over devices in one process, over all rounds of
    every golden FedOpt case (m and v reassembled from the device slices)."""
    from fedn_amd.aggregators.fedopt import Aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    case = load_case(name)
    uh = MemoryUpdateHandler()
    agg = Aggregator(uh, devices=[DEV] * ndev)
    for r, rd in enumerate(case["rounds"]):
        gid = uh.put_global_model(rd["old"], f"global-{r}")
        for arrays, n in rd["updates"]:
            uh.submit(arrays, n, model_id=gid)
        model, data = agg.combine_models(helper=None, delete_models=True, parameters=case["params"])
        assert_lists_identical(model, rd["out"], f"{name} x{ndev} r{r} out")
        assert data.get("nr_aggregated_models", -1) == rd["nr"]
        if rd["m"] is not None:
            assert_lists_identical(agg.m, rd["m"], f"{name} x{ndev} r{r} m")
            assert_lists_identical(agg.v, rd["v"], f"{name} x{ndev} r{r} v")
        else:
            assert agg.m is None and agg.v is None


def test_multidevice_fedopt_large_flat():
    """3 M params over 4 slices, two yogi rounds, against the oracle."""
    from fedn_amd.multidev import ShardedFedOptPipeline, ShardedFedOptState
    rng = np.random.default_rng(37)
    st, ost = ShardedFedOptState(), ref.FedOptState()
    params = {"serveropt": "yogi", "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
    old = [rng.standard_normal(3_000_017).astype(np.float32)]
    for r in range(2):
        ups, ns = _updates(rng, 5, 3_000_017)
        pipe = ShardedFedOptPipeline([DEV] * 4, old, [ups[0]])
        total = 0
        for u, n in zip(ups, ns):
            total += n
            pipe.add([u], n, total)
        got = pipe.server_step(st, params)
        want, nr = ref.fedopt_combine(ost, [([u], n) for u, n in zip(ups, ns)], old, params)
        assert nr == 5
        assert_lists_identical(got, want, f"r{r}")
        assert_lists_identical(st.m_host(), ost.m, f"r{r} m")
        old = got


def test_cyclic_fold_allgather_single_rank():
    """CyclicShardedFedAvg at world size 1: per-round fold launches over chunk views of the
    client buffers + the copy into natural order == one fold (the oracle)."""
    from fedn_amd.sharded import CyclicShardedFedAvg
    rng = np.random.default_rng(41)
    P = 2_500_003
    ups, ns = _updates(rng, 6, P)
    want = ref.fedavg_flat(ups, ns)
    cs = CyclicShardedFedAvg(P, chunk=600_000)
    assert cs.rounds == 5
    dev_ups = [cs.local(torch.from_numpy(u).to(DEV)) for u in ups]
    agg = torch.empty(cs.local_len, device=DEV)
    full = cs.fold_allgather(agg, dev_ups, ns, list(np.cumsum(ns)), init=True)
    assert_lists_identical([full.cpu().numpy()], [want], "cyclic")


@pytest.mark.parametrize("kind", ["fedavg", "fedopt"])
@pytest.mark.parametrize("ndev", [1, 2])
def test_returned_model_is_caller_owned(kind, ndev):
    """The model handed back lives in its own host block: three more rounds (which reuse
    every staging slot and the pinned-host cache) leave it untouched, and it is writable."""
    from fedn_amd.aggregators.fedavg import Aggregator as FedAvg
    from fedn_amd.aggregators.fedopt import Aggregator as FedOpt
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(43)
    uh = MemoryUpdateHandler()
    agg = (FedAvg if kind == "fedavg" else FedOpt)(uh, devices=[DEV] * ndev)
    shapes = [(300, 70), (70,), (1000,)]
    old = [rng.standard_normal(sh).astype(np.float32) for sh in shapes]
    kept, copies = [], []
    for r in range(4):
        gid = uh.put_global_model(old, f"g{r}")
        for _ in range(3):
            uh.submit([(o + 0.01 * rng.standard_normal(o.shape)).astype(np.float32) for o in old],
                      int(rng.integers(1, 5000)), model_id=gid)
        model, _ = agg.combine_models(helper=None, parameters={"serveropt": "adam"} if kind == "fedopt" else None)
        kept.append(model)
        copies.append([np.array(a, copy=True) for a in model])
        old = [np.asarray(a, dtype=np.float32) for a in model]
    for r, (m, c) in enumerate(zip(kept, copies)):
        assert_lists_identical(m, c, f"round {r} model changed after later rounds")
    kept[0][0][0, 0] = 123.0
    assert kept[1][0][0, 0] != 123.0


def test_multidevice_large_flat():
    from fedn_amd.multidev import ShardedFedAvgPipeline
    rng = np.random.default_rng(31)
    ups, ns = _updates(rng, 5, 3_000_017)
    want = ref.fedavg_flat(ups, ns)
    pipe = ShardedFedAvgPipeline([DEV] * 4, [ups[0]])
    total = ns[0]
    for u, n in zip(ups[1:], ns[1:]):
        total += n
        pipe.add([u], n, total)
    assert_lists_identical(pipe.result(), [want], "multidev flat")


# ------------------------------------------------------------------------- helper primitives on the GPU
def test_helper_primitives_golden():
    """fedn_amd.helper.Helper primitives vs the REAL numpyhelper outputs (helper_ops fixture)."""
    from fedn_amd.helper import Helper
    h = Helper()
    c = load_case("helper_ops")["raw"]
    x32, y32, x64 = c["x32"], c["y32"], c["x64"]
    got = {
        "add_32_32": h.add([x32], [y32], 0.9, 0.1)[0],
        "add_64_32": h.add([x64], [y32], 0.99, 1.0 - 0.99)[0],
        "sub_32_64": h.subtract([x32], [x64])[0],
        "mul_32_s": h.multiply([x32], [1.0 - 0.9])[0],
        "pow_32": h.power([x32], 2)[0],
        "sqrt_64": h.sqrt([np.abs(x64)])[0],
        "div_32_64": h.divide([x32], [np.abs(x64) + 1.0])[0],
        "sign_64": h.sign([np.concatenate([x64, [0.0, -0.0]])])[0],
        "ones_32": h.ones([x32], 1e-4 ** 2)[0],
    }
    for k, v in got.items():
        assert_lists_identical([v], [c[k]], k)


@pytest.mark.parametrize("name", ["fedopt_adam_3r", "fedopt_yogi_3r", "fedopt_adagrad_3r"])
def test_stock_fedopt_server_step_on_gpu_helper(name):
    """FEDn's stock serveropt_* (fedopt.py:151-258), written against the helper API, run with
    fedn_amd.helper.Helper: the pseudo-gradient from the oracle, the server step on the GPU."""
    import math
    from fedn_amd.helper import Helper
    h = Helper()
    case = load_case(name)
    opt = (case["params"] or {}).get("serveropt", "adam")
    b1, b2, lr, tau = 0.9, 0.99, 1e-3, 1e-4
    m = v = None
    for r, rd in enumerate(case["rounds"]):
        pg, nr, total = None, 0, 0
        for arrays, n in rd["updates"]:              # fedopt.py:86-94
            total += n
            pg = ref.subtract(arrays, rd["old"]) if nr == 0 else ref.increment_average(
                pg, ref.subtract(arrays, rd["old"]), n, total)
            nr += 1
        if v is None:
            v = h.ones(pg, math.pow(tau, 2))
        m = h.multiply(pg, [(1.0 - b1)] * len(pg)) if m is None else h.add(m, pg, b1, (1.0 - b1))
        p = h.power(pg, 2)
        if opt == "adam":
            v = h.add(v, p, b2, (1.0 - b2))
        elif opt == "yogi":
            s = h.multiply(h.sign(h.add(v, p, 1.0, -1.0)), p)
            v = h.add(v, s, 1.0, -(1.0 - b2))
        else:
            v = h.add(v, p, 1.0, 1.0)
        sv = h.add(h.sqrt(v), h.ones(v, tau))
        model = h.add(rd["old"], h.divide(m, sv), 1.0, lr)
        assert_lists_identical(model, rd["out"], f"{name} r{r}")
        assert_lists_identical(m, rd["m"], f"{name} r{r} m")
        assert_lists_identical(v, rd["v"], f"{name} r{r} v")


def test_fedopt_f64_updates_over_f32_model_streamed():
    """pg dtype comes from the UPDATES (f64 here), also in the K = 0 server step of the
    streamed (plug-in) path: fedopt.py with float64 client updates over a float32 seed."""
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(41)
    old = [rng.standard_normal(1001).astype(np.float32)]
    ups = [([(old[0] + 0.01 * rng.standard_normal(1001)).astype(np.float64)], int(n))
           for n in rng.integers(1, 5001, 4)]
    st = ref.FedOptState()
    want, _ = ref.fedopt_combine(st, ups, old, {"serveropt": "adam"})
    uh = MemoryUpdateHandler()
    gid = uh.put_global_model(old, "g")
    for arrays, n in ups:
        uh.submit(arrays, n, model_id=gid)
    agg = get_aggregator("fedopt", uh)
    model, _ = agg.combine_models(parameters={"serveropt": "adam"})
    assert_lists_identical(model, want, "f64 over f32")
    assert_lists_identical(agg.m, st.m, "m")


def test_sharded_fedopt_kernel_single_rank():
    """ShardedFedOpt's default step (the fused kernel) over two rounds, world size 1."""
    from fedn_amd.sharded import ShardedFedOpt
    rng = np.random.default_rng(43)
    P, K = 5000, 70                                    # K > 64: the chunked path with a pg workspace
    old = rng.standard_normal(P).astype(np.float32)
    sh = ShardedFedOpt(P)
    st = ref.FedOptState()
    for r in range(2):
        ups = [(old + 0.01 * rng.standard_normal(P)).astype(np.float32) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 5001, K)]
        want, _ = ref.fedopt_combine(st, [([u], k) for u, k in zip(ups, ns)], [old], {"serveropt": "adagrad"})
        out = sh.step(_to_dev(old), [_to_dev(u) for u in ups], ns, list(np.cumsum(ns)),
                      {"serveropt": "adagrad"})
        torch.cuda.synchronize()
        assert_lists_identical([out.cpu().numpy()], want, f"r{r}")
        old = want[0]


# ------------------------------------------------------------------------- server functions (§8(f)-4)
@pytest.mark.parametrize("name", case_names("sf_wavg"))
def test_sf_weighted_average_golden(name):
    """GPU aggregate == the reference's example server function (server_functions.py:53-68)."""
    from fedn_amd.serverfunctions import WeightedAverage
    c = load_case(name)
    got = WeightedAverage(device=DEV).aggregate(c["prev"], {k: [u, md] for k, (u, md) in c["updates"].items()})
    assert_lists_identical(got, c["out"], name)


@pytest.mark.parametrize("name", case_names("sf_inc"))
def test_sf_incremental_golden(name):
    """GPU incremental aggregate == the reference's example (sf_incremental_aggregation.py), all rounds
    on one instance (running total carried over, stale previous_global on an empty round)."""
    from fedn_amd.serverfunctions import IncrementalAverage
    c = load_case(name)
    sf = IncrementalAverage(device=DEV)
    for r, rd in enumerate(c["rounds"]):
        for cid, u, md in rd["updates"]:
            sf.incremental_aggregate(cid, u, md, rd["prev"])
        assert_lists_identical(sf.get_incremental_aggregate_model(), rd["out"], f"{name} r{r}")


@pytest.mark.parametrize("acc_dt,upd_dt", [(np.float32, np.float32), (np.float64, np.float32),
                                           (np.float64, np.float64), (np.float32, np.float64)])
def test_weighted_sum_ops_k70(acc_dt, upd_dt):
    """fa_weighted_sum over 70 clients in one call (two launches of <= 64) vs numpy's loop."""
    from fedn_amd import ops
    rng = np.random.default_rng(47)
    P, K = 100_003, 70
    ups = [rng.standard_normal(P).astype(upd_dt) for _ in range(K)]
    w = [int(v) for v in rng.integers(1, 5001, K)]
    w[3] = 2.75                                  # a python float weight
    want = np.zeros(P, acc_dt)
    for u, k in zip(ups, w):
        want += u * k
    acc = torch.zeros(P, dtype=ops.torch_dtype(np.dtype(acc_dt)), device=DEV)
    ops.weighted_sum(acc, [torch.from_numpy(u).to(DEV) for u in ups], w)
    assert_lists_identical([acc.cpu().numpy()], [want], "weighted_sum")


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_running_mean_ops(dt):
    from fedn_amd import ops
    rng = np.random.default_rng(53)
    P = 1_000_003
    g = rng.standard_normal(P).astype(dt)
    m = rng.standard_normal(P).astype(dt)
    g[:4] = [0.0, -0.0, np.inf, np.nan]
    T, n = 123_457, 4_999
    want = (g * (T - n) + m * n) / T
    gd = torch.from_numpy(g).to(DEV)
    ops.running_mean(gd, torch.from_numpy(m).to(DEV), T - n, n, T)
    assert_lists_identical([gd.cpu().numpy()], [want], "running_mean")


# ------------------------------------------------------------------------- multi-device + sharded ingest
@pytest.mark.parametrize("ndev,K,host_at", [(3, 70, {10, 40}), (2, 5, set()), (2, 1, set())])
def test_multidevice_sharded_ingest_fedavg(ndev, K, host_at):
    """Updates staged as parameter slices over the devices (StagingUpdateHandler(devices=)),
    folded in batched per-device launches (host updates interleaved), result streamed back
    chunk by chunk per device: bit-identical to the oracle; K = 1 returns the update itself."""
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(50 + K)
    devs = [DEV] * ndev
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, devices=devs, workers=3)
    ups = _mixed_round(rng, uh, st, [(300, 7), (1029,), (5,)], K, host_at)
    model, data = Aggregator(st, devices=devs).combine_models(helper=None)
    st.close()
    want, nr = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == nr == K
    assert_lists_identical(model, want, f"x{ndev} K={K}")


@pytest.mark.parametrize("ndev,K,host_at", [(3, 70, {0, 66}), (2, 6, set())])
def test_multidevice_sharded_ingest_fedopt(ndev, K, host_at):
    """FedOpt over device slices with sharded staged updates: two rounds, m / v carried per
    device, the global model streamed in per device with the fused step; == the oracle."""
    from fedn_amd.aggregators.fedopt import Aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(2000 + K)
    devs = [DEV] * ndev
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, devices=devs, workers=3)
    agg = Aggregator(st, devices=devs)
    shapes = [(64, 33), (17,)]
    old = [rng.standard_normal(s).astype(np.float32) for s in shapes] + [np.array([3], dtype=np.int64)]
    state = ref.FedOptState()
    params = {"serveropt": "adam", "learning_rate": 1e-2}
    for r in range(2):
        gid = uh.put_global_model(old, f"g{r}")
        ups = _mixed_round(rng, uh, st, shapes, K, host_at, model_id=gid,
                           base=[o.astype(np.float32) for o in old[:2]])
        model, data = agg.combine_models(helper=None, parameters=params)
        want, _ = ref.fedopt_combine(state, ups, old, params)
        assert data["nr_aggregated_models"] == K
        assert_lists_identical(model, want, f"x{ndev} K={K} r{r}")
        assert_lists_identical(agg.m, state.m, f"x{ndev} K={K} r{r} m")
        assert_lists_identical(agg.v, state.v, f"x{ndev} K={K} r{r} v")
        old = want
    st.close()


@pytest.mark.parametrize("native", [True, False])
def test_multidevice_sharded_ingest_npz(native):
    """npz bytes inflated (native codec) or decoded (helper) and staged as device slices."""
    import io
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.helper import Helper
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rd = load_case("fedavg_odd_k8")["rounds"][0]
    devs = [DEV] * 3
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=Helper(), devices=devs, workers=3, native_decode=native)
    for arrays, n in rd["updates"]:
        b = io.BytesIO()
        np.savez_compressed(b, **{str(i): a for i, a in enumerate(arrays)})
        uh.submit_bytes(b.getvalue(), n, via=st)
    model, data = Aggregator(st, devices=devs).combine_models(helper=Helper())
    st.close()
    assert data["nr_aggregated_models"] == rd["nr"]
    assert_lists_identical(model, rd["out"], "sharded npz")


# ------------------------------------------------------------------------- non-numpy FEDn helpers
def _helper_stub(kind):
    """An object that identifies as FEDn's helper plug-in ``kind`` the way the real one does
    (module fedn.utils.helpers.plugins.<kind>; androidhelper's ``name`` reads "Helper")."""
    cls = type("Helper", (), {"__module__": f"fedn.utils.helpers.plugins.{kind}"})
    h = cls()
    h.name = "Helper" if kind == "androidhelper" else kind
    if kind != "androidhelper":
        h.subtract = lambda *a: None     # numpyhelper's primitives exist (binaryhelper inherits them)
    return h


@pytest.mark.parametrize("agg_name", ["fedavg", "fedopt"])
def test_unknown_helper_is_refused_not_guessed(agg_name, caplog):
    """A helper plug-in the aggregators do not implement: its increment_average is
    not assumed to be numpyhelper's. Every update's fold raises UnsupportedHelper inside
    combine_models' per-update try (fedavg.py:75-78 / fedopt.py:103-106: logged and skipped), so
    the round returns (None, data) with nothing aggregated — never a model computed with another
    helper's arithmetic."""
    class HalfHelper:                     # e.g. a user plug-in with its own (different) rule
        name = "numpyhelper"              # a name alone does not make it numpyhelper

        def increment_average(self, m1, m2, n, N):
            return [(x + y) / 2 for x, y in zip(m1, m2)]

        def subtract(self, m1, m2, a=1.0, b=1.0):
            return [x * a - y * b for x, y in zip(m1, m2)]

    uh, agg = _plugin(agg_name)
    rng = np.random.default_rng(3)
    base = [rng.standard_normal(40).astype(np.float32)]
    if agg_name == "fedopt":
        uh.put_global_model(base, "global")
    for k in range(3):
        uh.submit([base[0] + np.float32(0.01 * k)], 10 + k, model_id="global")
    import logging
    with caplog.at_level(logging.ERROR, logger="fedn"):
        model, data = agg.combine_models(helper=HalfHelper())
    assert model is None
    assert data["nr_aggregated_models"] == 0
    assert "not supported by the fedn_amd aggregators" in caplog.text


@pytest.mark.parametrize("name", case_names("helper_fedavg"))
def test_helper_fedavg_plugin(name):
    """The plug-in folds with the session helper's rule: androidhelper's (1 - w)*x + w*y on one
    flat float64 array (returned as that array), binaryhelper's numpyhelper rule on [array]."""
    case = load_case(name)
    rd = case["rounds"][0]
    android = case["helper"] == "androidhelper"
    uh, agg = _plugin("fedavg")
    for u, n in rd["updates"]:
        uh.submit(u if android else [u], n)
    model, data = agg.combine_models(helper=_helper_stub(case["helper"]))
    assert data["nr_aggregated_models"] == rd["nr"]
    got = model if android else model[0]
    assert isinstance(got, np.ndarray)
    assert_lists_identical([got], [rd["out"]], name)


@pytest.mark.parametrize("name", case_names("helper_fedopt"))
def test_helper_fedopt_plugin(name):
    case = load_case(name)
    android = case["helper"] == "androidhelper"
    uh, agg = _plugin("fedopt")
    helper = _helper_stub(case["helper"])
    for r, rd in enumerate(case["rounds"]):
        gid = uh.put_global_model(rd["old"] if android else [rd["old"]], f"g{r}")
        for u, n in rd["updates"]:
            uh.submit(u if android else [u], n, model_id=gid)
        model, data = agg.combine_models(helper=helper, parameters=case["params"])
        assert data["nr_aggregated_models"] == rd["nr"]
        assert uh.model_updates.qsize() == rd["qsize"]
        if rd["out"] is None:
            assert model is None
        else:
            assert_lists_identical(model, [rd["out"]], f"{name} r{r}")
            assert_lists_identical(agg.m, [rd["m"]], f"{name} r{r} m")
            assert_lists_identical(agg.v, [rd["v"]], f"{name} r{r} v")


@pytest.mark.parametrize("name", ["binary_fedavg_k5", "android_fedavg_k9"])
def test_helper_sessions_through_ingest(name):
    """The streaming ingest leaves androidhelper updates to the host path and decodes binaryhelper
    bytes with the helper's load (never as npz); the plug-in result is unchanged."""
    import io
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    case = load_case(name)
    rd = case["rounds"][0]
    android = case["helper"] == "androidhelper"
    helper = _helper_stub(case["helper"])
    if not android:      # decode raw float64 bytes like numpyhelper.load(file_type="raw_binary")
        helper.load = lambda fh: [np.frombuffer(fh.read(), dtype=np.float64)]
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=helper, device=DEV, workers=2)
    for u, n in rd["updates"]:
        if android:
            uh.submit(u, n, via=st)
        else:
            uh.submit_bytes(np.asarray(u, dtype=np.float64).tobytes(), n, via=st)
    model, data = get_aggregator("fedavg", st).combine_models(helper=helper)
    st.close()
    assert data["nr_aggregated_models"] == rd["nr"]
    assert_lists_identical([model if android else model[0]], [rd["out"]], name)


# ------------------------------------------------------------------------- fa_cast (mixed.py operand prep)
@pytest.mark.parametrize("src,dst", [(np.float16, np.float32), (np.float16, np.float64), (np.float32, np.float64),
                                     (np.int32, np.int64), (np.int32, np.float64), (np.int64, np.float64),
                                     (np.float32, np.float32), (np.int64, np.int64), (np.float16, np.float16)])
@pytest.mark.parametrize("xshape,oshape", [((1000,), (1000,)), ((1,), (4099,)), ((), (3, 5)), ((3, 1), (3, 7)),
                                           ((1, 7), (5, 7)), ((2, 1, 3), (4, 2, 5, 3)), ((0,), (0,))])
def test_cast_broadcast_vs_numpy(src, dst, xshape, oshape):
    """fa_cast == np.broadcast_to(x, shape).astype(dst): numpy's operand conversion (values that
    stress int64 -> float64 rounding included)."""
    from fedn_amd import ops
    rng = np.random.default_rng(11)
    if np.dtype(src).kind == "i":
        x = rng.integers(np.iinfo(src).min, np.iinfo(src).max, size=xshape, dtype=src)
    else:
        x = (rng.standard_normal(xshape) * 100).astype(src)
    out = torch.empty(oshape, dtype=ops.torch_dtype(dst), device=DEV)
    ops.cast(out, torch.from_numpy(np.ascontiguousarray(x)).to(DEV))
    want = np.broadcast_to(x, oshape).astype(dst)
    assert_lists_identical([out.cpu().numpy()], [want], f"{src}->{dst} {xshape}->{oshape}")


def test_cast_strided_source():
    """A non-contiguous source view (a transposed slice) is read through its strides."""
    from fedn_amd import ops
    x = torch.arange(60, dtype=torch.float32, device=DEV).view(6, 10)[:, 2:7].t()   # (5, 6), strided
    out = torch.empty(5, 6, dtype=torch.float64, device=DEV)
    ops.cast(out, x)
    assert torch.equal(out.cpu(), x.cpu().double())


def test_cast_narrowing_rules():
    """fa_cast: the two narrowing float casts round to nearest even like numpy's astype (specials,
    overflow to inf, subnormal results included); every other narrowing conversion is refused."""
    from fedn_amd import _abi, ops
    rng = np.random.default_rng(12)
    x64 = np.concatenate([rng.standard_normal(5000) * 10.0 ** rng.integers(-45, 45, 5000),
                          [0.0, -0.0, np.inf, -np.inf, np.nan, 3.5e38, 1e-46, 2.0 ** -149, 65520.0]])
    with np.errstate(all="ignore"):
        want32 = x64.astype(np.float32)
        x32 = (rng.standard_normal(5000) * 10.0 ** rng.integers(-9, 6, 5000)).astype(np.float32)
        x32 = np.concatenate([x32, np.array([65519.0, 65520.0, 6e-8, 3e-8, -0.0, np.inf, np.nan], np.float32)])
        want16 = x32.astype(np.float16)
    g32 = ops.cast(torch.empty(x64.size, dtype=torch.float32, device=DEV), torch.from_numpy(x64).to(DEV))
    assert_lists_identical([g32.cpu().numpy()], [want32], "f64 -> f32")
    g16 = ops.cast(torch.empty(x32.size, dtype=torch.float16, device=DEV), torch.from_numpy(x32).to(DEV))
    assert_lists_identical([g16.cpu().numpy()], [want16], "f32 -> f16")
    for src, dst in ((torch.float64, torch.float16), (torch.int64, torch.int32), (torch.float32, torch.int32)):
        with pytest.raises(_abi.FedAggError):
            ops.cast(torch.empty(8, dtype=dst, device=DEV), torch.ones(8, dtype=src, device=DEV))


@pytest.mark.parametrize("ndev", [2, 3])
@pytest.mark.parametrize("name", ["fedavg_mix_f32_f64_k4", "fedavg_bcast_k4", "fedavg_mix_i64_f32_k3"])
def test_multidevice_sharded_ingest_mixed(name, ndev):
    """Updates staged as parameter slices over several devices (ShardedStagedModel) whose layouts
    differ: the round moves to the per-tensor path on the first device, bit-exact."""
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rd = load_case(name)["rounds"][0]
    uh = MemoryUpdateHandler()
    devs = [DEV] * ndev
    st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=2, devices=devs)
    for arrays, n in rd["updates"]:
        uh.submit(arrays, n, via=st)
    model, data = Aggregator(st, devices=devs).combine_models(helper=None)
    st.close()
    assert data["nr_aggregated_models"] == rd["nr"]
    assert_lists_identical(model, rd["out"], f"{name} x{ndev}")


@pytest.mark.parametrize("ndev", [2])
@pytest.mark.parametrize("name", ["fedopt_mix_adam_3r", "fedopt_layout_change_3r"])
def test_multidevice_sharded_ingest_fedopt_mixed(name, ndev):
    from fedn_amd.aggregators.fedopt import Aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    case = load_case(name)
    uh = MemoryUpdateHandler()
    devs = [DEV] * ndev
    st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=2, devices=devs)
    agg = Aggregator(st, devices=devs)
    for r, rd in enumerate(case["rounds"]):
        gid = uh.put_global_model(rd["old"], f"global-{r}")
        for arrays, n in rd["updates"]:
            uh.submit(arrays, n, model_id=gid, via=st)
        model, _ = agg.combine_models(helper=None, parameters=case["params"])
        assert_lists_identical(model, rd["out"], f"{name} x{ndev} r{r}")
        assert_lists_identical(agg.m, rd["m"], f"{name} x{ndev} r{r} m")
        assert_lists_identical(agg.v, rd["v"], f"{name} x{ndev} r{r} v")
    st.close()


# ------------------------------------------------------------------------- GPU helper: power / norm
def test_helper_power_golden():
    """fednamdhelper.power vs the REAL numpyhelper (fixture): dtypes exact; integer powers and x**2
    bit-exact; other float exponents within 1e-6 relative (float32, the north-star bar) / 1e-15
    (float64) — numpy's float power is its host SIMD library's and is not reproducible across hosts."""
    from fedn_amd.helper import Helper
    c = load_case("helper_power_norm")["raw"]
    h = Helper()
    for a, tag in ((0.5, "half"), (3, "i3"), (-1.5, "neg1p5"), (2, "sq"), (0.7, "p07")):
        for src, key, rtol in (("x32", "pow32", 1e-6), ("x64", "pow64", 1e-15)):
            got, want = h.power([c[src]], a)[0], c[f"{key}_{tag}"]
            assert got.dtype == want.dtype and got.shape == want.shape
            if a == 2:
                assert_lists_identical([got], [want], f"{key}_{tag}")
            else:
                np.testing.assert_allclose(got, want, rtol=rtol, atol=0, err_msg=f"{key}_{tag}")
    assert_lists_identical(h.power([c["i64"]], 3), [c["powi64_3"]], "i64^3")
    assert_lists_identical(h.power([c["i64"]], 0), [c["powi64_0"]], "i64^0")
    got = h.power([np.abs(c["i64"])], 0.5)[0]
    assert got.dtype == c["powi64_f"].dtype
    np.testing.assert_allclose(got, c["powi64_f"], rtol=1e-15, atol=0)
    with pytest.raises(ValueError):
        h.power([c["i64"]], -1)


def test_helper_norm_golden():
    """fednamdhelper.norm vs the REAL numpyhelper: the matrix 1-norm for 2-D tensors, the float32
    accumulation dtype of a float32 model, 1e-6 relative."""
    from fedn_amd.helper import Helper
    c = load_case("helper_power_norm")["raw"]
    h = Helper()
    for args, key in (([c["x32"]], "norm_vec32"), ([c["m32"]], "norm_mat32"),
                      ([c["m32"], c["x64"], c["i64"], c["m64"]], "norm_mixed")):
        got = h.norm(args)
        assert np.asarray(got).dtype == c[key].dtype, key
        np.testing.assert_allclose(float(got), float(c[key]), rtol=1e-6, atol=0, err_msg=key)
    with pytest.raises(ValueError):
        h.norm([np.float32(3.0)])


def test_helper_increment_average_reuses_slots():
    """Stock fedavg.py on the helper calls increment_average once per client: the staging slots of
    a layout are allocated once and reused; results stay bit-exact (mixed layouts included)."""
    from fedn_amd.helper import Helper
    rng = np.random.default_rng(21)
    h = Helper()
    base = [rng.standard_normal((300, 7)).astype(np.float32), rng.standard_normal(11).astype(np.float32)]
    model, want, total = base, base, 0
    ids = set()
    for k in range(6):
        nxt = [(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base]
        n = int(rng.integers(1, 5001))
        total += n
        model = h.increment_average(model, nxt, n, total)
        want = ref.increment_average(want, nxt, n, total)
        ids |= {id(s) for sl, _ in h._cache.values() for s in sl}
    assert_lists_identical(model, want, "cached slots")
    assert len(ids) <= 2            # one layout, two slots, reused by all six calls
    mixed = h.increment_average(model, [b.astype(np.float64) for b in base], 7, total + 7)
    assert_lists_identical(mixed, ref.increment_average(model, [b.astype(np.float64) for b in base], 7, total + 7),
                           "f32 model + f64 client")


@pytest.mark.parametrize("ndev", [1, 2])
def test_staging_ingest_fortran_member_falls_back(ndev):
    """An npz whose member is Fortran-ordered cannot be inflated into the flat layout by the native
    codec; the ingest decodes it through the helper (np.load) instead, as FEDn does, and the round
    is bit-exact (no update may be skipped for the codec's sake)."""
    import io
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.helper import Helper
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(5)
    uh = MemoryUpdateHandler()
    devs = [DEV] * ndev
    st = StagingUpdateHandler(uh, helper=Helper(), device=DEV, workers=2, devices=devs if ndev > 1 else None)
    ups = []
    for k in range(4):
        w = rng.standard_normal((33, 17)).astype(np.float32)
        arrays = [np.asfortranarray(w) if k % 2 else w, rng.standard_normal(9).astype(np.float32)]
        b = io.BytesIO()
        np.savez_compressed(b, **{str(i): a for i, a in enumerate(arrays)})
        n = int(rng.integers(1, 5001))
        uh.submit_bytes(b.getvalue(), n, via=st)
        ups.append(([np.ascontiguousarray(a) for a in arrays], n))
    agg = Aggregator(st, devices=devs) if ndev > 1 else Aggregator(st)
    model, data = agg.combine_models(helper=Helper())
    st.close()
    want, nr = ref.fedavg_combine(ups)
    assert data["nr_aggregated_models"] == nr == 4
    assert_lists_identical(model, want, f"fortran x{ndev}")


# ------------------------------------------------------------------------- configs[4]: waves from host
@pytest.mark.parametrize("ndev,W,fuse", [(1, 8, True), (2, 8, True), (3, 8, True), (2, 8, False), (2, 16, True),
                                          (2, 64, False), (1, 256, True)])
def test_fedopt_bf16_waves_two_rounds(ndev, W, fuse):
    """BASELINE configs[4] shape at 1 M params: bf16 updates streamed from pinned host memory in
    waves of W (FA_PG_FIRST wave, non-final waves, the last wave with FA_PG_FINAL fused; or, with
    ``fuse`` off, a separate K = 0 FA_PG_FINAL server step; W = 256 > K: one FIRST | FINAL wave),
    FedYogi, K = 130 (a 2-update last wave at W = 8 / 16 / 64; two 64-client kernel tables in a
    W = 256 wave), two rounds with m / v carried, sliced over 1-3 devices: bit-exact to the oracle
    run on the exact f32 upcasts."""
    from fedn_amd.waves import WaveFedOpt
    P, K = 1_000_003, 130
    g = torch.Generator().manual_seed(55)
    old = torch.randn(P, generator=g).numpy()                  # round-1 global model, float32
    params = {"serveropt": "yogi", "learning_rate": 1e-2}
    wf = WaveFedOpt([DEV] * ndev, P, wave=W, fuse_final=fuse)
    state = ref.FedOptState()
    old_np = old
    for r in range(2):
        base = torch.from_numpy(np.asarray(old_np, dtype=np.float32))
        host = [(base + 0.01 * torch.randn(P, generator=g)).to(torch.bfloat16).pin_memory() for _ in range(K)]
        ns = [int(v) for v in np.random.default_rng(r).integers(1, 5001, K)]
        outs = wf.round(host, ns, wf.slices(torch.from_numpy(np.asarray(old_np))), params)
        got = wf.gather(outs).numpy()
        want, nr = ref.fedopt_combine(state, [([h.float().numpy()], n) for h, n in zip(host, ns)], [old_np], params)
        assert nr == K
        assert_lists_identical([got], want, f"round {r} x{ndev}")
        assert_lists_identical([wf.gather(wf.m).numpy()], state.m, f"round {r} m")
        assert_lists_identical([wf.gather(wf.v).numpy()], state.v, f"round {r} v")
        old_np = want[0]


@pytest.mark.parametrize("fuse", [True, False])
@pytest.mark.parametrize("opt", ["adam", "adagrad"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_fedopt_waves_dtypes_three_rounds(dtype, opt, fuse):
    """The wave path for every client dtype the kernel takes (fp32 / fp16 / bf16 updates over a
    float32 first global model, then the float64 models FEDn stores), Adam and AdaGrad, with and
    without the server step fused into the last wave; waves of 4 over K = 19 (a 3-update last wave),
    P = 100,003 (a ragged last tile), two slices, three rounds with m / v carried: the oracle's bits
    on the exact f32 upcasts of the updates."""
    from fedn_amd.waves import WaveFedOpt
    P, K = 100_003, 19
    g = torch.Generator().manual_seed(71)
    old_np = torch.randn(P, generator=g).numpy()
    params = {"serveropt": opt, "learning_rate": 1e-2}
    wf = WaveFedOpt([DEV, DEV], P, wave=4, fuse_final=fuse)
    state = ref.FedOptState()
    for r in range(3):
        base = torch.from_numpy(np.asarray(old_np, dtype=np.float32))
        host = [(base + 0.01 * torch.randn(P, generator=g)).to(dtype).pin_memory() for _ in range(K)]
        ns = [int(v) for v in np.random.default_rng(r + 7).integers(1, 5001, K)]
        outs = wf.round(host, ns, wf.slices(torch.from_numpy(np.asarray(old_np))), params)
        got = wf.gather(outs).numpy()
        ups = [([h.float().numpy() if dtype == torch.bfloat16 else h.numpy()], n) for h, n in zip(host, ns)]
        want, nr = ref.fedopt_combine(state, ups, [old_np], params)
        assert nr == K
        assert_lists_identical([got], want, f"round {r} {dtype} {opt} fuse={fuse}")
        assert_lists_identical([wf.gather(wf.m).numpy()], state.m, f"round {r} m")
        assert_lists_identical([wf.gather(wf.v).numpy()], state.v, f"round {r} v")
        old_np = want[0]


# ------------------------------------------------------------------------- N > 1 with the HIP kernel
def _hip_gloo_worker(rank, world, port, P, K, q):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    from fedn_amd.sharded import CyclicShardedFedAvg, ShardedFedAvg, ShardedFedOpt
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        g = torch.Generator(device="cuda:0").manual_seed(3)
        base = torch.randn(P, generator=g, device="cuda:0")
        ups = [torch.randn(P, generator=g, device="cuda:0").mul_(0.01).add_(base) for _ in range(K)]
        ns = [int(v) for v in np.random.default_rng(3).integers(1, 5001, K)]
        Ns = [int(v) for v in np.cumsum(ns)]
        sh = ShardedFedAvg(P)                                     # default fold: the libfedagg kernel
        agg = torch.empty(sh.hi - sh.lo, device="cuda:0")
        sh.fold(agg, [sh.local(u) for u in ups], ns, Ns, init=True)
        host = sh.gather_to_host(agg)
        cs = CyclicShardedFedAvg(P, chunk=8192)
        aggc = torch.empty(cs.local_len, device="cuda:0")
        full = cs.fold_allgather(aggc, [cs.local(u) for u in ups], ns, Ns, init=True)
        # FedOpt: each rank's slice of old / m / v on the device, the float64 model gathered to the
        # node's shared host model (HostGather) on rank 0
        so = ShardedFedOpt(P)
        out = so.step(so.local(base), [so.local(u) for u in ups], ns, Ns,
                      {"serveropt": "adam", "learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4})
        host_opt = so.gather_to_host(out)
        torch.cuda.synchronize()
        q.put((rank, None if host is None else host.numpy().copy(), full.cpu().numpy().copy(),
               None if host_opt is None else host_opt.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_sharded_gloo_world2_hip_kernel():
    """The N > 1 exchange logic (parameter slices + gather to host, and the block-cyclic fold with the
    all-gather of each round) with the HIP kernel doing every fold: 2 gloo ranks on this box's GPU,
    bit-identical to one single-device fold (RCCL refuses two ranks on one GPU)."""
    import socket

    import torch.multiprocessing as mp

    from fedn_amd import ops
    P, K, world = 200_003, 7, 2
    s_ = socket.socket()
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
    s_.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_hip_gloo_worker, args=(world, port, P, K, q), nprocs=world, join=False,
                            start_method="spawn")
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    while not pc.join(timeout=60):
        pass
    g = torch.Generator(device=DEV).manual_seed(3)
    base = torch.randn(P, generator=g, device=DEV)
    ups = [torch.randn(P, generator=g, device=DEV).mul_(0.01).add_(base) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(3).integers(1, 5001, K)]
    want = torch.empty(P, device=DEV)
    ops.fedavg_fold(want, ups, ns, [int(v) for v in np.cumsum(ns)], init=True)
    want = want.cpu().numpy()
    assert np.array_equal(res[0][1].view(np.uint32), want.view(np.uint32))
    for rank, _, full, _ in res:
        assert np.array_equal(full.view(np.uint32), want.view(np.uint32)), f"rank {rank}"
    # FedOpt gathered to the host on rank 0 (float64) == the oracle's fedopt.py round
    want_opt, _ = ref.fedopt_combine(ref.FedOptState(), [([u.cpu().numpy()], n) for u, n in zip(ups, ns)],
                                     [base.cpu().numpy()], {"serveropt": "adam"})
    assert res[0][3].dtype == np.float64 and res[1][3] is None
    assert np.array_equal(res[0][3].view(np.uint64), want_opt[0].view(np.uint64))


def _p2p_gloo_worker(rank, world, port, P, K, chunk, q, double=False, engine="dma", bf16=False):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    from fedn_amd.sharded import CyclicShardedFedAvg, P2PAllGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        g = torch.Generator(device="cuda:0").manual_seed(5)
        base = torch.randn(P, generator=g, device="cuda:0")
        ups = [torch.randn(P, generator=g, device="cuda:0").mul_(0.01).add_(base) for _ in range(K)]
        if bf16:                                      # not fusable: the "fused" engine pushes with the kernel
            ups = [u.to(torch.bfloat16) for u in ups]
        ns = [int(v) for v in np.random.default_rng(5).integers(1, 5001, K)]
        Ns = [int(v) for v in np.cumsum(ns)]
        cs = CyclicShardedFedAvg(P, chunk=chunk)
        aggc = torch.empty(cs.local_len, device="cuda:0")
        loc = [cs.local(u) for u in ups]
        full = torch.full((cs.full_len,), float("nan"), device="cuda:0")
        spare = torch.full((cs.full_len,), float("nan"), device="cuda:0") if double else None
        p2p = P2PAllGather(full, spare=spare, engine=engine)   # IPC handles of every rank's buffers, opened once
        outs = []
        for step in range(4):                         # buffers reused: entry + exit fences, or alternation
            if step >= 2:                             # later rounds of the session: other updates
                loc = [cs.local(u.add(1.0).to(u.dtype)) for u in ups]
            out = cs.fold_allgather(aggc, loc, ns, Ns, init=True, p2p=p2p)
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy().copy())
        # a continuation (init=False) folds onto the running aggregate agg_local, and agg_local holds
        # this rank's folded chunks afterwards (gather_to_host copies it), whatever the engine
        out = cs.fold_allgather(aggc, loc, ns, [x + Ns[-1] for x in Ns], init=False, p2p=p2p)
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy().copy())
        host = cs.gather_to_host(aggc)
        outs.append(None if host is None else host.numpy().copy())
        rel = p2p.check_release()
        p2p.close()
        q.put((rank, outs, rel))
    finally:
        dist.destroy_process_group()


def _check_p2p_results(res, want, want2, want3, engine=None):
    """Steps 0-3 (init, other updates from step 2), the continuation step (init=False, step 4) and
    rank 0's host model gathered from agg_local (step 5); the release grids covered every XCD."""
    want, want2, want3 = (w.cpu().numpy() for w in (want, want2, want3))
    for rank, outs, rel in res:
        for step, got in enumerate(outs[:5]):
            w = want3 if step == 4 else (want2 if step >= 2 else want)
            assert np.array_equal(got.view(np.uint32), w.view(np.uint32)), f"rank {rank} step {step}"
        if rank == 0:
            assert np.array_equal(outs[5].view(np.uint32), want3.view(np.uint32)), "gather_to_host(agg_local)"
        else:
            assert outs[5] is None
        assert rel["misses"] == 0
        if engine in ("kernel", "fused"):
            assert rel["launches"] > 0 and rel["misses"] == 0 and rel["seen_mask"] == rel["expect_mask"]


def test_p2p_allgather_fused_engine_bf16_falls_back():
    """The fused engine applies to fp32 updates; bf16 updates fold with the regular kernel and push
    with the push kernel — still bit-identical to one single-device fold (2 processes, one GPU)."""
    import socket

    import torch.multiprocessing as mp

    from fedn_amd import ops
    P, K, world, chunk = 200_003, 9, 2, 8192
    s_ = socket.socket()
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
    s_.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_p2p_gloo_worker, args=(world, port, P, K, chunk, q, True, "fused", True), nprocs=world,
                            join=False, start_method="spawn")
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    while not pc.join(timeout=60):
        pass
    g = torch.Generator(device=DEV).manual_seed(5)
    base = torch.randn(P, generator=g, device=DEV)
    ups = [torch.randn(P, generator=g, device=DEV).mul_(0.01).add_(base).to(torch.bfloat16) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(5).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    want = torch.empty(P, device=DEV)
    ops.fedavg_fold(want, ups, ns, Ns, init=True)
    want2 = torch.empty(P, device=DEV)
    ops.fedavg_fold(want2, [u.add(1.0).to(torch.bfloat16) for u in ups], ns, Ns, init=True)
    want3 = want2.clone()
    ops.fedavg_fold(want3, [u.add(1.0).to(torch.bfloat16) for u in ups], ns, [x + Ns[-1] for x in Ns], init=False)
    _check_p2p_results(res, want, want2, want3)


@pytest.mark.parametrize("engine", ["dma", "kernel", "fused"])
@pytest.mark.parametrize("world,P,chunk,double", [(2, 200_003, 8192, False), (3, 1_000_000, 65536, False),
                                                  (2, 200_003, 8192, True), (3, 1_000_000, 65536, True)])
def test_p2p_allgather_gloo_hip(world, P, chunk, double, engine):
    """The direct peer-to-peer all-gather (sharded.P2PAllGather: IPC handles exchanged once,
    pieces pushed into every peer's buffer — fa_copy_async on one copy stream per peer, or one
    fa_push kernel per piece — entry / exit fences) with the HIP fold: ranks share this box's GPU
    (each maps the others' buffers through IPC), four steps, every rank's whole model bit-identical
    to one single-device fold."""
    import socket

    import torch.multiprocessing as mp

    from fedn_amd import ops
    K = 9
    s_ = socket.socket()
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
    s_.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_p2p_gloo_worker, args=(world, port, P, K, chunk, q, double, engine), nprocs=world,
                            join=False, start_method="spawn")
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    while not pc.join(timeout=60):
        pass
    g = torch.Generator(device=DEV).manual_seed(5)
    base = torch.randn(P, generator=g, device=DEV)
    ups = [torch.randn(P, generator=g, device=DEV).mul_(0.01).add_(base) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(5).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    want = torch.empty(P, device=DEV)
    ops.fedavg_fold(want, ups, ns, Ns, init=True)
    want2 = torch.empty(P, device=DEV)
    ops.fedavg_fold(want2, [u.add(1.0) for u in ups], ns, Ns, init=True)
    want3 = want2.clone()
    ops.fedavg_fold(want3, [u.add(1.0) for u in ups], ns, [x + Ns[-1] for x in Ns], init=False)
    _check_p2p_results(res, want, want2, want3, engine)


@pytest.mark.parametrize("K", [1, 3, 9, 64, 70])
@pytest.mark.parametrize("P,ndst", [(1, 1), (4099, 0), (4099, 3), (1_000_003, 7)])
def test_fedavg_fold_push(K, P, ndst):
    """fa_fedavg_fold_push: the fold written to agg AND to every destination, bit-identical to
    fa_fedavg_fold (clients beyond one 64-entry table folded first, the last table pushes; a ragged
    last strip); init and continuation; misaligned addresses refused."""
    from fedn_amd import ops
    from fedn_amd._abi import FedAggError
    g = torch.Generator(device=DEV).manual_seed(K * 7 + ndst)
    base = torch.randn(P, generator=g, device=DEV)
    ups = [torch.randn(P, generator=g, device=DEV).mul_(0.01).add_(base) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(K).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    want = torch.empty(P, device=DEV)
    ops.fedavg_fold(want, ups, ns, Ns, init=True)
    agg = torch.full((P + 64,), float("nan"), device=DEV)
    dsts = [torch.full((P + 64,), float("nan"), device=DEV) for _ in range(ndst)]
    st = torch.cuda.current_stream(DEV)
    ops.fedavg_fold_push(agg.data_ptr(), [u.data_ptr() for u in ups], ns, Ns, P, True, [d.data_ptr() for d in dsts],
                         st, DEV)
    torch.cuda.synchronize()
    for t in [agg] + dsts:
        assert torch.equal(t[:P].view(torch.int32), want.view(torch.int32))
        assert bool(torch.isnan(t[P:]).all())
    # continuation (init=False): fold the same clients again onto the result, as fa_fedavg_fold does
    want2 = want.clone()
    ops.fedavg_fold(want2, ups, ns, [x + Ns[-1] for x in Ns], init=False)
    ops.fedavg_fold_push(agg.data_ptr(), [u.data_ptr() for u in ups], ns, [x + Ns[-1] for x in Ns], P, False,
                         [d.data_ptr() for d in dsts], st, DEV)
    torch.cuda.synchronize()
    for t in [agg] + dsts:
        assert torch.equal(t[:P].view(torch.int32), want2.view(torch.int32))
    if P > 1:
        with pytest.raises(FedAggError, match="aligned"):
            ops.fedavg_fold_push(agg.data_ptr() + 4, [u.data_ptr() for u in ups], ns, Ns, P - 1, True, [], st, DEV)
        with pytest.raises(FedAggError, match="aligned"):
            ops.fedavg_fold_push(agg.data_ptr(), [u.data_ptr() for u in ups], ns, Ns, P, True, [agg.data_ptr() + 8],
                                 st, DEV)


@pytest.mark.parametrize("nbytes", [16, 4004, 1 << 20, (64 << 20) + 12])
@pytest.mark.parametrize("ndst", [1, 3, 7])
def test_push_kernel(nbytes, ndst):
    """fa_push: the source's bytes land in every destination exactly (16-B words plus a ragged
    tail), nothing past the end is written; misaligned pointers and too many destinations refused."""
    from fedn_amd import ops
    from fedn_amd._abi import FedAggError
    g = torch.Generator(device=DEV).manual_seed(nbytes + ndst)
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=DEV, generator=g)
    dsts = [torch.full((nbytes + 64,), 0xA5, dtype=torch.uint8, device=DEV) for _ in range(ndst)]
    st = torch.cuda.current_stream(DEV)
    ops.push([d.data_ptr() for d in dsts], src, nbytes, st)
    torch.cuda.synchronize()
    for d in dsts:
        assert torch.equal(d[:nbytes], src)
        assert bool((d[nbytes:] == 0xA5).all())
    with pytest.raises(FedAggError, match="aligned"):
        ops.push([dsts[0].data_ptr() + 4], src, 16, st)
    with pytest.raises(FedAggError, match="destinations"):
        ops.push([dsts[0].data_ptr()] * 17, src, 16, st)


@pytest.mark.parametrize("engine", ["dma", "kernel"])
@pytest.mark.parametrize("ndev,P", [(2, 300_001), (3, 1 << 20)])
def test_allgather_devices_in_process(ndev, P, engine):
    """multidev.allgather_devices (the in-process form of the direct all-gather: fa_peer_enable +
    fa_copy_async per (source, destination) pair on its own stream): each "device" (this box's GPU
    listed ndev times) folds its slice with the HIP kernel, every device ends with the whole model,
    bit-identical to the oracle."""
    from fedn_amd import ops
    from fedn_amd.multidev import allgather_devices
    from fedn_amd.sharded import shard_bounds
    rng = np.random.default_rng(9)
    K = 5
    base = rng.standard_normal(P).astype(np.float32)
    ups = [(base + 0.01 * rng.standard_normal(P)).astype(np.float32) for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    parts = []
    for lo, hi in shard_bounds(P, ndev):
        agg = torch.empty(hi - lo, device=DEV)
        ops.fedavg_fold(agg, [torch.from_numpy(u[lo:hi]).to(DEV) for u in ups], ns, Ns, init=True)
        parts.append((DEV, agg, lo))
    fulls = allgather_devices(parts, P, engine=engine)
    want = ref.fedavg_flat(ups, ns)
    assert len(fulls) == ndev
    for d, f in enumerate(fulls):
        assert np.array_equal(f.cpu().numpy().view(np.uint32), want.view(np.uint32)), f"device entry {d}"


def test_waves_reject_mismatched_updates():
    """WaveFedOpt refuses updates whose dtype / size differ from the first (a copy into the bf16
    wave slots would otherwise round an fp32 update silently) and misplaced old slices."""
    from fedn_amd.waves import WaveFedOpt
    P = 10_000
    wf = WaveFedOpt([DEV, DEV], P, wave=4)
    old = wf.slices(torch.zeros(P, dtype=torch.float64))
    ups = [torch.zeros(P, dtype=torch.bfloat16) for _ in range(3)]
    with pytest.raises(ValueError, match="update 2"):
        wf.round(ups[:2] + [torch.zeros(P)], [1, 2, 3], old, {})
    with pytest.raises(ValueError, match="update 1"):
        wf.round([ups[0], torch.zeros(P - 1, dtype=torch.bfloat16)], [1, 2], old, {})
    with pytest.raises(ValueError, match="num_examples"):
        wf.round(ups, [1, 2], old, {})
    with pytest.raises(ValueError, match="old"):
        wf.round(ups, [1, 2, 3], [o.cpu() for o in old], {})
    assert len(wf.round(ups, [1, 2, 3], old, {"serveropt": "yogi"})) == 2


@pytest.mark.parametrize("kind", ["fedavg", "fedopt"])
def test_small_host_updates_arena_batches(kind):
    """Host updates of <= SMALL_UPDATE_BYTES fold in arena batches: K = 70 updates of a ~1.6 MB
    two-group model (arena capacity 40 -> flushes at 40 and at the end, both arenas reused)
    through the plug-in, two rounds, bit-exact to the oracle."""
    from fedn_amd import staging
    rng = np.random.default_rng(21)
    shapes = [(300, 1000), (1000,), (7, 3)]
    base = [rng.standard_normal(shapes[0]).astype(np.float32), rng.standard_normal(shapes[1]).astype(np.float32),
            rng.integers(-100, 100, shapes[2]).astype(np.int64)]
    nbytes = sum(a.nbytes for a in base)
    assert nbytes <= staging.SMALL_UPDATE_BYTES and staging.ARENA_BYTES // nbytes < 64
    K = 70
    ups = [[(base[0] + 0.01 * rng.standard_normal(shapes[0])).astype(np.float32),
            (base[1] + 0.01 * rng.standard_normal(shapes[1])).astype(np.float32),
            rng.integers(-100, 100, shapes[2]).astype(np.int64)] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    uh, agg = _plugin(kind)
    params = {"serveropt": "yogi", "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
    st = ref.FedOptState()
    old = [b.astype(np.float32) for b in base[:2]]
    if kind == "fedopt":
        ups = [u[:2] for u in ups]
    for r in range(2):
        gid = uh.put_global_model(old, f"g{r}") if kind == "fedopt" else "global"
        for a, n in zip(ups, ns):
            uh.submit(a, n, model_id=gid)
        model, data = agg.combine_models(helper=None, delete_models=True,
                                         parameters=params if kind == "fedopt" else None)
        if kind == "fedavg":
            want, nr = ref.fedavg_combine(list(zip(ups, ns)))
        else:
            want, nr = ref.fedopt_combine(st, list(zip(ups, ns)), old, params)
            old = want
        assert data["nr_aggregated_models"] == nr == K
        assert_lists_identical(model, want, f"{kind} round {r}")


@pytest.mark.parametrize("kind", ["fedavg", "fedopt"])
def test_small_float_updates_native_admission(kind):
    """Float-only small models are admitted and packed by the native call (layout.fast_admission,
    csrc/fastpack.c). K = 70 mnist-shaped updates (the arena flushes at 64) with updates the native
    test must refuse mixed in: a Fortran-ordered tensor and a tuple (same layout: the Python pack),
    a float64 tensor late in the round (numpy promotion: the per-tensor path). Two rounds through the
    plug-in, bit-exact to the oracle, every update counted."""
    from fedn_amd import layout as L
    assert L._fast(), "the _fastpack extension is not built"
    rng = np.random.default_rng(33)
    shapes = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]
    base = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    K = 70
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
    ups[5] = [np.asfortranarray(ups[5][0])] + ups[5][1:]
    ups[9] = tuple(ups[9])
    ups[66] = [ups[66][0].astype(np.float64)] + ups[66][1:]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    uh, agg = _plugin(kind)
    params = {"serveropt": "adam", "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
    st = ref.FedOptState()
    old = base
    for r in range(2):
        gid = uh.put_global_model(old, f"g{r}") if kind == "fedopt" else "global"
        for a, n in zip(ups, ns):
            uh.submit(a, n, model_id=gid)
        model, data = agg.combine_models(helper=None, delete_models=True,
                                         parameters=params if kind == "fedopt" else None)
        if kind == "fedavg":
            want, nr = ref.fedavg_combine(list(zip(ups, ns)))
        else:
            want, nr = ref.fedopt_combine(st, list(zip(ups, ns)), old, params)
            old = want
        assert data["nr_aggregated_models"] == nr == K
        assert_lists_identical(model, want, f"{kind} round {r}")


@pytest.mark.parametrize("K", [2, 5, 15, 16, 40])
def test_small_round_zero_copy(K, monkeypatch):
    """A small FedAvg round whose updates never left the pinned arena folds straight from it into the
    pinned result block (staging.ZERO_COPY_BYTES: no H2D / D2H) — since round 6 through the one-call
    round (smallround.py) while the round fits its arena (19 mnist updates in 4 MiB), through the
    general pipeline's arena beyond. Bit-exact to the oracle and to the copy path (forced with
    ZERO_COPY_BYTES = 0), three rounds of one session; the zero-copy rounds enqueue no H2D
    (time_h2d == 0), larger rounds (partial uploads from 16 updates on) copy as before."""
    from fedn_amd import staging
    rng = np.random.default_rng(40 + K)
    shapes = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]
    base = [rng.standard_normal(sh).astype(np.float32) for sh in shapes]
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    want, nr = ref.fedavg_combine(list(zip(ups, ns)))
    for zc in (True, False):
        monkeypatch.setattr(staging, "ZERO_COPY_BYTES", (4 << 20) if zc else 0)
        uh, agg = _plugin("fedavg")
        for r in range(3):
            for a, n in zip(ups, ns):
                uh.submit(a, n)
            model, data = agg.combine_models(helper=None, delete_models=True)
            assert data["nr_aggregated_models"] == nr == K
            assert_lists_identical(model, want, f"K={K} zero_copy={zc} round {r}")
            zero = zc and K <= staging.ZERO_COPY_BYTES // 210_688     # the one-call round's arena
            assert (data["time_h2d"] == 0) == zero, data


@pytest.mark.parametrize("opt", ["adam", "yogi", "adagrad"])
@pytest.mark.parametrize("K", [1, 3, 15, 40])
def test_small_fedopt_zero_copy(K, opt, monkeypatch):
    """A small FedOpt round whose updates never left the pinned arena runs its fused FIRST + FINAL
    step zero-copy (clients and global model read from pinned memory, the new model written into the
    caller's pinned block; m / v in HBM). Three rounds of one session (m / v carried, the global model
    the previous round's float64 output), bit-exact to the oracle and to the copy path."""
    from fedn_amd import staging
    rng = np.random.default_rng(60 + K)
    shapes = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]
    base = [rng.standard_normal(sh).astype(np.float32) for sh in shapes]
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    params = {"serveropt": opt, "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
    for zc in (True, False):
        monkeypatch.setattr(staging, "ZERO_COPY_BYTES", (4 << 20) if zc else 0)
        uh, agg = _plugin("fedopt")
        st, old = ref.FedOptState(), base
        for r in range(3):
            gid = uh.put_global_model(old, f"g{r}")
            for a, n in zip(ups, ns):
                uh.submit(a, n, model_id=gid)
            model, data = agg.combine_models(helper=None, delete_models=True, parameters=params)
            want, nr = ref.fedopt_combine(st, list(zip(ups, ns)), old, params)
            assert data["nr_aggregated_models"] == nr == K
            assert_lists_identical(model, want, f"K={K} {opt} zero_copy={zc} round {r}")
            zero = zc and K < staging.ARENA_UPLOAD_EVERY
            assert (data["time_h2d"] == 0) == zero, data
            old = model


@pytest.mark.parametrize("K,staged_at,mixed_last", [(1, (), False), (2, (), False), (3, (), False),
                                                     (5, (), False), (5, (2,), False), (4, (3,), False),
                                                     (4, (), True)])
def test_large_host_updates_piecewise_staging(K, staged_at, mixed_last):
    """Updates >= STAGE_PIECES_MIN are packed and uploaded piece by piece and folded on arrival one
    launch per piece (each behind its own H2D piece); after the round's last such update the
    result's D2H chunks wait only for the fold chunks they read. Two groups (a ~17 M fp32 group,
    ragged, and a small fp64 one); staged (device-resident) updates interleaved keep FIFO order; a
    last update of another dtype moves the round to the per-tensor path. Bit-exact to the oracle,
    two rounds."""
    from fedn_amd import staging
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    rng = np.random.default_rng(70 + K)
    shapes = [(4099, 4099), (777,), (1001,)]
    dtypes = [np.float32, np.float32, np.float64]
    base = [rng.standard_normal(sh).astype(d) for sh, d in zip(shapes, dtypes)]
    nbytes = sum(b.nbytes for b in base)
    assert nbytes >= staging.STAGE_PIECES_MIN and nbytes % staging.STAGE_PIECE
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(b.dtype) for b in base] for _ in range(K)]
    if mixed_last:
        ups[-1] = [ups[-1][0].astype(np.float64)] + ups[-1][1:]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    want, nr = ref.fedavg_combine(list(zip(ups, ns)))
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, device=DEV, workers=2)
    agg = get_aggregator("fedavg", st)
    try:
        for r in range(2):
            for k, (a, n) in enumerate(zip(ups, ns)):
                uh.submit(a, n, via=st if k in staged_at else None)
            model, data = agg.combine_models(helper=None, delete_models=True)
            assert data["nr_aggregated_models"] == nr == K
            assert_lists_identical(model, want, f"K={K} staged_at={staged_at} mixed_last={mixed_last} round {r}")
    finally:
        st.close()


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("K,P", [(3, 1), (64, 4099), (130, 8192 * 3 + 7), (9, 100_003)])
def test_fedavg_pipelined_geometry_forced_small(dt, K, P):
    """The product folds client buffers under 160 MiB with the 1-strip kernel and larger ones with
    the pipelined 4-strip kernel (bf16: 8 strips of 4). The probe library forces the pipelined
    geometry at small sizes so its whole tiles, ragged tile and K > 64 continuation stay covered
    against the oracle; both geometries must give the same bits."""
    from fedn_amd import _abi, ops
    rng = np.random.default_rng(K + P)
    ups, ns = _updates(rng, K, P)
    if dt == "bf16":
        dev = [torch.from_numpy(u).to(torch.bfloat16).to(DEV) for u in ups]
        ups = [d.to(torch.float32).cpu().numpy() for d in dev]
    else:
        dev = [_to_dev(u) for u in ups]
    want = ref.fedavg_flat(ups, ns)
    auto = _fold_dev(dev, ns, torch.float32)
    with _abi.use_probe():
        ops.tune(auto_geom=0)
        try:
            forced = _fold_dev(dev, ns, torch.float32)
        finally:
            ops.tune(auto_geom=1)
    assert_lists_identical([auto], [want], f"{dt} auto")
    assert_lists_identical([forced], [want], f"{dt} pipelined")


@pytest.mark.parametrize("threshold,sliced", [(64 << 20, False), (1000, True)])
def test_multidevice_size_rule(monkeypatch, threshold, sliced):
    """FEDN_AMD_DEVICES slices a model over the GPUs only when it is at least MULTIDEV_MIN_BYTES
    packed; smaller models stay on the first GPU — in the ingest and in both aggregators alike.
    FedAvg and FedOpt (two rounds) through the ingest, bit-exact either way."""
    from fedn_amd import layout, staging
    from fedn_amd.aggregators.fedavg import Aggregator as FedAvg, make_fedavg_pipeline
    from fedn_amd.aggregators.fedopt import Aggregator as FedOpt
    from fedn_amd.ingest import ShardedStagedModel, StagedModel, StagingUpdateHandler
    from fedn_amd.multidev import ShardedFedAvgPipeline
    from fedn_amd.updatehandler import MemoryUpdateHandler
    monkeypatch.setattr(layout, "MULTIDEV_MIN_BYTES", threshold)
    devs = [DEV, DEV, DEV]
    case = load_case("fedavg_odd_k8")
    rd = case["rounds"][0]
    assert isinstance(make_fedavg_pipeline(rd["updates"][0][0], devices=devs),
                      ShardedFedAvgPipeline if sliced else staging.FedAvgPipeline)
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, devices=devs, workers=2)
    for arrays, n in rd["updates"]:
        uh.submit(arrays, n, via=st)
    staged = [st._staged[k].result()[0] for k in list(st._staged)]
    assert all(isinstance(x, ShardedStagedModel if sliced else StagedModel) for x in staged)
    model, data = FedAvg(st, devices=devs).combine_models(helper=None)
    assert_lists_identical(model, rd["out"], "fedavg size rule")
    case = load_case("fedopt_adam_3r")
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, devices=devs, workers=2)
    agg = FedOpt(st, devices=devs)
    for r, rd in enumerate(case["rounds"][:2]):
        gid = uh.put_global_model(rd["old"], f"g{r}")
        for arrays, n in rd["updates"]:
            uh.submit(arrays, n, model_id=gid, via=st)
        model, data = agg.combine_models(helper=None, parameters=case["params"])
        assert_lists_identical(model, rd["out"], f"fedopt size rule round {r}")
    assert agg.sharded is sliced
    st.close()
