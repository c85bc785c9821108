"""Host-side logic of the plug-ins that needs no GPU: layout, parameters, loader, empty rounds."""
import numpy as np
import pytest
import torch

from fedn_amd import ops
from fedn_amd.aggregators import get_aggregator
from fedn_amd.exceptions import InvalidParameterError
from fedn_amd.layout import ALIGN, Layout
from fedn_amd.parameters import Parameters
from fedn_amd.updatehandler import MemoryUpdateHandler


def test_layout_groups_alignment_roundtrip():
    rng = np.random.default_rng(0)
    arrays = [rng.standard_normal((3, 5)).astype(np.float32), np.arange(7, dtype=np.int64),
              rng.standard_normal(11).astype(np.float32), np.float32(2.5) * np.ones((), np.float32),
              rng.standard_normal((2, 2)).astype(np.float64)]
    lay = Layout.of(arrays)
    assert [str(d) for d in lay.groups] == ["float32", "int64", "float64"]
    for dt in lay.groups:
        assert lay.group_byte_offset[dt] % ALIGN == 0
    assert lay.group_elems[np.dtype(np.float32)] == 15 + 11 + 1
    buf = np.zeros(lay.nbytes, np.uint8)
    lay.pack(arrays, buf)
    out = [None] * len(arrays)
    for dt in lay.groups:
        lay.unpack_group(lay.group_view(buf, dt), dt, out)
    for a, b in zip(arrays, out):
        assert a.dtype == b.dtype and a.shape == b.shape
        np.testing.assert_array_equal(a, b)


def test_layout_check_mismatch():
    lay = Layout.of([np.zeros((3,), np.float32)])
    with pytest.raises(ValueError):
        lay.check([np.zeros((4,), np.float32)])
    with pytest.raises(ValueError):
        lay.check([np.zeros((3,), np.float32)] * 2)
    with pytest.raises(TypeError):
        lay.check([np.zeros((3,), np.float64)])


def test_parameters_validate_mirror():
    schema = {"serveropt": str, "learning_rate": float}
    assert Parameters({"serveropt": "adam", "learning_rate": 0.1}).validate(schema)
    with pytest.raises(InvalidParameterError):
        Parameters({"learning_rate": 1}).validate(schema)     # int rejected, like FEDn
    with pytest.raises(InvalidParameterError):
        Parameters({"momentum": 0.1}).validate(schema)
    assert not issubclass(InvalidParameterError, Exception)   # BaseException, fedn/common/exceptions.py:9


def test_result_dtype_rules():
    f32, f64, f16, bf, i64 = torch.float32, torch.float64, torch.float16, torch.bfloat16, torch.int64
    assert ops.fold_result_dtype(f32, f32) == f32
    assert ops.fold_result_dtype(f32, f64) == f64
    assert ops.fold_result_dtype(f16, f16) == f16
    assert ops.fold_result_dtype(f32, bf) == f32
    assert ops.fold_result_dtype(i64, i64) == f64
    assert ops.fedopt_dtypes(f32, f32, None) == (f32, f32)
    assert ops.fedopt_dtypes(f32, f64, f32) == (f64, f64)
    assert ops.fedopt_dtypes(bf, f32, None) == (f32, f32)


@pytest.mark.parametrize("name", ["fedavg", "fedopt"])
def test_get_aggregator_and_empty_round(name):
    uh = MemoryUpdateHandler()
    agg = get_aggregator(name, uh)
    assert agg.name == name and agg.update_handler is uh
    model, data = agg.combine_models(helper=None, delete_models=True, parameters=None)
    assert model is None
    assert data["nr_aggregated_models"] == 0
    assert data["time_model_load"] == 0.0 and data["time_model_aggregation"] == 0.0


@pytest.mark.parametrize("params", [{"learning_rate": 1}, {"momentum": 0.5}])
def test_fedopt_bad_parameters_leave_queue(params):
    """fedopt.py:62-66: invalid kwargs -> (None, data) before the queue is touched."""
    uh = MemoryUpdateHandler()
    uh.submit([np.zeros(3, np.float32)], 10)
    model, data = get_aggregator("fedopt", uh).combine_models(parameters=params)
    assert model is None and "nr_aggregated_models" not in data
    assert uh.model_updates.qsize() == 1


def test_update_handler_rejects_missing_metadata():
    from fedn_amd.updatehandler import ModelUpdate
    uh = MemoryUpdateHandler()
    assert not uh.on_model_update(ModelUpdate("g", "u", '{"training_metadata": {}}'))
    assert uh.model_updates.empty()


@pytest.mark.parametrize("workers", [1, 4])
def test_reduce_load_error_propagates_in_order(workers):
    """Control.reduce (control.py:674-690): a model whose decode raises is decoded again in the
    except branch, which raises out of reduce — after the earlier combiners' deletions and
    before any later one, also when later models were already decoded ahead."""
    from fedn_amd.reduce import reduce_models
    calls = []

    def load(data):
        calls.append(data)
        raise ValueError(f"cannot decode {data}")

    deleted = []
    combiners = [{"name": f"c{c}", "model_id": f"m{c}"} for c in range(5)]
    fetch = {"m1": "b1", "m2": "b2", "m3": "b3", "m4": "b4"}.__getitem__     # m0 missing
    with pytest.raises(ValueError, match="cannot decode b1"):
        reduce_models(combiners, fetch=fetch, load=load, delete=deleted.append, workers=workers)
    assert deleted == ["m0"]
    assert calls.count("b1") == 2


@pytest.mark.parametrize("ahead", [1, 3, 8])
def test_queued_updates_fifo_errors_and_late_arrivals(ahead):
    """aggregatorbase.queued_updates: FIFO order, a failing load raises from its own load()
    (the caller skips it), and updates enqueued while the round drains are consumed too."""
    from fedn_amd.aggregators.aggregatorbase import queued_updates
    uh = MemoryUpdateHandler()
    for k in range(5):
        uh.submit([np.full(3, k, np.float32)], k + 1)
    uh.store.models[list(uh.store.models)[2]] = None          # update 2 cannot be loaded
    seen, errors = [], 0
    for i, (mu, load) in enumerate(queued_updates(uh, None, ahead=ahead)):
        try:
            arrays, meta = load()
            seen.append((int(arrays[0][0]), meta["num_examples"]))
        except RuntimeError:
            errors += 1
        if i == 1:
            uh.submit([np.full(3, 9, np.float32)], 10)          # arrives mid-round
    assert seen == [(0, 1), (1, 2), (3, 4), (4, 5), (9, 10)] and errors == 1
    assert uh.model_updates.empty()


class _Abort(BaseException):
    """Escapes the aggregators' per-update ``except Exception`` (like InvalidParameterError)."""


def _ids(q):
    return [mu.model_update_id for mu in list(q.queue)]


@pytest.mark.parametrize("ahead", [1, 3, 8])
@pytest.mark.parametrize("where", ["body", "load"])
def test_queued_updates_lossless_on_abort(ahead, where):
    """An exception that escapes the caller's per-update handling mid-round — raised by the loop
    body, or by load_model_update itself (a BaseException travels out of the worker's future) —
    leaves exactly what FEDn's sequential loop leaves queued (fedavg.py:47-78): every update after
    the one being processed, in FIFO order; the read-ahead puts back what it dequeued early."""
    import contextlib

    from fedn_amd.aggregators.aggregatorbase import queued_updates
    uh = MemoryUpdateHandler()
    for k in range(10):
        uh.submit([np.full(3, k, np.float32)], k + 1)
    order = _ids(uh.model_updates)
    if where == "load":
        inner = uh.load_model_update

        def load_model_update(mu, helper):
            if mu.model_update_id == order[3]:
                raise _Abort()
            return inner(mu, helper)
        uh.load_model_update = load_model_update
    got = []
    with pytest.raises(_Abort):
        with contextlib.closing(queued_updates(uh, None, ahead=ahead)) as it:
            for mu, load in it:
                arrays, _ = load()
                got.append(int(arrays[0][0]))
                if where == "body" and len(got) == 4:
                    raise _Abort()
    assert _ids(uh.model_updates) == order[4:]          # update 3 was being processed: consumed
    assert got == [0, 1, 2, 3] if where == "body" else got == [0, 1, 2]


def test_queued_updates_byte_cap():
    """Once one decoded update's size is known, the read-ahead holds at most ahead_bytes of
    decoded updates (at least one), whatever ``ahead`` says."""
    import threading

    from fedn_amd.aggregators.aggregatorbase import queued_updates
    uh = MemoryUpdateHandler()
    for k in range(12):
        uh.submit([np.full(250, k, np.float32)], 1)          # 1000 bytes per update
    started, lock = [], threading.Lock()
    inner = uh.load_model_update

    def load_model_update(mu, helper):
        with lock:
            started.append(mu.model_update_id)
        return inner(mu, helper)
    uh.load_model_update = load_model_update
    consumed = 0
    for mu, load in queued_updates(uh, None, ahead=8, ahead_bytes=2500):
        load()
        consumed += 1
        # the budget holds 2 decoded updates, counting the one being folded: at most one more started
        assert len(started) <= consumed + 1
    assert consumed == 12


def test_queued_updates_staged_models_read_ahead(monkeypatch):
    """Updates that are staged objects (a ``layout`` with ``nbytes``, like ingest.StagedModel) size
    the read-ahead by their packed layout, so it opens past one update; no polling wait happens when
    no npz size peek is pending (a handler without load_model_update_byte): the drain's Event is
    never waited on."""
    import threading
    import types

    from fedn_amd.aggregators import aggregatorbase
    from fedn_amd.aggregators.aggregatorbase import model_nbytes, queued_updates
    waits = []

    class CountingEvent(threading.Event):
        def wait(self, timeout=None):
            waits.append(timeout)
            return super().wait(timeout)

    monkeypatch.setattr(aggregatorbase, "threading", types.SimpleNamespace(Event=CountingEvent))
    staged = lambda k: types.SimpleNamespace(layout=types.SimpleNamespace(nbytes=1000), k=k)  # noqa: E731
    assert model_nbytes(staged(0)) == 1000
    assert model_nbytes([np.zeros(10, np.float32)]) == 40
    uh = MemoryUpdateHandler()
    for k in range(40):
        uh.submit([np.zeros(1, np.float32)], 1)
    inner = uh.load_model_update
    # the UpdateHandler surface WITHOUT load_model_update_byte: no npz size peek can be issued
    h = types.SimpleNamespace(model_updates=uh.model_updates, next_model_update=uh.next_model_update,
                              delete_model=uh.delete_model,
                              load_model_update=lambda mu, helper: (staged(mu.model_update_id), inner(mu, helper)[1]))
    ahead_seen = []
    for mu, load in queued_updates(h, None, ahead=8, ahead_bytes=1 << 30):
        load()
        ahead_seen.append(40 - 1 - len(ahead_seen) - uh.model_updates.qsize())
    assert len(ahead_seen) == 40
    assert max(ahead_seen) > 1                      # read-ahead opened past one update
    assert waits == []                              # no size peek pending: never polled


def test_reduce_byte_cap_keeps_order():
    """reduce_models with a byte budget smaller than one model still folds in combiner order."""
    import fedn_amd.reduce as red
    seen = []

    class Pipe:
        def __init__(self, dev, m, batch=True):
            seen.append(("first", int(m[0][0])))

        def add(self, m, n, N):
            seen.append((int(m[0][0]), N))

        def result(self):
            return "ok"
    saved = red.FedAvgPipeline, red.LOAD_AHEAD_BYTES
    red.FedAvgPipeline, red.LOAD_AHEAD_BYTES = Pipe, 10
    try:
        combiners = [{"name": f"c{c}", "model_id": c} for c in range(6)]
        model, _ = red.reduce_models(combiners, fetch=lambda c: c, load=lambda c: [np.full(100, c, np.float32)],
                                     device="cpu", workers=4)
    finally:
        red.FedAvgPipeline, red.LOAD_AHEAD_BYTES = saved
    assert model == "ok"
    assert seen == [("first", 0), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6)]


def test_mixed_fold_plan_is_numpy():
    """mixed.fold_plan / sub_plan infer numpy's result dtypes and shapes (numpyhelper.py:32, :44)
    from metadata alone, and raise where numpy raises."""
    from fedn_amd import mixed
    f4, f8, i4, i8, f2 = (np.dtype(t) for t in (np.float32, np.float64, np.int32, np.int64, np.float16))
    cases = [((f4, (7,)), (f8, (7,))), ((i8, (3,)), (f4, (3,))), ((f2, (2, 1)), (f4, (1, 5))),
             ((i4, ()), (i8, (4,))), ((f8, (1,)), (i4, (6,)))]
    for (xd, xs), (yd, ys) in cases:
        (d, r, shape), = mixed.fold_plan([(xs, xd)], [(ys, yd)], 37, 1234)
        x, y = np.ones(xs, xd), np.ones(ys, yd)
        want = np.add(x, 37 * (y - x) / 1234)
        assert (r, shape) == (want.dtype, want.shape) and d == (y - x).dtype
    with pytest.raises(ValueError):
        mixed.fold_plan([((5,), f4)], [((4,), f4)], 1, 2)
    assert len(mixed.fold_plan([((1,), f4)] * 3, [((1,), f4)] * 2, 1, 2)) == 2       # zip truncates
    (d, r, shape), = mixed.fold_plan([((3,), i8)], [((3,), i8)], 2.5, 4)             # int diff, float n
    assert (d, r) == (i8, np.add(np.ones(3, i8), 2.5 * (np.ones(3, i8) - np.ones(3, i8)) / 4).dtype)
    assert mixed.float_n(2.5) and not mixed.float_n(3) and not mixed.float_n(1.0) and not mixed.float_n(np.int64(2))
    assert mixed.int_float_n([i8, f4], 0, 2.5) and not mixed.int_float_n([i8], 1, 2.5)
    assert not mixed.int_float_n([f4, f8], 0, 2.5) and not mixed.int_float_n([i8], 0, 4)
    (r, shape), = mixed.sub_plan([((3,), i8)], [((1,), f4)])
    assert r == (np.ones(3, i8) * 1.0 + np.ones(1, f4) * -1.0).dtype and shape == (3,)


def test_reduce_admits_by_npz_directory_size():
    """reduce_models learns a model's decoded size from the first payload's zip directory, so
    the other decodes start at once (not after the first decode), and never more are in flight
    than the byte budget allows (the model being waited for included)."""
    import io
    import threading
    import time

    import fedn_amd.reduce as red

    class Pipe:
        def __init__(self, dev, m, batch=True):
            pass

        def add(self, m, n, N):
            pass

        def result(self):
            return "ok"

    repo = {}
    for c in range(6):
        b = io.BytesIO()
        np.savez_compressed(b, **{"0": np.zeros(250_000, np.float32)})      # 1 MB decoded
        repo[c] = b.getvalue()
    assert red.npz_decoded_bytes(repo[0]) >= 1_000_000
    assert red.npz_decoded_bytes(b"not a zip") is None
    live, peak, lock = [0], [0], threading.Lock()

    def load(data):
        with lock:
            live[0] += 1
            peak[0] = max(peak[0], live[0])
        time.sleep(0.2)
        with lock:
            live[0] -= 1
        return [np.zeros(250_000, np.float32)]

    saved = red.FedAvgPipeline, red.LOAD_AHEAD_BYTES
    red.FedAvgPipeline = Pipe
    try:
        combiners = [{"name": f"c{c}", "model_id": c} for c in range(6)]
        red.LOAD_AHEAD_BYTES = 1 << 30
        red.reduce_models(combiners, fetch=repo.__getitem__, load=load, device="cpu", workers=8)
        assert peak[0] == 6                       # all decodes overlapped, the first one included
        peak[0] = 0
        red.LOAD_AHEAD_BYTES = 3_100_000          # three decoded models
        red.reduce_models(combiners, fetch=repo.__getitem__, load=load, device="cpu", workers=8)
        assert peak[0] == 3
    finally:
        red.FedAvgPipeline, red.LOAD_AHEAD_BYTES = saved


def test_queued_updates_size_hint_across_rounds():
    """With the size of the previous round's updates (size_box), a round's read-ahead starts its
    decodes together instead of decoding the first update alone; without it, one at a time until
    the first decode shows the size."""
    import threading
    import time

    from fedn_amd.aggregators.aggregatorbase import queued_updates
    box = [None]
    for rnd in range(2):
        uh = MemoryUpdateHandler()
        for k in range(6):
            uh.submit([np.full(250, k, np.float32)], 1)          # 1000 bytes per update
        live, peak, lock = [0], [0], threading.Lock()
        inner = uh.load_model_update

        def load_model_update(mu, helper, inner=inner, live=live, peak=peak):
            with lock:
                live[0] += 1
                peak[0] = max(peak[0], live[0])
            time.sleep(0.05)
            with lock:
                live[0] -= 1
            return inner(mu, helper)
        uh.load_model_update = load_model_update
        it = queued_updates(uh, None, ahead=8, ahead_bytes=1 << 20, size_box=box)
        mu, load = next(it)
        time.sleep(0.03)                         # round 2: the others are already decoding
        first_peak = peak[0]
        load()
        for mu, load in it:
            load()
        assert box[0] == 1000
        assert first_peak == (1 if rnd == 0 else 6)


def test_queued_updates_first_round_peeks_npz_size():
    """With no size yet, the first update's raw npz bytes (load_model_update_byte) show the decoded
    size from the zip directory, so the first round's decodes start together too."""
    import io
    import threading
    import time

    from fedn_amd.aggregators.aggregatorbase import queued_updates

    class Helper:
        def load(self, f):
            z = np.load(f)
            return [z[k] for k in sorted(z.files, key=int)]

    uh = MemoryUpdateHandler()
    for k in range(5):
        b = io.BytesIO()
        np.savez_compressed(b, **{"0": np.full(250, k, np.float32)})
        uh.submit_bytes(b.getvalue(), 1)
    live, peak, lock = [0], [0], threading.Lock()
    inner = uh.load_model_update

    def load_model_update(mu, helper):
        with lock:
            live[0] += 1
            peak[0] = max(peak[0], live[0])
        time.sleep(0.05)
        with lock:
            live[0] -= 1
        return inner(mu, helper)
    uh.load_model_update = load_model_update
    box = [None]
    got = []
    it = queued_updates(uh, Helper(), ahead=8, ahead_bytes=1 << 20, size_box=box)
    mu, load = next(it)
    time.sleep(0.03)
    assert peak[0] == 5                          # every decode running before the first one ended
    got.append(int(load()[0][0][0]))
    for mu, load in it:
        got.append(int(load()[0][0][0]))
    assert got == [0, 1, 2, 3, 4] and box[0] == 1000


@pytest.mark.parametrize("R", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_pmc_rank_geometry_matches_bench(world, R, monkeypatch):
    """tools/pmc_rank_fold.py replays one rank's fold of bench.py --gpus N; its chunk / rounds /
    local length must be CyclicShardedFedAvg's for bench.py's chunk choice (P / (N * R)) for every
    candidate R of bench.AG_ROUNDS."""
    import bench
    import fedn_amd.sharded as sh
    from tools.pmc_rank_fold import rank_geometry
    monkeypatch.setattr(sh.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(sh.dist, "get_world_size", lambda group=None: world)
    monkeypatch.setattr(sh.dist, "get_rank", lambda group=None: 0)
    P = 100_000_000
    assert R in bench.AG_ROUNDS
    cyc = sh.CyclicShardedFedAvg(P, chunk=-(-P // (world * R)))
    assert rank_geometry(P, world, R) == (cyc.C, cyc.rounds, cyc.local_len)


def test_staging_cache_keeps_two_sizes_and_hands_out_once():
    """staging.StagingCache: a round's resources come back for the next round of the same size on
    the same device, are taken at most once, and at most ``keep`` sizes are kept (oldest dropped)."""
    from fedn_amd.staging import StagingCache
    c = StagingCache(keep=2)
    a, b, d = {"slots": ["a"]}, {"slots": ["b"]}, {"slots": ["d"]}
    c.give("cuda:0", 100, a)
    c.give("cuda:0", 200, b)
    assert c.take("cuda:1", 100) is None                  # another device: nothing
    assert c.take("cuda:0", 100) is a and c.take("cuda:0", 100) is None
    c.give("cuda:0", 100, a)
    c.give("cuda:0", 300, d)                              # third size: the oldest (200) goes
    assert c.take("cuda:0", 200) is None
    assert c.take("cuda:0", 100) is a and c.take("cuda:0", 300) is d


def test_narrow_int_fold_kinds():
    """numpy's rule for n * (y - x) on integer differences (numpyhelper.py:32): a python int n takes a
    narrow / unsigned dtype (wrapping: NFOLD), a float n or a numpy int that promotes to float64
    multiplies in float64 (IFOLD), an n outside the dtype raises OverflowError as numpy does."""
    import numpy as np
    import pytest
    from fedn_amd import mixed
    assert mixed._int_fold_kind(np.dtype(np.int8), 3) == "nfold"
    assert mixed._int_fold_kind(np.dtype(np.uint64), 7) == "nfold"
    assert mixed._int_fold_kind(np.dtype(np.int16), 2.5) == "ifold"
    assert mixed._int_fold_kind(np.dtype(np.uint8), 1.0) == "ifold"
    assert mixed._int_fold_kind(np.dtype(np.uint64), np.int64(3)) == "ifold"
    assert mixed._int_fold_kind(np.dtype(np.int32), 3) == "int"
    with pytest.raises(OverflowError):
        mixed._int_fold_kind(np.dtype(np.int8), 300)
    with pytest.raises(TypeError):
        mixed._int_fold_kind(np.dtype(np.int8), np.int64(3))    # int64 product: not instantiated
    with pytest.raises(TypeError):
        mixed._int_fold_kind(np.dtype(np.uint64), 1 << 60)
    with pytest.raises(TypeError):                              # numpy's boolean-subtract refusal
        mixed.fold_plan([((3,), np.dtype(bool))], [((3,), np.dtype(bool))], 2, 3)
    assert mixed.per_tensor_dtypes([np.float32, np.uint16]) and mixed.per_tensor_dtypes([np.bool_])
    assert not mixed.per_tensor_dtypes([np.float32, np.int64, np.float16])
    plan = mixed.fold_plan([((5,), np.dtype(np.int8))], [((1,), np.dtype(np.int16))], 9, 13)
    assert plan == [(np.dtype(np.int16), np.dtype(np.float64), (5,))]


def test_hbm_budget_accounting():
    """budget.HbmBudget: all-or-nothing reservations per device, release on garbage collection of
    the staged object, byte-count parsing (no GPU needed with an explicit limit)."""
    import gc

    from fedn_amd.budget import HbmBudget, parse_bytes
    assert parse_bytes("0") == 0 and parse_bytes("512") == 512 and parse_bytes("4K") == 4096
    assert parse_bytes("1.5G") == 3 << 29 and parse_bytes("2GiB") == 2 << 30 and parse_bytes("1T") == 1 << 40
    with pytest.raises(ValueError):
        parse_bytes("lots")
    b = HbmBudget(limit=1000)
    assert b.reserve([("cuda:0", 600)])
    assert not b.reserve([("cuda:0", 500)])                 # over the cap: refused, nothing taken
    assert b.reserve([("cuda:1", 900)])                     # devices are budgeted separately
    assert not b.reserve([("cuda:0", 100), ("cuda:1", 200)])   # all or nothing
    assert b.used("cuda:0") == 600 and b.used("cuda:1") == 900 and b.refused == 2

    class Staged:
        pass

    s = b.hold(Staged(), [("cuda:0", 600)])
    del s
    gc.collect()
    assert b.used("cuda:0") == 0
    b.release([("cuda:1", 900)])
    assert b.used("cuda:1") == 0


def test_helper_kind_recognises_plugins_and_refuses_others():
    """staging.helper_kind: FEDn's three helper plug-ins by module, this package's Helper, None as
    numpyhelper; anything else raises UnsupportedHelper (strict) or reads "unknown" (the ingest's
    non-strict query) — a ``name`` attribute alone never selects numpyhelper's arithmetic."""
    from fedn_amd.helper import Helper
    from fedn_amd.staging import UnsupportedHelper, helper_kind
    for kind in ("numpyhelper", "binaryhelper", "androidhelper"):
        cls = type("Helper", (), {"__module__": f"fedn.utils.helpers.plugins.{kind}"})
        assert helper_kind(cls()) == kind
    assert helper_kind(None) == "numpyhelper"
    assert helper_kind(Helper()) == "fednamdhelper"

    class Custom:
        name = "numpyhelper"
    with pytest.raises(UnsupportedHelper, match="not supported"):
        helper_kind(Custom())
    assert helper_kind(Custom(), strict=False) == "unknown"


def test_temp_file_store_mirrors_tempmodelstorage(tmp_path):
    """updatehandler.TempFileModelStore: bytes updates on disk (written chunk by chunk through
    MemoryModelService.Upload), read back whole, deleted with os.remove (tempmodelstorage.py:27-76)."""
    import os

    from fedn_amd.updatehandler import MemoryModelService, TempFileModelStore, _NpzBytes, upload_requests
    st = TempFileModelStore(str(tmp_path))
    svc = MemoryModelService(st)
    data = bytes(range(256)) * 9000
    svc.Upload(upload_requests(data, "u1", chunk=4096), None)
    assert os.path.getsize(st.path("u1")) == len(data)
    assert st.get("u1").data == data
    st.put("g", [1, 2])
    assert st.get("g") == [1, 2]
    st.put("u2", _NpzBytes(b"abc"))
    assert st.delete("u1") and not os.path.exists(st.path("u1"))
    assert st.delete("u2") and st.delete("g") and not st.delete("g")


def test_delete_model_hands_own_copies_to_the_reaper():
    """StagingUpdateHandler.delete_model: this handler's own copies of the update dropped on the
    reaper thread; the wrapped handler's delete (the store's) done by close() at the latest; both
    parts timed."""
    import gc
    import threading
    import weakref

    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    uh = MemoryUpdateHandler()
    st = StagingUpdateHandler(uh, helper=None, device="cpu", workers=1)

    class Big:
        nbytes = 1 << 20                 # AdoptedUploads accounts decoded uploads by size
    obj = Big()
    freed_on = []
    weakref.finalize(obj, lambda: freed_on.append(threading.current_thread().name))
    mu = uh.submit([np.zeros(4, np.float32)], 3)          # not via st: nothing staged
    from concurrent.futures import Future
    fut = Future()
    fut.set_result(obj)
    st._uploads.put(mu.model_update_id, fut)                  # as if decoded during its upload
    del obj, fut
    st.delete_model(mu)
    st.close()                                               # waits for the reaper
    gc.collect()
    assert freed_on == ["fedn_amd_reaper"]
    assert st.delete_times["count"] == 1 and st.delete_times["store_s"] >= 0 and st.delete_times["plugin_s"] >= 0
    assert uh.store.get(mu.model_update_id) is None           # the store's delete has run


class _SlowStoreHandler:
    """A wrapped UpdateHandler whose store delete takes ``delay`` seconds (os.remove of a large
    file) and raises for the ids in ``bad``."""

    def __init__(self, delay, bad=()):
        import threading
        self.delay, self.bad = delay, set(bad)
        self.deleted, self.threads = [], set()
        self._lock = threading.Lock()

    def delete_model(self, mu):
        import threading
        import time
        time.sleep(self.delay)
        if mu.model_update_id in self.bad:
            raise OSError(f"cannot delete {mu.model_update_id}")
        with self._lock:
            self.deleted.append(mu.model_update_id)
            self.threads.add(threading.current_thread().name)


def _mus(n):
    from types import SimpleNamespace
    return [SimpleNamespace(model_update_id=f"u{i}") for i in range(n)]


@pytest.mark.parametrize("workers", [0, 4])
def test_store_deletes_run_side_by_side_and_finish_before_the_round_ends(workers):
    """delete_workers > 0: the round's store deletes (tempmodelstorage.py:66-76, inline in
    fedavg.py:73-74) run concurrently; finish_deletes — what the aggregators call before
    combine_models returns — waits for every one, so the storage state at return is the
    reference's. delete_workers = 0: one after another inside delete_model, as the reference."""
    import time

    from fedn_amd.ingest import StagingUpdateHandler
    inner = _SlowStoreHandler(0.15)
    st = StagingUpdateHandler(inner, helper=None, device="cpu", workers=1, delete_workers=workers)
    mus = _mus(4)
    st.begin_deletes()                       # what combine_models does first
    t0 = time.perf_counter()
    for mu in mus:
        st.delete_model(mu)
    issued = time.perf_counter() - t0
    assert st.finish_deletes() == []
    total = time.perf_counter() - t0
    assert sorted(inner.deleted) == ["u0", "u1", "u2", "u3"]      # all done at "return"
    if workers:
        assert issued < 0.1 and total < 0.45 and all(t.startswith("fedn_amd_delete") for t in inner.threads)
    else:
        assert issued >= 0.6 and inner.threads == {"MainThread"}
    assert st.delete_times["count"] == 4 and st.delete_times["store_s"] >= 0.6
    st.close()


def test_a_failed_store_delete_is_logged_as_the_reference_logs_it(caplog):
    """A store delete that raises: the reference's per-update try logs it (fedavg.py:75-78) and the
    update stays counted; here finish_deletes hands it to the aggregator, which logs the same."""
    import logging

    from fedn_amd.aggregators.aggregatorbase import AggregatorBase
    from fedn_amd.ingest import StagingUpdateHandler
    inner = _SlowStoreHandler(0.0, bad={"u1"})
    st = StagingUpdateHandler(inner, helper=None, device="cpu", workers=1, delete_workers=2)
    class Agg(AggregatorBase):
        def __init__(self, uh):
            super().__init__(uh)
            self.name = "fedavg"

        def combine_models(self, helper=None, delete_models=True, parameters=None):
            return None, {}
    agg = Agg(st)
    agg._begin_deletes()
    for mu in _mus(3):
        st.delete_model(mu)
    with caplog.at_level(logging.ERROR, logger="fedn"):
        agg._finish_deletes()
    assert sorted(inner.deleted) == ["u0", "u2"]
    assert any("Error encoutered while processing model update: cannot delete u1" in r.getMessage()
               for r in caplog.records)
    st.close()


def test_deletes_outside_a_round_run_inline_and_a_failed_wait_still_finishes_them(caplog):
    """a delete_model made outside combine_models runs inline (nobody would wait for a
    background one), and the round's deletes are waited for even when the pipeline's quiesce raises —
    their failures logged, the round's own exception not masked."""
    import logging

    from fedn_amd.aggregators.aggregatorbase import AggregatorBase
    from fedn_amd.ingest import StagingUpdateHandler
    inner = _SlowStoreHandler(0.0, bad={"u2"})
    st = StagingUpdateHandler(inner, helper=None, device="cpu", workers=1, delete_workers=2)
    mus = _mus(4)
    st.delete_model(mus[0])                  # no round: inline, on this thread
    assert inner.deleted == ["u0"] and inner.threads == {"MainThread"}
    with pytest.raises(OSError):
        st.delete_model(mus[2])              # inline: the store's error reaches the caller

    class Agg(AggregatorBase):
        def __init__(self, uh):
            super().__init__(uh)
            self.name = "fedavg"

        def combine_models(self, helper=None, delete_models=True, parameters=None):
            return None, {}

    class Stuck:
        def quiesce(self):
            raise RuntimeError("gather thread failed")
    agg = Agg(st)
    agg._begin_deletes()
    st.delete_model(mus[1])
    st.delete_model(mus[2])
    with caplog.at_level(logging.ERROR, logger="fedn"), pytest.raises(RuntimeError, match="gather thread"):
        agg._end_round(Stuck())
    assert sorted(inner.deleted) == ["u0", "u1"] and not st._deletes
    assert any("cannot delete u2" in r.getMessage() for r in caplog.records)
    st.delete_model(mus[3])                  # the round is over: inline again
    assert "u3" in inner.deleted
    st.close()
