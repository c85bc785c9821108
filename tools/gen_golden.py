"""Generate the golden parity fixtures under ``tests/golden/`` by running FEDn ITSELF.

THIS SCRIPT IS TEST INFRASTRUCTURE. It runs only in the build container where the
read-only reference checkout exists at ``/root/reference``; it refuses to run anywhere
else (the GPU box has no reference). Only its OUTPUT (small ``.npz`` data files:
inputs + expected outputs) is committed and shipped; no reference source travels.

What it drives (all real reference code, imported from /root/reference):
  * ``fedn/utils/helpers/plugins/numpyhelper.py``   Helper (increment_average, add, ...)
  * ``fedn/network/combiner/aggregators/fedavg.py``  Aggregator.combine_models
  * ``fedn/network/combiner/aggregators/fedopt.py``  Aggregator.combine_models (adam/yogi/adagrad)
  * ``fedn/network/combiner/updatehandler.py``       UpdateHandler (FIFO queue, load_model_update)
  * ``fedn/network/combiner/modelservice.py``        ModelService (npz wire codec, temp storage)
Updates are pushed exactly as the combiner receives them: npz bytes uploaded through
``ModelService.set_model`` and a ``fedn_pb2.ModelUpdate`` proto with
``meta = {"training_metadata": {"num_examples": n}, "config": ...}`` handed to
``UpdateHandler.on_model_update``.

Import workaround: ``fedn/__init__.py`` and ``fedn/common/log_config.py``
pull in opentelemetry (not installed). We pre-register a bare ``fedn`` package and a stub
``fedn.common.log_config`` exposing ``logger``; nothing else is stubbed. ``Control.reduce`` is
run from control.py's own source without importing its module (which needs the absent
``tenacity``): see ``_control_reduce``.

Usage:  python tools/gen_golden.py            (writes tests/golden/*.npz + manifest.json: every fixture)
        python tools/gen_golden.py --out DIR  (the same into DIR; tools/verify_golden.py diffs it)
"""
import io
import json
import logging
import os
import struct
import sys
import tempfile
import types
import uuid

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden")


def _import_reference():
    if not os.path.isdir(os.path.join(REF, "fedn")):
        raise SystemExit("gen_golden: /root/reference is absent; fixtures are generated only in the build container")
    sys.dont_write_bytecode = True  # /root/reference is read-only
    os.environ.setdefault("FEDN_MODEL_DIR", tempfile.mkdtemp(prefix="fedn_models_"))
    pkg = types.ModuleType("fedn")
    pkg.__path__ = [os.path.join(REF, "fedn")]
    sys.modules["fedn"] = pkg
    common = types.ModuleType("fedn.common")
    common.__path__ = [os.path.join(REF, "fedn", "common")]
    sys.modules["fedn.common"] = common
    lc = types.ModuleType("fedn.common.log_config")
    lg = logging.getLogger("fedn")
    lg.setLevel(logging.CRITICAL)
    lc.logger = lg
    sys.modules["fedn.common.log_config"] = lc
    from fedn.network.combiner.aggregators import fedavg, fedopt  # noqa: E402
    from fedn.network.combiner.modelservice import ModelService  # noqa: E402
    from fedn.network.combiner.updatehandler import UpdateHandler  # noqa: E402
    from fedn.network.grpc import fedn_pb2  # noqa: E402
    from fedn.utils.helpers.plugins.numpyhelper import Helper  # noqa: E402
    from fedn.utils.parameters import Parameters  # noqa: E402

    return dict(fedavg=fedavg, fedopt=fedopt, ModelService=ModelService, UpdateHandler=UpdateHandler,
                pb2=fedn_pb2, Helper=Helper, Parameters=Parameters)


class Harness:
    """One combiner-side session: ModelService + UpdateHandler + an aggregator instance."""

    def __init__(self, ref, agg_name):
        self.ref = ref
        self.ms = ref["ModelService"]()
        self.uh = ref["UpdateHandler"](self.ms)
        self.helper = ref["Helper"]()
        self.agg = ref[agg_name].Aggregator(self.uh)

    def put_model(self, arrays, model_id):
        self.ms.set_model(arrays, model_id)

    def push_update(self, arrays, n, global_model_id):
        uid = str(uuid.uuid4())
        self.put_model(arrays, uid)
        meta = json.dumps({"training_metadata": {"num_examples": n, "batch_size": 32, "epochs": 1},
                           "config": json.dumps({"round_id": "1"})})
        mu = self.ref["pb2"].ModelUpdate(model_id=global_model_id, model_update_id=uid, meta=meta)
        self.uh.on_model_update(mu)

    def combine(self, parameters=None):
        return self.agg.combine_models(helper=self.helper, delete_models=True, parameters=parameters)


def _store_list(d, prefix, arrays):
    for t, a in enumerate(arrays):
        d[f"{prefix}_t{t}"] = np.asarray(a)
    d[f"{prefix}_len"] = np.array(len(arrays))


def _rng_model(rng, shapes, dtype):
    return [rng.standard_normal(s).astype(dtype) for s in shapes]


def _perturb(rng, model, dtype, scale=0.01):
    return [(np.asarray(w, dtype=np.float64) + scale * rng.standard_normal(np.shape(w))).astype(dtype) for w in model]


ODD_SHAPES = [(7,), (3, 5, 11), (1,), (129, 3), ()]
MNIST_SHAPES = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]  # examples/mnist-pytorch/client/model.py:18-32


def fedavg_mixed_case(ref, name, rng, nks):
    """A model with float32 weights and int64 counters (BatchNorm-like), folded by FedAvg."""
    h = Harness(ref, "fedavg")
    d = {"kind": np.array("fedavg"), "name": np.array(name)}
    base = _rng_model(rng, [(16, 3), (3,)], np.float64)
    for k, n in enumerate(nks):
        u = _perturb(rng, base, np.float32) + [np.array(1000 + 37 * k, dtype=np.int64),
                                               (np.arange(4) * (k + 3)).astype(np.int64)]
        h.push_update(u, int(n), "global-0")
        _store_list(d, f"r0_u{k}", u)
    d["r0_n"] = np.array(nks, dtype=np.int64)
    d["r0_K"] = np.array(len(nks))
    model, data = h.combine()
    d["r0_nr"] = np.array(data["nr_aggregated_models"])
    d["r0_data_keys"] = np.array(json.dumps(sorted(data)))
    d["r0_qsize"] = np.array(h.uh.model_updates.qsize())
    d["r0_out_none"] = np.array(model is None)
    _store_list(d, "r0_out", model)
    d["rounds"] = np.array(1)
    return d


def fedavg_case(ref, name, rng, shapes, dtype, nks, bad_index=None, special=None, int_vals=False):
    h = Harness(ref, "fedavg")
    d = {"kind": np.array("fedavg"), "name": np.array(name)}
    base = _rng_model(rng, shapes, np.float64)
    if special == "tiny":
        base = [w * np.float64(1e-41) for w in base]  # fp32 denormal range
    ups = []
    for k, n in enumerate(nks):
        if int_vals:
            u = [rng.integers(-1000, 1000, size=s).astype(dtype) for s in shapes]
        else:
            scale = 1e-41 if special == "tiny" else 0.01
            u = _perturb(rng, base, dtype, scale)
            if special == "wide":
                u = [w * np.asarray(10.0 ** rng.integers(-30, 30, size=np.shape(w)), dtype=dtype) for w in u]
                for w in u:
                    if w.size > 2:
                        w.flat[0] = 0.0
                        w.flat[1] = -0.0
        if bad_index is not None and k == bad_index:
            u = [np.zeros((s[0] + 1,) + tuple(s[1:]) if len(s) else (2,), dtype) for s in shapes]
        ups.append(u)
        h.push_update(u, int(n), "global-0")
        _store_list(d, f"r0_u{k}", u)
    d["r0_n"] = np.array(nks, dtype=np.int64)
    d["r0_K"] = np.array(len(nks))
    model, data = h.combine()
    d["r0_nr"] = np.array(data["nr_aggregated_models"])
    d["r0_data_keys"] = np.array(json.dumps(sorted(data)))
    d["r0_qsize"] = np.array(h.uh.model_updates.qsize())
    d["r0_out_none"] = np.array(model is None)
    if model is not None:
        _store_list(d, "r0_out", model)
    d["rounds"] = np.array(1)
    return d


def _mixed_model(rng, old):
    """float32 weights + an int64 counter (like BatchNorm's num_batches_tracked)."""
    return [old[0], np.asarray(old[1])]


def fedopt_case(ref, name, rng, shapes, nks_per_round, params=None, old_dtype=np.float32, upd_dtype=np.float32,
                int_tensor=False):
    h = Harness(ref, "fedopt")
    d = {"kind": np.array("fedopt"), "name": np.array(name)}
    d["params"] = np.array(json.dumps(params if params is not None else None))
    old = _rng_model(rng, shapes, old_dtype)
    if int_tensor:
        old = old + [np.array(100, dtype=np.int64), np.arange(5, dtype=np.int64)]
    for r, nks in enumerate(nks_per_round):
        gid = f"global-{r}"
        h.put_model(old, gid)
        _store_list(d, f"r{r}_old", old)
        for k, n in enumerate(nks):
            if int_tensor:
                u = _perturb(rng, old[:-2], upd_dtype) + [np.array(100 + 10 * (r + 1) + k, dtype=np.int64),
                                                         (np.arange(5) * (k + 2) + r).astype(np.int64)]
            else:
                u = _perturb(rng, old, upd_dtype)
            h.push_update(u, int(n), gid)
            _store_list(d, f"r{r}_u{k}", u)
        d[f"r{r}_n"] = np.array(nks, dtype=np.int64)
        d[f"r{r}_K"] = np.array(len(nks))
        p = ref["Parameters"](params) if params is not None else None
        model, data = h.combine(p)
        d[f"r{r}_nr"] = np.array(data.get("nr_aggregated_models", -1))
        d[f"r{r}_data_keys"] = np.array(json.dumps(sorted(data)))
        d[f"r{r}_qsize"] = np.array(h.uh.model_updates.qsize())
        d[f"r{r}_out_none"] = np.array(model is None)
        if model is not None:
            _store_list(d, f"r{r}_out", model)
        d[f"r{r}_m_none"] = np.array(h.agg.m is None)
        d[f"r{r}_v_none"] = np.array(h.agg.v is None)
        if h.agg.m is not None:
            _store_list(d, f"r{r}_m", h.agg.m)
        if h.agg.v is not None:
            _store_list(d, f"r{r}_v", h.agg.v)
        if model is not None:
            old = model  # next round's global model is this round's output (fp64), as in FEDn
    d["rounds"] = np.array(len(nks_per_round))
    return d


def helper_kat(ref):
    """numpyhelper known-answer test, fedn/utils/helpers/tests/test_numpyhelper.py:20-29."""
    h = ref["Helper"]()
    res = h.increment_average([np.array([1, 2, 3])], [np.array([4, 5, 6])], 10, 20)
    return {"kind": np.array("helper_kat"), "name": np.array("kat_int64"), "m1_t0": np.array([1, 2, 3]),
            "m2_t0": np.array([4, 5, 6]), "a": np.array(10), "W": np.array(20), "out_t0": res[0]}


def helper_ops(ref, rng):
    """Elementwise helper primitives a9 (numpyhelper.py:34-142) on mixed dtypes."""
    h = ref["Helper"]()
    x32 = rng.standard_normal(257).astype(np.float32)
    y32 = rng.standard_normal(257).astype(np.float32)
    x64 = rng.standard_normal(257)
    d = {"kind": np.array("helper_ops"), "name": np.array("helper_ops"), "x32": x32, "y32": y32, "x64": x64}
    d["add_32_32"] = h.add([x32], [y32], 0.9, 0.1)[0]
    d["add_64_32"] = h.add([x64], [y32], 0.99, 1.0 - 0.99)[0]
    d["sub_32_64"] = h.subtract([x32], [x64])[0]
    d["mul_32_s"] = h.multiply([x32], [1.0 - 0.9])[0]
    d["pow_32"] = h.power([x32], 2)[0]
    d["sqrt_64"] = h.sqrt([np.abs(x64)])[0]
    d["div_32_64"] = h.divide([x32], [np.abs(x64) + 1.0])[0]
    d["sign_64"] = h.sign([np.concatenate([x64, [0.0, -0.0]])])[0]
    d["ones_32"] = h.ones([x32], 1e-4 ** 2)[0]
    d["norm_32"] = np.array(h.norm([x32, y32]))
    return d


def helper_power_norm(ref, rng):
    """numpyhelper.power with general exponents and numpyhelper.norm (numpyhelper.py:94-117), the
    real helper on float32 / float64 / int64 tensors, vectors and matrices."""
    h = ref["Helper"]()
    x32 = np.abs(rng.standard_normal(513)).astype(np.float32) + np.float32(0.01)
    x64 = np.abs(rng.standard_normal(257)) + 0.01
    i64 = rng.integers(-50, 50, 129).astype(np.int64)
    m32 = rng.standard_normal((37, 11)).astype(np.float32)
    m64 = rng.standard_normal((5, 300))
    d = {"kind": np.array("helper_ops2"), "name": np.array("helper_power_norm"), "x32": x32, "x64": x64, "i64": i64,
         "m32": m32, "m64": m64}
    for a, tag in ((0.5, "half"), (3, "i3"), (-1.5, "neg1p5"), (2, "sq"), (0.7, "p07")):
        d[f"pow32_{tag}"] = h.power([x32], a)[0]
        d[f"pow64_{tag}"] = h.power([x64], a)[0]
    d["powi64_3"] = h.power([i64], 3)[0]
    d["powi64_0"] = h.power([i64], 0)[0]
    d["powi64_f"] = h.power([np.abs(i64)], 0.5)[0]
    d["norm_vec32"] = np.array(h.norm([x32]))
    d["norm_mat32"] = np.array(h.norm([m32]))
    d["norm_mixed"] = np.array(h.norm([m32, x64, i64, m64]))
    return d


class _Repository:
    """The controller's model repository as Control.reduce uses it (control.py:668,690):
    get_model(model_id) -> the stored bytes (raises for a model that cannot be fetched),
    delete_model(model_id)."""

    def __init__(self, blobs):
        self.blobs, self.deleted = blobs, []

    def get_model(self, model_id):
        if self.blobs[model_id] is None:
            raise RuntimeError(f"model {model_id} not in the repository")
        return self.blobs[model_id]

    def delete_model(self, model_id):
        self.deleted.append(model_id)


def _control_reduce(ref, models, plan):
    """Run the REAL ``Control.reduce`` (fedn/network/controller/control.py:648-693).

    control.py's module imports ``tenacity`` (absent from the image; it decorates other methods),
    so the module itself is not imported. The method is taken from control.py's own source with
    ``ast`` and compiled from that file (line numbers kept), in a namespace holding the real
    objects its body names: ``time``, the fedn logger and modelservice.load_model_from_bytes.
    ``self`` supplies ``repository`` (get_model / delete_model) and ``get_helper()`` -> the real
    numpyhelper. Each combiner model is stored as the bytes the real
    modelservice.serialize_model_to_BytesIO writes; "missing" makes get_model raise."""
    import ast
    import time

    from fedn.common.log_config import logger
    from fedn.network.combiner.modelservice import load_model_from_bytes, serialize_model_to_BytesIO
    path = os.path.join(REF, "fedn", "network", "controller", "control.py")
    with open(path) as f:
        tree = ast.parse(f.read(), path)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Control")
    fn = next(n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == "reduce")
    ns = {"time": time, "logger": logger, "load_model_from_bytes": load_model_from_bytes}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), path, "exec"), ns)  # noqa: S102
    helper = ref["Helper"]()
    blobs = {f"model-{c}": None if kind == "missing" else serialize_model_to_BytesIO(m, helper).getvalue()
             for c, (m, kind) in enumerate(zip(models, plan))}
    ctl = types.SimpleNamespace(repository=_Repository(blobs), get_helper=lambda: helper)
    combiners = [{"name": f"combiner-{c}", "model_id": f"model-{c}"} for c in range(len(models))]
    model, meta = ns["reduce"](ctl, combiners)
    assert ctl.repository.deleted == [c["model_id"] for c in combiners]
    assert sorted(meta) == ["time_aggregate_model", "time_fetch_model", "time_load_model"]
    return model


def reduce_case(ref, name, rng, shapes, plan):
    """Control.reduce (control.py:648-693), the real method (_control_reduce).
    plan: per combiner "ok" | "missing" (fetch fails -> data None) | "bad" (shape mismatch)."""
    d = {"kind": np.array("reduce"), "name": np.array(name), "plan": np.array(json.dumps(plan))}
    base = _rng_model(rng, shapes, np.float32)
    models = []
    for c, kind in enumerate(plan):
        if kind == "bad":
            m = [np.ones((s[0] + 2,) + tuple(s[1:]) if len(s) else (3,), np.float32) for s in shapes]
        else:
            m = _perturb(rng, base, np.float32, 0.05)
        models.append(m)
        _store_list(d, f"c{c}", m)
    model = _control_reduce(ref, models, plan)
    d["out_none"] = np.array(model is None)
    if model is not None:
        _store_list(d, "out", model)
    return d


def _tensor(rng, shape, dtype):
    """One client tensor: integers for integer dtypes, ~1 + 0.01 N(0,1) for floats."""
    dtype = np.dtype(dtype)
    if dtype.kind in "iu":
        return rng.integers(-1000, 1000, size=shape).astype(dtype)
    return (1.0 + 0.01 * rng.standard_normal(shape)).astype(dtype)


def fedavg_clients_case(ref, name, rng, clients, nks):
    """FedAvg over clients whose tensors differ from the first client's in dtype and/or
    (broadcastable) shape: numpyhelper.py:32 promotes and broadcasts them. ``clients`` holds,
    per client, a list of (shape, dtype) per tensor."""
    h = Harness(ref, "fedavg")
    d = {"kind": np.array("fedavg"), "name": np.array(name)}
    for k, (spec, n) in enumerate(zip(clients, nks)):
        u = [_tensor(rng, s, dt) for s, dt in spec]
        h.push_update(u, int(n), "global-0")
        _store_list(d, f"r0_u{k}", u)
    d["r0_n"] = np.array(nks, dtype=np.int64)
    d["r0_K"] = np.array(len(nks))
    model, data = h.combine()
    d["r0_nr"] = np.array(data["nr_aggregated_models"])
    d["r0_data_keys"] = np.array(json.dumps(sorted(data)))
    d["r0_qsize"] = np.array(h.uh.model_updates.qsize())
    d["r0_out_none"] = np.array(model is None)
    if model is not None:
        _store_list(d, "r0_out", model)
    d["rounds"] = np.array(1)
    return d


def fedopt_clients_case(ref, name, rng, old_spec, rounds, params=None):
    """FedOpt rounds whose clients differ from the global model (and from each other) in dtype
    and/or broadcastable shape (fedopt.py:89-94: subtract + increment_average promote and
    broadcast). ``rounds`` holds, per round, per client a list of (shape, dtype); a round's
    global model is the previous round's output."""
    h = Harness(ref, "fedopt")
    d = {"kind": np.array("fedopt"), "name": np.array(name)}
    d["params"] = np.array(json.dumps(params))
    old = [_tensor(rng, s, dt) for s, dt in old_spec]
    for r, clients in enumerate(rounds):
        gid = f"global-{r}"
        h.put_model(old, gid)
        _store_list(d, f"r{r}_old", old)
        nks = rng.integers(1, 5001, len(clients))
        for k, (spec, n) in enumerate(zip(clients, nks)):
            u = [_tensor(rng, s, dt) for s, dt in spec]
            h.push_update(u, int(n), gid)
            _store_list(d, f"r{r}_u{k}", u)
        d[f"r{r}_n"] = np.array(nks, dtype=np.int64)
        d[f"r{r}_K"] = np.array(len(clients))
        model, data = h.combine(ref["Parameters"](params) if params is not None else None)
        d[f"r{r}_nr"] = np.array(data.get("nr_aggregated_models", -1))
        d[f"r{r}_data_keys"] = np.array(json.dumps(sorted(data)))
        d[f"r{r}_qsize"] = np.array(h.uh.model_updates.qsize())
        d[f"r{r}_out_none"] = np.array(model is None)
        if model is not None:
            _store_list(d, f"r{r}_out", model)
        d[f"r{r}_m_none"] = np.array(h.agg.m is None)
        d[f"r{r}_v_none"] = np.array(h.agg.v is None)
        if h.agg.m is not None:
            _store_list(d, f"r{r}_m", h.agg.m)
        if h.agg.v is not None:
            _store_list(d, f"r{r}_v", h.agg.v)
        if model is not None:
            old = model
    d["rounds"] = np.array(len(rounds))
    return d


def reduce_dtypes_case(ref, name, rng, shapes, dtypes):
    """Control.reduce (control.py:648-693, the real method: _control_reduce) over combiner models
    saved in different dtypes."""
    plan = ["ok"] * len(dtypes)
    d = {"kind": np.array("reduce"), "name": np.array(name), "plan": np.array(json.dumps(plan))}
    models = []
    for c, dt in enumerate(dtypes):
        m = [_tensor(rng, s, dt) for s in shapes]
        models.append(m)
        _store_list(d, f"c{c}", m)
    model = _control_reduce(ref, models, plan)
    _store_list(d, "out", model)
    d["out_none"] = np.array(False)
    return d


F16, F32, F64, I32, I64 = np.float16, np.float32, np.float64, np.int32, np.int64
MIX_SHAPES = [(7,), (3, 5), (2053,), ()]


def _spec(dtypes, shapes=MIX_SHAPES):
    """(shape, dtype) per tensor; one dtype for all tensors or one per tensor."""
    if not isinstance(dtypes, (list, tuple)):
        dtypes = [dtypes] * len(shapes)
    return list(zip(shapes, dtypes))


def mixed_cases(ref):
    """Clients whose updates differ in dtype or broadcastable shape."""
    rng = np.random.default_rng(7)
    nk = lambda K: rng.integers(1, 5001, K)  # noqa: E731
    cases = [
        fedavg_clients_case(ref, "fedavg_mix_f32_f64_k4", rng, [_spec(F32), _spec(F64), _spec(F32), _spec(F64)], nk(4)),
        fedavg_clients_case(ref, "fedavg_mix_f64_f32_k3", rng, [_spec(F64), _spec(F32), _spec(F32)], nk(3)),
        fedavg_clients_case(ref, "fedavg_mix_i64_f32_k3", rng, [_spec(I64), _spec(F32), _spec(I64)], nk(3)),
        fedavg_clients_case(ref, "fedavg_mix_f32_i64_i32_k4", rng,
                            [_spec(F32), _spec(I64), _spec(I32), _spec(F32)], nk(4)),
        fedavg_clients_case(ref, "fedavg_mix_i32_i64_k3", rng, [_spec(I32), _spec(I64), _spec(I32)], nk(3)),
        fedavg_clients_case(ref, "fedavg_mix_f16_f32_k4", rng, [_spec(F16), _spec(F32), _spec(F16), _spec(F32)], nk(4)),
        fedavg_clients_case(ref, "fedavg_mix_f32_f16_k3", rng, [_spec(F32), _spec(F16), _spec(F16)], nk(3)),
        fedavg_clients_case(ref, "fedavg_mix_pertensor_k5", rng,
                            [_spec(F32), _spec([F32, F64, F32, F32]), _spec(F32), _spec([F32, F32, F64, I64]),
                             _spec(F32)], nk(5)),
        fedavg_clients_case(ref, "fedavg_bcast_k4", rng,
                            [_spec(F32, [(1,), (3, 5), (1, 6), ()]), _spec(F32, [(7,), (1, 5), (4, 1), (9,)]),
                             _spec(F32, [(7,), (3, 5), (4, 6), ()]), _spec(F64, [(1,), (3, 1), (4, 6), (9,)])],
                            nk(4)),
        fedavg_clients_case(ref, "fedavg_fewer_tensors_k3", rng,          # zip() truncates the model
                            [_spec(F32), _spec(F32, MIX_SHAPES[:3]), _spec(F32)], nk(3)),
        fedavg_clients_case(ref, "fedavg_bcast_then_bad_k4", rng,
                            [_spec(F32, [(5,), (2, 3)]), _spec(F32, [(1,), (2, 3)]),
                             _spec(F32, [(4,), (2, 3)]), _spec(F32, [(5,), (3,)])], nk(4)),
    ]
    fo = [(7,), (3, 5), (2053,)]
    for opt in ("adam", "yogi", "adagrad"):
        params = None if opt == "adam" else {"serveropt": opt}
        cases.append(fedopt_clients_case(
            ref, f"fedopt_mix_{opt}_3r", rng, _spec(F32, fo),
            [[_spec(F32, fo), _spec(F64, fo), _spec(F32, fo)],      # one float64 client mid-round
             [_spec(F64, fo), _spec(F32, fo)],                      # the first client is float64
             [_spec(F32, fo), _spec([F32, I64, F32], fo), _spec(F32, fo)]], params))
    cases.append(fedopt_clients_case(ref, "fedopt_layout_change_3r", rng, _spec(F32, fo),
                                     [[_spec(F32, fo)] * 3, [_spec(F64, fo)] * 2, [_spec(F32, fo)] * 2]))
    cases.append(fedopt_clients_case(ref, "fedopt_f64_clients_f32_model_2r", rng, _spec(F32, fo),
                                     [[_spec(F64, fo)] * 3, [_spec(F64, fo)] * 2], {"serveropt": "yogi"}))
    cases.append(fedopt_clients_case(ref, "fedopt_bcast_2r", rng, _spec(F32, [(7,), (3, 5)]),
                                     [[_spec(F32, [(7,), (3, 5)]), _spec(F32, [(1,), (1, 5)]),
                                       _spec(F32, [(7,), (3, 1)])],
                                      [_spec(F32, [(1,), (3, 5)]), _spec(F32, [(7,), (3, 5)])]]))
    rng = np.random.default_rng(8)
    cases.append(reduce_dtypes_case(ref, "reduce_mix_f32_f64_f32", rng, ODD_SHAPES, [F32, F64, F32]))
    cases.append(reduce_dtypes_case(ref, "reduce_mix_f64_f32", rng, ODD_SHAPES, [F64, F32, F32]))
    return cases


def _example_server_functions(ref, filename):
    """The REAL example class, instantiated the way the hooks server does it (hooks.py:187-205:
    compile the user file, exec it, exec ``ServerFunctions()``). Its first line imports
    ``fedn.network.combiner.hooks.allowed_import``, whose module body builds an APIClient
    (network); we register that module with the names it re-exports taken from their real
    sources (numpy, typing, the real ServerFunctionsBase) and ``api_client = None`` — the
    aggregation methods do not use it."""
    import typing

    from fedn.network.combiner.hooks.serverfunctionsbase import ServerFunctionsBase
    ai = types.ModuleType("fedn.network.combiner.hooks.allowed_import")
    ai.Dict, ai.List, ai.Tuple = typing.Dict, typing.List, typing.Tuple
    ai.np, ai.ServerFunctionsBase, ai.api_client = np, ServerFunctionsBase, None
    ai.logger = logging.getLogger("fedn")
    ai.print = lambda *a, **k: None
    sys.modules["fedn.network.combiner.hooks.allowed_import"] = ai
    path = os.path.join(REF, "examples", "server-functions", filename)
    with open(path) as f:
        code = compile(f.read(), path, "exec")
    ns = {"print": ai.print}
    exec(code, ns)  # noqa: S102 — reference example code, as hooks.py runs it
    return ns["ServerFunctions"]


def _meta(rng, k, kind):
    if kind == "int":
        return {"num_examples": int(rng.integers(1, 5001))}
    if kind == "float":
        return {"num_examples": float(rng.integers(1, 50000)) / 8.0}
    if kind == "missing" and k == 1:
        return {"training_loss": 0.5}            # no num_examples -> metadata.get(..., 1)
    return {"num_examples": int(rng.integers(1, 5001))}


def sf_wavg_case(ref, name, rng, shapes, K, prev_dtype=np.float32, upd_dtype=np.float32, meta="int"):
    """examples/server-functions/server_functions.py:53-68 run on client_updates built as
    hooks.py:88-101 builds them ({client_id: [model, metadata]}, arrival order)."""
    SF = _example_server_functions(ref, "server_functions.py")
    d = {"kind": np.array("sf_wavg"), "name": np.array(name), "K": np.array(K)}
    prev = _rng_model(rng, shapes, prev_dtype)
    _store_list(d, "prev", prev)
    updates = {}
    for k in range(K):
        u = _perturb(rng, prev, upd_dtype)
        md = _meta(rng, k, meta)
        _store_list(d, f"u{k}", u)
        d[f"meta{k}"] = np.array(json.dumps(md))
        updates[f"client-{k}"] = [u, md]
    out = SF().aggregate(prev, updates)
    _store_list(d, "out", out)
    return d


def sf_inc_case(ref, name, rng, shapes, Ks, dtype=np.float32, meta="int"):
    """examples/server-functions/sf_incremental_aggregation.py over several rounds on ONE
    instance (the hooks server keeps it across rounds), fed as hooks.py:107-117 feeds it."""
    SF = _example_server_functions(ref, "sf_incremental_aggregation.py")
    sf = SF()
    d = {"kind": np.array("sf_inc"), "name": np.array(name), "rounds": np.array(len(Ks))}
    prev = _rng_model(rng, shapes, dtype)
    for r, K in enumerate(Ks):
        d[f"r{r}_K"] = np.array(K)
        _store_list(d, f"r{r}_prev", prev)
        for k in range(K):
            u = _perturb(rng, prev, dtype)
            md = _meta(rng, k, meta)
            _store_list(d, f"r{r}_u{k}", u)
            d[f"r{r}_meta{k}"] = np.array(json.dumps(md))
            sf.incremental_aggregate(f"client-{k}", [np.array(a) for a in u], md, prev)
        # K == 0: the example returns the previous_global it last saw in incremental_aggregate
        # (it is only set there, sf_incremental_aggregation.py:26), i.e. an earlier round's
        out = [np.array(a) for a in sf.get_incremental_aggregate_model()]
        _store_list(d, f"r{r}_out", out)
        prev = out
    return d


def sf_cases(ref):
    rng = np.random.default_rng(6)
    return [
        sf_wavg_case(ref, "sf_wavg_mnist_k2", rng, MNIST_SHAPES, 2),
        sf_wavg_case(ref, "sf_wavg_f64prev_k4", rng, ODD_SHAPES, 4, prev_dtype=np.float64),
        sf_wavg_case(ref, "sf_wavg_f64upd_f32acc_k3", rng, ODD_SHAPES, 3, upd_dtype=np.float64),
        sf_wavg_case(ref, "sf_wavg_f64_k3", rng, ODD_SHAPES, 3, prev_dtype=np.float64, upd_dtype=np.float64),
        sf_wavg_case(ref, "sf_wavg_floatw_k4", rng, ODD_SHAPES, 4, meta="float"),
        sf_wavg_case(ref, "sf_wavg_missingw_k3", rng, ODD_SHAPES, 3, meta="missing"),
        sf_wavg_case(ref, "sf_wavg_empty", rng, ODD_SHAPES, 0),
        sf_wavg_case(ref, "sf_wavg_k70", rng, [(1031,)], 70),
        sf_inc_case(ref, "sf_inc_3r", rng, ODD_SHAPES + [(2053,)], [4, 3, 2]),
        sf_inc_case(ref, "sf_inc_f64_2r", rng, ODD_SHAPES, [3, 2], dtype=np.float64),
        sf_inc_case(ref, "sf_inc_floatw_2r", rng, ODD_SHAPES, [3, 3], meta="float"),
        sf_inc_case(ref, "sf_inc_empty_round", rng, ODD_SHAPES, [2, 0, 2]),
    ]


def _payload(helper_name, vals):
    """Update bytes as the helper's save() writes them (androidhelper.py:62-76: struct of
    float32; binaryhelper -> numpyhelper.save raw_binary: float64 tofile)."""
    if helper_name == "androidhelper":
        return struct.pack("f" * len(vals), *np.asarray(vals, dtype=np.float32).tolist())
    return np.asarray(vals, dtype=np.float64).tobytes()


def helper_case(ref, name, helper_cls, agg_name, rng, P, nks_per_round, params=None):
    """FedAvg / FedOpt with a non-numpy helper FEDn accepts (package.py:24): the aggregator folds
    with THAT helper (fedavg.py:68 helper.increment_average; fedopt.py:89-94 helper.subtract ...).
    Updates are uploaded as the helper's bytes and loaded back by UpdateHandler.load_model_update
    with the helper (updatehandler.py:90-117, modelservice.py:110-125)."""
    h = Harness(ref, agg_name)
    h.helper = helper_cls()
    hn = type(h.helper).__module__.rsplit(".", 1)[-1]   # androidhelper sets name, HelperBase resets it
    d = {"kind": np.array("helper_" + agg_name), "name": np.array(name), "helper": np.array(hn)}
    if params is not None:
        d["params"] = np.array(json.dumps(params))
    unwrap = (lambda m: m) if hn == "androidhelper" else (lambda m: m[0])
    old = rng.standard_normal(P)
    for r, nks in enumerate(nks_per_round):
        gid = f"global-{r}"
        h.ms.set_model(io.BytesIO(_payload(hn, old)), gid)
        d[f"r{r}_old"] = np.asarray(unwrap(h.helper.load(io.BytesIO(_payload(hn, old)))))
        for k, n in enumerate(nks):
            vals = old + 0.01 * rng.standard_normal(P)
            uid = str(uuid.uuid4())
            h.ms.set_model(io.BytesIO(_payload(hn, vals)), uid)
            meta = json.dumps({"training_metadata": {"num_examples": int(n)}, "config": json.dumps({"round_id": "1"})})
            h.uh.on_model_update(ref["pb2"].ModelUpdate(model_id=gid, model_update_id=uid, meta=meta))
            d[f"r{r}_u{k}"] = np.asarray(unwrap(h.helper.load(io.BytesIO(_payload(hn, vals)))))
        d[f"r{r}_n"] = np.array(nks, dtype=np.int64)
        d[f"r{r}_K"] = np.array(len(nks))
        model, data = h.combine(ref["Parameters"](params) if params is not None else None)
        d[f"r{r}_nr"] = np.array(data["nr_aggregated_models"])
        d[f"r{r}_qsize"] = np.array(h.uh.model_updates.qsize())
        d[f"r{r}_out_none"] = np.array(model is None)
        if model is not None:
            d[f"r{r}_out"] = np.asarray(unwrap(model))
            old = np.asarray(unwrap(model), dtype=np.float64)
        if agg_name == "fedopt" and h.agg.m is not None:
            d[f"r{r}_m"] = np.asarray(unwrap(h.agg.m))
            d[f"r{r}_v"] = np.asarray(unwrap(h.agg.v))
    d["rounds"] = np.array(len(nks_per_round))
    return d


def helper_cases(ref):
    from fedn.utils.helpers.plugins.androidhelper import Helper as Android
    from fedn.utils.helpers.plugins.binaryhelper import Helper as Binary
    rng = np.random.default_rng(6)
    return [
        helper_case(ref, "android_fedavg_k1", Android, "fedavg", rng, 1000, [[77]]),
        helper_case(ref, "android_fedavg_k2", Android, "fedavg", rng, 1000, [list(rng.integers(1, 5001, 2))]),
        helper_case(ref, "android_fedavg_k9", Android, "fedavg", rng, 4099, [list(rng.integers(1, 5001, 9))]),
        helper_case(ref, "android_fedopt_k3", Android, "fedopt", rng, 1000, [list(rng.integers(1, 5001, 3))]),
        helper_case(ref, "binary_fedavg_k5", Binary, "fedavg", rng, 2053, [list(rng.integers(1, 5001, 5))]),
        helper_case(ref, "binary_fedopt_2r", Binary, "fedopt", rng, 2053,
                    [list(rng.integers(1, 5001, 4)), list(rng.integers(1, 5001, 3))], {"serveropt": "yogi"}),
    ]


def fedavg_numex_case(ref, name, rng, spec, nks):
    """FedAvg where num_examples arrive as JSON numbers of either type (int or float): numpy folds an
    integer tensor's difference with an int n in the integer dtype but with a float n in float64
    (numpyhelper.py:32). ``spec`` = (shape, dtype) per tensor; ``nks`` = python ints / floats."""
    h = Harness(ref, "fedavg")
    d = {"kind": np.array("fedavg"), "name": np.array(name)}
    for k, n in enumerate(nks):
        u = [_tensor(rng, s, dt) for s, dt in spec]
        h.push_update(u, n, "global-0")
        _store_list(d, f"r0_u{k}", u)
    d["r0_n"] = np.array([float(n) for n in nks], dtype=np.float64)
    d["r0_n_isfloat"] = np.array([isinstance(n, float) for n in nks])
    d["r0_K"] = np.array(len(nks))
    model, data = h.combine()
    d["r0_nr"] = np.array(data["nr_aggregated_models"])
    d["r0_data_keys"] = np.array(json.dumps(sorted(data)))
    d["r0_qsize"] = np.array(h.uh.model_updates.qsize())
    d["r0_out_none"] = np.array(model is None)
    if model is not None:
        _store_list(d, "r0_out", model)
    d["rounds"] = np.array(1)
    return d


def numex_cases(ref):
    """num_examples reported as floats (VERDICT r2 follow-up: integer tensors folded with a float n)."""
    rng = np.random.default_rng(12)
    i64 = [((5,), I64), ((2, 3), F32), ((7,), I64)]
    return [
        fedavg_numex_case(ref, "fedavg_int64_float_n_k4", rng, i64, [7.5, 12.25, 3, 100.0]),
        fedavg_numex_case(ref, "fedavg_int32_float_n_k3", rng, [((6,), I32), ((4,), I32)], [5, 2.5, 4]),
        fedavg_numex_case(ref, "fedavg_int64_n_one_float_k3", rng, i64, [3, 1.0, 2.5]),
        fedavg_numex_case(ref, "fedavg_int64_bign_float_k3", rng, [((9,), I64)], [2, 3.0e15, 7.75]),
        fedavg_numex_case(ref, "fedavg_f32_float_n_k4", rng, [((33,), F32), ((2, 2), F64)], [1.5, 2, 0.25, 1e6]),
    ]


def narrow_cases(ref):
    """Models with 8 / 16-bit and unsigned integer tensors: the first fold's difference and (python
    int n) product wrap in the narrow dtype, a float n multiplies in float64, an n outside the dtype's
    range makes numpy raise (FEDn skips that update), bool tensors never fold (boolean subtract)."""
    rng = np.random.default_rng(14)
    I8, I16, U8, U16, U32, U64 = np.int8, np.int16, np.uint8, np.uint16, np.uint32, np.uint64
    return [
        fedavg_numex_case(ref, "fedavg_int8_k4", rng, [((5,), I8), ((2, 3), F32), ((7,), I8)], [7, 12, 3, 100]),
        fedavg_numex_case(ref, "fedavg_u8_i16_n_overflow_k4", rng, [((9,), U8), ((4,), I16)], [5, 300, 7, 2]),
        fedavg_numex_case(ref, "fedavg_unsigned_k3", rng, [((6,), U16), ((5,), U32), ((4,), U64)], [40000, 7, 3]),
        fedavg_numex_case(ref, "fedavg_narrow_float_n_k3", rng, [((6,), I8), ((5,), U16), ((3,), U64)], [3, 2.5, 4]),
        fedavg_clients_case(ref, "fedavg_narrow_mixed_k3", rng,
                            [_spec([I8, U8, I16], [(5,), (4,), (3,)]), _spec([I16, I8, U16], [(1,), (4,), (3,)]),
                             _spec([F16, U8, I16], [(5,), (4,), (1,)])], [9, 4, 6]),
        fedavg_numex_case(ref, "fedavg_bool_k3", rng, [((4,), np.bool_), ((3,), F32)], [2, 3, 4]),
        fedopt_clients_case(ref, "fedopt_int8_2r", rng, _spec(I8, [(7,), (3, 5)]),
                            [[_spec(I8, [(7,), (3, 5)])] * 3, [_spec(I8, [(7,), (3, 5)])] * 2]),
        fedopt_clients_case(ref, "fedopt_u8_old_i16_upd_2r", rng, _spec(U8, [(6,), (2, 2)]),
                            [[_spec(I16, [(6,), (2, 2)])] * 2, [_spec(U32, [(6,), (2, 2)])] * 2], {"serveropt": "yogi"}),
        reduce_dtypes_case(ref, "reduce_int8_3", rng, ODD_SHAPES, [I8, I8, I8]),
        reduce_dtypes_case(ref, "reduce_mix_u16_i8_f32", rng, ODD_SHAPES, [U16, I8, F32]),
    ]


def f16_fedopt_cases(ref):
    """FedOpt sessions on a float16 global model (VERDICT r2 follow-up): numpy computes the pseudo-
    gradient in half while it is half (round 1), then float64; m stays half until it meets a float64
    pseudo-gradient."""
    rng = np.random.default_rng(13)
    fo = [(7,), (3, 5), (2053,)]
    return [
        fedopt_clients_case(ref, "fedopt_f16_adam_3r", rng, _spec(F16, fo),
                            [[_spec(F16, fo)] * 3, [_spec(F16, fo)] * 2, [_spec(F16, fo)] * 3]),
        fedopt_clients_case(ref, "fedopt_f16_yogi_k70_2r", rng, _spec(F16, fo),
                            [[_spec(F16, fo)] * 70, [_spec(F16, fo)] * 2], {"serveropt": "yogi"}),
        fedopt_clients_case(ref, "fedopt_f16_adagrad_2r", rng, _spec(F16, fo),
                            [[_spec(F16, fo)] * 4, [_spec(F16, fo)] * 3], {"serveropt": "adagrad"}),
        fedopt_clients_case(ref, "fedopt_f16_upd_f32_old_2r", rng, _spec(F32, fo),
                            [[_spec(F16, fo)] * 3, [_spec(F16, fo)] * 2]),
        fedopt_clients_case(ref, "fedopt_f32_upd_f16_old_2r", rng, _spec(F16, fo),
                            [[_spec(F32, fo)] * 3, [_spec(F32, fo)] * 2], {"serveropt": "yogi"}),
        # per-tensor path: a broadcast client keeps the pg half; a float32 client promotes it
        fedopt_clients_case(ref, "fedopt_f16_bcast_2r", rng, _spec(F16, fo),
                            [[_spec(F16, fo), _spec(F16, [(1,), (3, 5), (2053,)]), _spec(F16, fo)],
                             [_spec(F16, fo)] * 2]),
        fedopt_clients_case(ref, "fedopt_f16_mixed_2r", rng, _spec(F16, fo),
                            [[_spec(F16, fo), _spec(F32, fo), _spec(F16, [(7,), (1, 5), (2053,)])],
                             [_spec(F16, fo)] * 2], {"serveropt": "adagrad"}),
    ]


def edge_cases(ref):
    """Zero-size tensors (alone and among others) and rounds of more than 64 clients (the
    kernarg client table's size: several launches / arena batches per round)."""
    rng = np.random.default_rng(11)
    zshapes = [(4,), (0,), (2, 0, 3), (5,)]
    return [
        fedavg_case(ref, "fedavg_zero_size_k3", rng, zshapes, np.float32, rng.integers(1, 5001, 3)),
        fedavg_case(ref, "fedavg_all_empty_k2", rng, [(0,), (0, 4)], np.float32, rng.integers(1, 5001, 2)),
        fedavg_case(ref, "fedavg_odd_k70", rng, ODD_SHAPES, np.float32, rng.integers(1, 5001, 70)),
        fedopt_case(ref, "fedopt_zero_size_2r", rng, zshapes, [list(rng.integers(1, 5001, 3)) for _ in range(2)]),
        fedopt_case(ref, "fedopt_yogi_k70", rng, ODD_SHAPES, [list(rng.integers(1, 5001, 70)), [3, 9]],
                    {"serveropt": "yogi"}),
    ]


def reduce_cases(ref):
    """Control.reduce (control.py:648-693) over combiner models."""
    rng = np.random.default_rng(4)
    return [reduce_case(ref, "reduce_3", rng, ODD_SHAPES, ["ok", "ok", "ok"]),
            reduce_case(ref, "reduce_missing", rng, ODD_SHAPES, ["missing", "ok", "missing", "ok", "ok"]),
            reduce_case(ref, "reduce_bad_replaces", rng, ODD_SHAPES, ["ok", "ok", "bad", "ok"]),
            reduce_case(ref, "reduce_single", rng, ODD_SHAPES, ["ok"])]


# views save cases hand to numpyhelper.save (rebuilt from the stored base by tests/test_savez_golden.py)
SAVE_VIEWS = {
    "T": lambda b: b.T,
    "cols3": lambda b: b[:, ::3],
    "rev": lambda b: b[::-1],
    "perm201": lambda b: b.transpose(2, 0, 1),
    "bcast": lambda b: np.broadcast_to(b, (7,) + b.shape),
}


def save_case(ref, name, weights, views=None, raw=True):
    """numpyhelper.Helper.save (numpyhelper.py:144-169, np.savez_compressed at :162): the archive bytes
    the reference writes for ``weights`` (``views[i]``: weights[i] is SAVE_VIEWS[views[i]] of the
    stored base), and the raw_binary bytes (:164-169) where the weights concatenate."""
    helper = ref["Helper"]()
    views = views or [""] * len(weights)
    arrays = [SAVE_VIEWS[v](w) if v else w for w, v in zip(weights, views)]
    d = {"kind": np.array("save"), "name": np.array(name), "views": np.array(json.dumps(views))}
    _store_list(d, "w", weights)
    with tempfile.TemporaryDirectory() as tmp:
        path = helper.save(arrays, os.path.join(tmp, "m.npz"))
        with open(path, "rb") as f:
            d["npz"] = np.frombuffer(f.read(), dtype=np.uint8)
        try:
            if not raw:
                raise ValueError
            path = helper.save(arrays, os.path.join(tmp, "m.bin"), file_type="raw_binary")
            with open(path, "rb") as f:
                d["raw_binary"] = np.frombuffer(f.read(), dtype=np.uint8)
        except ValueError:                  # np.concatenate of 0-d / mismatched ranks
            pass
    return d


def save_cases(ref):
    """The reference's model serialisation bytes: mnist shapes, mixed dtypes, 0-d and empty arrays,
    Fortran order, non-contiguous views, many members, a member past numpy's 16 MiB write size."""
    rng = np.random.default_rng(21)
    mixed = [rng.standard_normal((3, 4)).astype(np.float16), rng.standard_normal(9).astype(np.float32),
             rng.standard_normal((2, 3, 2)), rng.integers(-100, 100, 11).astype(np.int8),
             rng.integers(-2**31, 2**31 - 1, 6).astype(np.int32), rng.integers(-2**62, 2**62, 5),
             rng.integers(0, 255, 13).astype(np.uint8), rng.random(10) < 0.5, np.array(3.25), np.array(7),
             np.zeros((0,), np.float32), np.zeros((2, 0, 3)), (rng.standard_normal(4) + 1j).astype(np.complex64),
             np.array(["ab", "c", "xyz"]), np.arange(4, dtype=">f8"), np.ones((1,) * 20, np.float32)]
    sparse = np.where(rng.random(5_000_000) < 0.004, rng.standard_normal(5_000_000), 0).astype(np.float32)
    return [
        save_case(ref, "save_mnist", _rng_model(rng, MNIST_SHAPES, np.float32)),
        save_case(ref, "save_odd", _rng_model(rng, ODD_SHAPES, np.float32)),
        save_case(ref, "save_mixed_dtypes", mixed),
        save_case(ref, "save_fortran", [np.asfortranarray(rng.standard_normal((31, 17))),
                                        np.asfortranarray(rng.integers(0, 9, (5, 6, 7)).astype(np.int32))]),
        save_case(ref, "save_views", [rng.standard_normal((40, 60)).astype(np.float32),
                                      rng.standard_normal((30, 9)).astype(np.float32),
                                      np.arange(50, dtype=np.int64), rng.standard_normal((4, 5, 6)),
                                      np.arange(5, dtype=np.float32)],
                  ["T", "cols3", "rev", "perm201", "bcast"]),
        save_case(ref, "save_70_members", [rng.standard_normal(int(rng.integers(1, 40))).astype(np.float32)
                                           for _ in range(70)]),
        save_case(ref, "save_sparse_20MB", [sparse, np.arange(300_000, dtype=np.int64) // 7], raw=False),
        save_case(ref, "save_empty_model", []),
    ]


def main():
    global OUT
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    if "--out" in sys.argv:          # tools/verify_golden.py regenerates into a scratch directory
        OUT = sys.argv[sys.argv.index("--out") + 1]
    ref = _import_reference()
    os.makedirs(OUT, exist_ok=True)
    if only == "sf":      # regenerate just these fixtures; the others stay byte-identical
        return _write(sf_cases(ref), merge=True)
    if only == "helpers":
        return _write(helper_cases(ref), merge=True)
    if only == "mixed":
        return _write(mixed_cases(ref), merge=True)
    if only == "power_norm":
        return _write([helper_power_norm(ref, np.random.default_rng(9))], merge=True)
    if only == "edge":
        return _write(edge_cases(ref), merge=True)
    if only == "f16opt":
        return _write(f16_fedopt_cases(ref), merge=True)
    if only == "narrow":
        return _write(narrow_cases(ref), merge=True)
    if only == "numex":
        return _write(numex_cases(ref), merge=True)
    if only == "save":
        return _write(save_cases(ref), merge=True)
    if only == "reduce":
        return _write(reduce_cases(ref) + mixed_cases(ref)[-2:], merge=True)
    cases = []
    cases.append(helper_kat(ref))
    rng = np.random.default_rng(1)
    cases.append(helper_ops(ref, rng))
    # FedAvg ------------------------------------------------------------------------
    rng = np.random.default_rng(2)
    cases.append(fedavg_case(ref, "fedavg_mnist_k2", rng, MNIST_SHAPES, np.float32, rng.integers(1, 5001, 2)))
    for K in (1, 2, 3, 8, 17):
        cases.append(fedavg_case(ref, f"fedavg_odd_k{K}", rng, ODD_SHAPES, np.float32, rng.integers(1, 5001, K)))
    cases.append(fedavg_case(ref, "fedavg_f64_k3", rng, ODD_SHAPES, np.float64, rng.integers(1, 5001, 3)))
    cases.append(fedavg_case(ref, "fedavg_bigN_k5", rng, ODD_SHAPES, np.float32,
                             rng.integers(5_000_000, 20_000_000, 5)))
    cases.append(fedavg_case(ref, "fedavg_int64_k3", rng, ODD_SHAPES, np.int64, rng.integers(1, 5001, 3), int_vals=True))
    cases.append(fedavg_case(ref, "fedavg_int32_k3", rng, ODD_SHAPES, np.int32, rng.integers(1, 5001, 3), int_vals=True))
    cases.append(fedavg_case(ref, "fedavg_skipbad_k4", rng, ODD_SHAPES, np.float32, rng.integers(1, 5001, 4), bad_index=2))
    cases.append(fedavg_case(ref, "fedavg_empty", rng, ODD_SHAPES, np.float32, []))
    cases.append(fedavg_case(ref, "fedavg_tiny_k6", rng, [(1000,)], np.float32, rng.integers(1, 5001, 6), special="tiny"))
    cases.append(fedavg_case(ref, "fedavg_wide_k6", rng, [(1000,)], np.float32, rng.integers(1, 5001, 6), special="wide"))
    cases.append(fedavg_case(ref, "fedavg_flat_k8", rng, [(4099,)], np.float32, rng.integers(1, 5001, 8)))
    # FedOpt ------------------------------------------------------------------------
    rng = np.random.default_rng(3)
    for opt in ("adam", "yogi", "adagrad"):
        params = None if opt == "adam" else {"serveropt": opt}
        cases.append(fedopt_case(ref, f"fedopt_{opt}_3r", rng, ODD_SHAPES,
                                 [list(rng.integers(1, 5001, 3)) for _ in range(3)], params))
        cases.append(fedopt_case(ref, f"fedopt_{opt}_lr1e-2_k8", rng, [(2053,)],
                                 [list(rng.integers(1, 5001, 8)), list(rng.integers(1, 5001, 5))],
                                 {"serveropt": opt, "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "tau": 1e-3}))
    cases.append(fedopt_case(ref, "fedopt_adam_k1", rng, ODD_SHAPES, [[17], [4000]]))
    cases.append(fedopt_case(ref, "fedopt_adam_f64old", rng, ODD_SHAPES, [list(rng.integers(1, 5001, 4))],
                             None, old_dtype=np.float64))
    cases.append(fedopt_case(ref, "fedopt_adam_int_tensors", rng, [(7,), (3, 4)], [[5, 9, 2], [4, 4]], None,
                             int_tensor=True))
    cases.append(fedopt_case(ref, "fedopt_yogi_int_tensors", rng, [(7,), (3, 4)], [[5, 9], [3]], {"serveropt": "yogi"},
                             int_tensor=True))
    cases.append(fedopt_case(ref, "fedopt_badparam_int_lr", rng, ODD_SHAPES, [[10, 20]], {"learning_rate": 1}))
    cases.append(fedopt_case(ref, "fedopt_badparam_key", rng, ODD_SHAPES, [[10, 20]], {"momentum": 0.5}))
    cases.append(fedopt_case(ref, "fedopt_badopt", rng, ODD_SHAPES, [[10, 20]], {"serveropt": "sgd"}))

    rng = np.random.default_rng(5)
    cases.append(fedavg_mixed_case(ref, "fedavg_mixed_int_k5", rng, rng.integers(1, 5001, 5)))

    cases += reduce_cases(ref)

    cases += sf_cases(ref)
    cases += helper_cases(ref)
    cases += mixed_cases(ref)
    cases.append(helper_power_norm(ref, np.random.default_rng(9)))
    cases += edge_cases(ref)
    cases += numex_cases(ref)
    cases += f16_fedopt_cases(ref)
    cases += narrow_cases(ref)
    cases += save_cases(ref)
    _write(cases, merge=False)


def _write(cases, merge):
    manifest = []
    if merge:
        with open(os.path.join(OUT, "manifest.json")) as f:
            manifest = [n for n in json.load(f)["cases"] if n not in {str(c["name"]) for c in cases}]
    for c in cases:
        name = str(c["name"])
        # the save fixtures hold large, compressible inputs: compressed on disk (np.load reads both)
        (np.savez_compressed if name.startswith("save_") else np.savez)(os.path.join(OUT, name + ".npz"), **c)
        manifest.append(name)
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump({"generator": "tools/gen_golden.py", "numpy": np.__version__, "cases": manifest}, f, indent=1)
    total = sum(os.path.getsize(os.path.join(OUT, n + ".npz")) for n in manifest)
    print(f"wrote {len(manifest)} fixtures, {total / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
