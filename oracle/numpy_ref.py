"""CPU ORACLE — test infrastructure only. NOT part of the product path.

A numpy restatement of FEDn's combiner-side aggregation (FEDn v0.33.0), used
  * by ``tests/`` as the parity checker for the HIP kernels,
  * by ``__graft_entry__.smoke()`` as the checker of its one GPU invocation,
  * by ``bench.py`` as the ``cpu_baseline`` leg (``kind: "port"``),
and by nothing else. The product (``fedn_amd``) never imports this module.

Parity PINNED: every function here is checked bit-for-bit (values AND dtypes)
against golden fixtures produced by running the reference itself
(``tools/gen_golden.py`` → ``tests/golden/*.npz``; see ``tests/test_oracle_golden.py``),
including the reference's own known-answer test
(fedn/utils/helpers/tests/test_numpyhelper.py:20-29).

Each function restates one reference expression with the same numpy ops in the
same order (numpy 2 / NEP 50 promotion: Python scalars are "weak", so an fp32
array times a Python int/float stays fp32; ``np.ones`` is fp64).
"""
import math

import numpy as np


# --------------------------------------------------------------------------------------
# numpyhelper primitives — fedn/utils/helpers/plugins/numpyhelper.py
# --------------------------------------------------------------------------------------
def increment_average(m1, m2, n, N):
    """numpyhelper.py:18-32 — per tensor: t = y - x; t = n * t; t = t / N; x + t."""
    out = []
    for x, y in zip(m1, m2):
        t = np.subtract(y, x)
        t = np.multiply(n, t)
        t = np.true_divide(t, N)
        out.append(np.add(x, t))
    return out


def add(m1, m2, a=1.0, b=1.0):
    """numpyhelper.py:34-44 — m1*a + m2*b."""
    return [np.add(np.multiply(x, a), np.multiply(y, b)) for x, y in zip(m1, m2)]


def subtract(m1, m2, a=1.0, b=1.0):
    """numpyhelper.py:46-56 — add(m1, m2, a, -b)."""
    return add(m1, m2, a, -b)


def divide(m1, m2):
    """numpyhelper.py:58-68."""
    return [np.true_divide(x, y) for x, y in zip(m1, m2)]


def multiply(m1, m2):
    """numpyhelper.py:70-80."""
    return [np.multiply(x, y) for x, y in zip(m1, m2)]


def sqrt(m1):
    """numpyhelper.py:82-92."""
    return [np.sqrt(x) for x in m1]


def power(m1, a):
    """numpyhelper.py:94-104."""
    return [np.power(x, a) for x in m1]


def norm(m):
    """numpyhelper.py:106-117 — sum of per-tensor L1 norms."""
    total = 0.0
    for x in m:
        total += np.linalg.norm(x, 1)
    return total


def sign(m):
    """numpyhelper.py:119-127."""
    return [np.sign(x) for x in m]


def ones(m1, a):
    """numpyhelper.py:129-142 — np.ones(shape) (fp64!) times a."""
    return [np.multiply(np.ones(np.shape(x)), a) for x in m1]


# --------------------------------------------------------------------------------------
# FedAvg — fedn/network/combiner/aggregators/fedavg.py:22-83
# --------------------------------------------------------------------------------------
def android_increment_average(model, model_next, num_examples, total_examples):
    """androidhelper.Helper.increment_average, fedn/utils/helpers/plugins/androidhelper.py:21-39:
    one flat float64 array (its load, :78-92)."""
    w = num_examples / total_examples
    return (1 - w) * model + w * model_next


def fedavg_combine(updates, increment=None):
    """Fold ``updates`` = [(arrays, num_examples), ...] in FIFO order.

    Returns (model or None, nr_aggregated_models). Mirrors fedavg.py:47-78: the
    running total is incremented BEFORE the fold (fedavg.py:62), the first update
    is aliased (fedavg.py:65-66), and a fold that raises is skipped while its
    examples stay counted (fedavg.py:75-78).
    """
    increment = increment or increment_average      # the session helper's rule (fedavg.py:68)
    model, nr, total = None, 0, 0
    for arrays, n in updates:
        total += n
        try:
            if nr == 0:
                model = arrays
            else:
                model = increment(model, arrays, n, total)
        except Exception:  # noqa: BLE001  (reference logs and continues)
            continue
        nr += 1
    return model, nr


def fedavg_flat(updates, ns):
    """FedAvg over flat 1-D buffers (bench / large-size parity): same recurrence."""
    model, total = None, 0
    for k, (y, n) in enumerate(zip(updates, ns)):
        total += int(n)
        if k == 0:
            model = y
        else:
            t = np.subtract(y, model)
            t = np.multiply(int(n), t)
            t = np.true_divide(t, total)
            model = np.add(model, t)
    return model


# --------------------------------------------------------------------------------------
# FedOpt — fedn/network/combiner/aggregators/fedopt.py:40-258
# --------------------------------------------------------------------------------------
DEFAULT_FEDOPT = {"serveropt": "adam", "learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
_SCHEMA = {"serveropt": str, "learning_rate": float, "beta1": float, "beta2": float, "tau": float}


class InvalidParameter(Exception):
    pass


def validate_parameters(parameters):
    """fedopt.py:123-137 + fedn/utils/parameters.py:28-51 (isinstance schema check)."""
    if parameters:
        for k, v in parameters.items():
            if k not in _SCHEMA:
                raise InvalidParameter(f"Parameter {k} not in paramter schema")
            if not isinstance(v, _SCHEMA[k]):
                raise InvalidParameter(f"Parameter {k} has invalid type")
    else:
        parameters = {}
    return {**DEFAULT_FEDOPT, **parameters}


class FedOptState:
    """The aggregator-instance state fedopt.py:36-38 (m, v live across rounds)."""

    def __init__(self):
        self.m = None
        self.v = None


def _server_step(state, pg, old, p):
    b1, b2, lr, tau = p["beta1"], p["beta2"], p["learning_rate"], p["tau"]
    opt = p["serveropt"]
    if opt not in ("adam", "yogi", "adagrad"):
        raise ValueError(f"Unsupported server optimizer: {opt}")
    if not state.v:                                              # fedopt.py:170-171 (and twins)
        state.v = ones(pg, math.pow(tau, 2))
    if not state.m:                                              # fedopt.py:173-176
        state.m = multiply(pg, [(1.0 - b1)] * len(pg))
    else:
        state.m = add(state.m, pg, b1, (1.0 - b1))
    sq = power(pg, 2)
    if opt == "adam":                                            # fedopt.py:178-179
        state.v = add(state.v, sq, b2, (1.0 - b2))
    elif opt == "yogi":                                          # fedopt.py:214-217
        s = sign(add(state.v, sq, 1.0, -1.0))
        s = multiply(s, sq)
        state.v = add(state.v, s, 1.0, -(1.0 - b2))
    else:                                                        # fedopt.py:251-252
        state.v = add(state.v, sq, 1.0, 1.0)
    sv = add(sqrt(state.v), ones(state.v, tau))
    t = divide(state.m, sv)
    return add(old, t, 1.0, lr)


def fedopt_combine(state, updates, old, parameters=None):
    """One round of fedopt.Aggregator.combine_models (fedopt.py:40-121).

    updates = [(arrays, num_examples), ...] in FIFO order; ``old`` = the global model
    the clients started from (fedopt.py:90). Returns (model or None, nr_aggregated).
    """
    try:
        p = validate_parameters(parameters)
    except InvalidParameter:
        return None, -1
    pg, nr, total = None, 0, 0
    for arrays, n in updates:
        total += n
        try:
            if nr == 0:
                pg = subtract(arrays, old)
            else:
                pg = increment_average(pg, subtract(arrays, old), n, total)
        except Exception:  # noqa: BLE001
            continue
        nr += 1
    if not pg:
        return None, nr
    try:
        return _server_step(state, pg, old, p), nr
    except Exception:  # noqa: BLE001  (fedopt.py:113-116)
        return None, nr


def fedopt_combine_f32state(state, updates, old, parameters=None):
    """The fp32-STATE mode's definition (fedn_amd.aggregators.fedopt_f32state, SURVEY.md §7 step 5;
    a mode of this build, not a reference behaviour): one fedopt.py round (``fedopt_combine``, i.e.
    fedopt.py:40-121 + 151-258) on the stored float32 state — ``v`` widened exactly to float64, the
    dtype the reference keeps it in — after which m, v and the model of every tensor whose global
    model is float32 are rounded once to float32 (other tensors keep the reference's dtypes).
    ``state`` is updated in place like FedOptState; returns (model or None, nr_aggregated)."""
    st = FedOptState()
    st.m = None if state.m is None else [np.asarray(x) for x in state.m]
    st.v = None if state.v is None else [np.asarray(x).astype(np.float64) for x in state.v]
    model, nr = fedopt_combine(st, updates, old, parameters)
    if model is None:
        return None, nr
    f32 = [np.asarray(o).dtype == np.float32 for o in old]
    rnd = lambda xs: [np.asarray(x).astype(np.float32) if f else x for x, f in zip(xs, f32)]  # noqa: E731
    state.m, state.v = rnd(st.m), rnd(st.v)
    return rnd(model), nr


# --------------------------------------------------------------------------------------
# Control.reduce — fedn/network/controller/control.py:648-693
# --------------------------------------------------------------------------------------
def control_reduce(fetched):
    """``fetched`` = per combiner, the loaded model or None (fetch failed). control.py:662-690:
    the first model is taken after increment_average(None, ...) raises, later ones fold with
    n = 1.0, N = i; a fold that raises REPLACES the running model; i counts fetched models."""
    i, model = 1, None
    for data in fetched:
        if data is not None:
            try:
                if model is None:
                    raise TypeError("'NoneType' object is not iterable")
                model = increment_average(model, data, 1.0, i)
            except Exception:  # noqa: BLE001
                model = data
            i += 1
    return model


# ---------------------------------------------------------------------------------------------
# Server-function aggregation examples (hooks.py:109-143 calls them)
# ---------------------------------------------------------------------------------------------
def sf_weighted_average(previous_global, client_updates):
    """examples/server-functions/server_functions.py:53-68 (ServerFunctions.aggregate).

    ``client_updates``: {client_id: (arrays, metadata)} in arrival order (hooks.py:88-101 stores
    ``[model, metadata]`` lists). Running sum in previous_global's dtypes (np.zeros_like),
    in-place ``+=`` of ``params * num_examples``, then ``/ total_weight``.
    """
    if len(client_updates) == 0:
        return previous_global
    weighted_sum = [np.zeros_like(param) for param in previous_global]
    total_weight = 0
    for _cid, (client_parameters, metadata) in client_updates.items():
        num_examples = metadata.get("num_examples", 1)
        total_weight += num_examples
        for i in range(len(weighted_sum)):
            weighted_sum[i] += client_parameters[i] * num_examples
    return [weighted / total_weight for weighted in weighted_sum]


class SfIncrementalAverage:
    """examples/server-functions/sf_incremental_aggregation.py:10-48 (the aggregation part).

    Note the example never resets ``total_examples`` (:12, :30): the running total carries
    over into later rounds, and so it does here.
    """

    def __init__(self):
        self.global_model = None
        self.total_examples = 0
        self.previous_global = None

    def incremental_aggregate(self, client_id, model, client_metadata, previous_global):
        self.previous_global = previous_global
        num_examples = client_metadata.get("num_examples", 1)
        self.total_examples += num_examples
        if self.global_model is None:
            self.global_model = model
        else:
            for i in range(len(self.global_model)):
                self.global_model[i] = (self.global_model[i] * (self.total_examples - num_examples)
                                        + model[i] * num_examples) / self.total_examples

    def get_incremental_aggregate_model(self):
        ret = self.global_model
        self.global_model = None
        if ret is None:
            return self.previous_global
        return ret
