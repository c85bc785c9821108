"""Load the golden fixtures written by tools/gen_golden.py (data only: inputs + expected outputs)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names(kind=None):
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        names = json.load(f)["cases"]
    if kind is None:
        return names
    out = []
    for n in names:
        with np.load(os.path.join(GOLDEN, n + ".npz"), allow_pickle=False) as z:
            if str(z["kind"]) == kind:
                out.append(n)
    return out


def _list(z, prefix):
    key = f"{prefix}_len"
    if key not in z:
        return None
    return [z[f"{prefix}_t{t}"] for t in range(int(z[key]))]


def _ns(z, key):
    """num_examples as the python numbers the reference saw: int, or float where the case says so."""
    isf = z.get(key + "_isfloat")
    vals = z[key]
    if isf is None:
        return [int(v) for v in vals]
    return [float(v) if f else int(v) for v, f in zip(vals, isf)]


def load_case(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        z = {k: z[k] for k in z.files}
    case = {"name": name, "kind": str(z["kind"]), "raw": z}
    if case["kind"] == "reduce":
        plan = json.loads(str(z["plan"]))
        case["plan"] = plan
        case["models"] = [_list(z, f"c{c}") for c in range(len(plan))]
        case["out"] = None if bool(z["out_none"]) else _list(z, "out")
    if case["kind"] == "sf_wavg":
        K = int(z["K"])
        case["prev"] = _list(z, "prev")
        case["updates"] = {f"client-{k}": (_list(z, f"u{k}"), json.loads(str(z[f"meta{k}"]))) for k in range(K)}
        case["out"] = _list(z, "out")
    if case["kind"] == "sf_inc":
        case["rounds"] = []
        for r in range(int(z["rounds"])):
            K = int(z[f"r{r}_K"])
            case["rounds"].append({
                "prev": _list(z, f"r{r}_prev"),
                "updates": [(f"client-{k}", _list(z, f"r{r}_u{k}"), json.loads(str(z[f"r{r}_meta{k}"])))
                            for k in range(K)],
                "out": _list(z, f"r{r}_out"),
            })
    if case["kind"] in ("helper_fedavg", "helper_fedopt"):
        # a session on a non-numpy helper: one flat array per model (see tools/gen_golden.py helper_case)
        case["helper"] = str(z["helper"])
        case["params"] = json.loads(str(z["params"])) if "params" in z else None
        case["rounds"] = []
        for r in range(int(z["rounds"])):
            K = int(z[f"r{r}_K"])
            ns = [int(v) for v in z[f"r{r}_n"]]
            case["rounds"].append({
                "updates": [(z[f"r{r}_u{k}"], ns[k]) for k in range(K)],
                "old": z[f"r{r}_old"],
                "out": None if bool(z[f"r{r}_out_none"]) else z[f"r{r}_out"],
                "nr": int(z[f"r{r}_nr"]),
                "qsize": int(z[f"r{r}_qsize"]),
                "m": z.get(f"r{r}_m"),
                "v": z.get(f"r{r}_v"),
            })
    if case["kind"] in ("fedavg", "fedopt"):
        case["params"] = json.loads(str(z["params"])) if "params" in z else None
        rounds = []
        for r in range(int(z["rounds"])):
            K = int(z[f"r{r}_K"])
            ns = _ns(z, f"r{r}_n")
            rd = {
                "updates": [(_list(z, f"r{r}_u{k}"), ns[k]) for k in range(K)],
                "old": _list(z, f"r{r}_old"),
                "out": None if bool(z[f"r{r}_out_none"]) else _list(z, f"r{r}_out"),
                "nr": int(z[f"r{r}_nr"]),
                "qsize": int(z[f"r{r}_qsize"]),
                "data_keys": json.loads(str(z[f"r{r}_data_keys"])),
                "m": _list(z, f"r{r}_m"),
                "v": _list(z, f"r{r}_v"),
            }
            rounds.append(rd)
        case["rounds"] = rounds
    return case


def assert_lists_identical(got, want, what=""):
    """Bitwise equality of values (NaN == NaN) and exact dtype/shape equality."""
    assert (got is None) == (want is None), f"{what}: None mismatch"
    if want is None:
        return
    assert len(got) == len(want), f"{what}: {len(got)} tensors vs {len(want)}"
    for i, (g, w) in enumerate(zip(got, want)):
        g = np.asarray(g)
        w = np.asarray(w)
        assert g.dtype == w.dtype, f"{what}[{i}]: dtype {g.dtype} vs {w.dtype}"
        assert g.shape == w.shape, f"{what}[{i}]: shape {g.shape} vs {w.shape}"
        if g.dtype.kind == "f":
            gi = g.view(np.uint64 if g.dtype.itemsize == 8 else (np.uint32 if g.dtype.itemsize == 4 else np.uint16))
            wi = w.view(gi.dtype)
            both_nan = np.isnan(g) & np.isnan(w)
            bad = (gi != wi) & ~both_nan
            assert not bad.any(), (f"{what}[{i}]: {int(bad.sum())} of {g.size} elements differ bitwise; "
                                   f"first at {np.argwhere(bad)[0]}: {g[tuple(np.argwhere(bad)[0])]!r} vs "
                                   f"{w[tuple(np.argwhere(bad)[0])]!r}")
        else:
            np.testing.assert_array_equal(g, w, err_msg=what)
