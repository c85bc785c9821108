"""Per-tensor path of the plug-ins: client updates that differ from the running model in dtype
or in broadcastable shape — numpy's promotion and broadcasting, replayed on the GPU.

The uniform-round pipelines (staging.py, multidev.py) pack a model into one buffer per dtype
group and fold every client with one launch per group, which needs every update to carry the
first update's shapes and dtypes. FEDn's numpy helper does not need that:
``np.add(x, n*(y-x)/N)`` (numpyhelper.py:32) folds a float64 client into a float32 model and
returns float64, turns an int64 model folded with a float32 client into float64, and
broadcasts a (1,) tensor against (n,); ``subtract`` (numpyhelper.py:44-56) does the same for
FedOpt's pseudo-gradient (fedopt.py:91-94); ``zip`` truncates to the shorter model. When a
round meets such an update, the pipeline hands its state to the classes here, which keep one
device tensor per model tensor and replay numpy's rules tensor by tensor:

* result dtypes and shapes come from numpy itself, evaluated on EMPTY arrays — type
  inference only, no element is computed on the host — so the promotion table, the weak
  python-scalar rules for n and N, and numpy's errors (non-broadcastable shapes, a python int
  that does not fit an integer dtype) are numpy's own;
* operands are widened and broadcast on the GPU by ``fa_cast`` (exact conversions, or int ->
  float64 rounded to nearest, the conversion numpy's ufunc loop performs);
* the arithmetic is the same libfedagg kernels: ``fa_fedavg_fold`` for increment_average,
  ``fa_elementwise(AXPBY)`` for subtract, ``fa_fedopt_step`` (K = 0, FINAL) for the server step.

Every check runs before any launch, so an update numpy would refuse leaves the state untouched,
as the reference's list comprehension either completes or raises before the assignment.
"""
import numpy as np
import torch

from . import ops, reuse

_NARROW = {np.dtype(t) for t in (np.int8, np.int16, np.uint8, np.uint16, np.uint32, np.uint64)}
_SUPPORTED = {np.dtype(t) for t in (np.float16, np.float32, np.float64, np.int32, np.int64)} | _NARROW


def per_tensor_dtypes(dtypes):
    """Whether a layout holds tensors only the per-tensor path folds (8 / 16-bit and unsigned
    integers: fa_cast + fa_elementwise IFOLD / NFOLD; the fused kernels take f16..f64 / i32 / i64),
    or bool tensors, whose fold numpy refuses (boolean subtract) before anything changes."""
    return any(np.dtype(d) in _NARROW or np.dtype(d) == np.bool_ for d in dtypes)


def _int_fold_kind(d, n):
    """How an integer difference of dtype ``d`` is multiplied by num_examples ``n``
    (numpyhelper.py:32, ``n * (y - x)``): "ifold" in float64 (a float n, or numpy promoting the
    product to float64), "int" in int32 / int64 (the fused kernel's integer first fold), or
    "nfold" wrapping in a narrow / unsigned dtype (a python int n, weak, takes d's dtype)."""
    if float_n(n):
        return "ifold"
    if d in (np.dtype(np.int32), np.dtype(np.int64)):
        return "int"
    p = np.multiply(n, _e(d)).dtype                # raises OverflowError as numpy does
    if p == np.float64:
        return "ifold"
    if p != d:
        raise TypeError(f"a {type(n).__name__} num_examples times a {d} difference ({p}) is not supported")
    if abs(int(n)) >= 1 << 53:
        raise TypeError(f"num_examples {n} is too large for the {d} fold")
    return "nfold"


def np_dtype(t):
    """numpy dtype of a torch dtype, for type inference (bf16 is defined as its f32 upcast)."""
    if t == torch.bfloat16:
        return np.dtype(np.float32)
    return ops.numpy_dtype(t)


def meta_of(tensors):
    """[(shape, numpy dtype)] of device tensors."""
    return [(tuple(t.shape), np_dtype(t.dtype)) for t in tensors]


def host_meta(arrays):
    out = []
    for a in arrays:
        a = np.asarray(a)
        out.append((tuple(a.shape), a.dtype))
    return out


def _e(dt):
    return np.empty(0, dtype=dt)


def fold_plan(xs, ys, n, N):
    """numpyhelper.increment_average(x, y, n, N) per tensor pair (numpyhelper.py:32), from
    metadata: [(difference dtype, result dtype, result shape)], zip-truncated. Raises what numpy
    raises (broadcasting, integer overflow of n/N), and TypeError for dtypes libfedagg lacks."""
    plan = []
    for (xshape, xdt), (yshape, ydt) in zip(xs, ys):
        shape = tuple(np.broadcast_shapes(xshape, yshape))
        x0 = _e(xdt)
        d = np.subtract(_e(ydt), x0)
        t = np.true_divide(np.multiply(n, d), N)
        r = np.add(x0, t)
        if d.dtype not in _SUPPORTED or xdt not in _SUPPORTED or ydt not in _SUPPORTED:
            raise TypeError(f"unsupported dtypes for the fold: model {xdt}, update {ydt}")
        if d.dtype.kind in "iu":
            _int_fold_kind(d.dtype, n)
        plan.append((d.dtype, r.dtype, shape))
    return plan


def float_n(n):
    """True when numpy multiplies an integer difference by ``n`` in float64 (a python float or numpy
    float num_examples) rather than in the integer dtype (a python / numpy int). n == 1.0 gives the
    same bits either way (the integer product by 1 is the difference itself)."""
    return not isinstance(n, (int, np.integer)) and n != 1.0


def int_float_n(dtypes, nfolds, n):
    """Whether folding an update with num_examples ``n`` into a running model that is still the
    first update (``nfolds == 0``) multiplies an INTEGER difference by a float n — the fused
    kernels fold integer tensors with an integer n only, so such a fold runs per tensor."""
    return nfolds == 0 and float_n(n) and any(np.dtype(d).kind == "i" for d in dtypes)


def sub_plan(ys, olds):
    """numpyhelper.subtract(next, old) = next*1.0 + old*(-1.0) per tensor (numpyhelper.py:44-56):
    [(result dtype, shape)], zip-truncated; float16 / float32 / float64 results (fa_elementwise)."""
    plan = []
    for (yshape, ydt), (oshape, odt) in zip(ys, olds):
        shape = tuple(np.broadcast_shapes(yshape, oshape))
        r = np.add(np.multiply(_e(ydt), 1.0), np.multiply(_e(odt), -1.0))
        if ydt not in _SUPPORTED or odt not in _SUPPORTED or r.dtype not in (np.float16, np.float32, np.float64):
            raise TypeError(f"unsupported dtypes for the pseudo-gradient: update {ydt}, global model {odt}")
        plan.append((r.dtype, shape))
    return plan


def converted(t, dtype, shape, stream):
    """``t`` broadcast to ``shape`` and widened to ``dtype`` (a new device tensor; fa_cast)."""
    out = torch.empty(shape, dtype=dtype, device=t.device)
    ops.cast(out, t, stream=stream)
    return out


def _as(t, dtype, shape, stream):
    """``t`` itself when it already has ``dtype``, ``shape`` and is contiguous, else a converted copy."""
    if t.dtype == dtype and tuple(t.shape) == tuple(shape) and t.is_contiguous():
        return t
    return converted(t, dtype, shape, stream)


def upload(arrays, device, stream):
    """Host arrays -> device tensors (one per model tensor) on ``stream``."""
    out = []
    with torch.cuda.device(device), torch.cuda.stream(stream):
        for a in arrays:
            a = np.asarray(a)
            if a.dtype not in _SUPPORTED:
                raise TypeError(f"unsupported dtype {a.dtype}")
            out.append(reuse.watch(torch.from_numpy(a if a.flags.c_contiguous else a.copy()).to(device)))   # keeps 0-d shapes
    return out


def tensor_views(layout, flats, tensors=None):
    """Per-tensor views (model order, model shapes) of group-flat device tensors ``flats``
    ({group dtype: flat tensor}) laid out by ``layout``."""
    out = [None] * len(layout.shapes)
    for dt in layout.groups:
        f = flats[dt]
        for i, off in layout.members[dt]:
            out[i] = f[off:off + layout.sizes[i]].view(layout.shapes[i])
    return out


def u8_flats(layout, dev_u8):
    """{group dtype: flat typed view} of a layout-packed uint8 device buffer."""
    out = {}
    for dt in layout.groups:
        off = layout.group_byte_offset[dt]
        n = layout.group_elems[dt]
        out[dt] = dev_u8[off:off + n * dt.itemsize].view(ops.torch_dtype(dt))
    return out


def gather_flats(layout, bounds, devices, slices, device):
    """Group-flat tensors on ``device`` assembled from per-device parameter slices
    (``slices[d][dt]`` = device d's [lo, hi) of group dt, multidev.py's layout)."""
    out = {}
    for dt in layout.groups:
        rdt = slices[0][dt].dtype
        flat = torch.empty(layout.group_elems[dt], dtype=rdt, device=device)
        for d in range(len(devices)):
            lo, hi = bounds[dt][d]
            if hi > lo:
                flat[lo:hi].copy_(slices[d][dt])
        out[dt] = flat
    return out


class TensorFedAvg:
    """The running FedAvg model as one device tensor per model tensor (numpyhelper.py:32 with
    numpy's promotion and broadcasting). ``tensors`` start the state; ``owned`` says whether
    they may be written in place (False: views of a staged update, copied on first write)."""

    def __init__(self, device, stream, tensors, owned):
        self.device = torch.device(device)
        self.stream = stream
        self.x = list(tensors)
        self.owned = [bool(owned)] * len(self.x)
        self.hold = []

    def meta(self):
        return meta_of(self.x)

    def fold(self, ys, n, N, plan=None):
        """Fold update ``ys`` (device tensors, model order) with num_examples n, running total N."""
        if plan is None:
            plan = fold_plan(self.meta(), meta_of(ys), n, N)
        self.hold.append(ys)                     # inputs stay alive until the round's result
        new = []
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            for (d1, r, shape), x, y, own in zip(plan, self.x, ys, self.owned):
                td = ops.torch_dtype(d1)
                if d1.kind == "f":               # fold in the promoted float dtype, in place
                    xc = x if (own and x.dtype == td and tuple(x.shape) == shape and x.is_contiguous()) \
                        else converted(x, td, shape, self.stream)
                    yc = _as(y, td, shape, self.stream)
                    ops.fedavg_fold(xc.view(-1), [yc.view(-1)], [n], [N], init=False, stream=self.stream)
                    new.append(xc)
                else:                            # integer difference (numpy's wrapping int subtract)
                    xc = _as(x, td, shape, self.stream)
                    yc = _as(y, td, shape, self.stream)
                    out = torch.empty(shape, dtype=torch.float64, device=self.device)
                    kind = _int_fold_kind(d1, n)
                    if kind == "ifold":              # n * d in float64, / N, + x (fa_elementwise IFOLD)
                        ops.elementwise("ifold", out.view(-1), xc.view(-1), yc.view(-1), float(n), float(N),
                                        stream=self.stream)
                    elif kind == "nfold":            # n * d wrapping in the narrow dtype (NFOLD)
                        ops.elementwise("nfold", out.view(-1), xc.view(-1), yc.view(-1), float(int(n)), float(N),
                                        stream=self.stream)
                    else:                            # int multiply by n, then true_divide to float64
                        ops.fedavg_fold(out.view(-1), [xc.view(-1), yc.view(-1)], [0, n], [1, N], init=True,
                                        stream=self.stream)
                    new.append(out)
        self.x = new
        self.owned = [True] * len(new)

    def result(self):
        """The model as new host arrays (caller-owned)."""
        self.stream.synchronize()
        return [t.to("cpu").numpy() for t in self.x]


class TensorFedOpt:
    """FedOpt's pseudo-gradient loop (fedopt.py:89-94) and server step (fedopt.py:151-258) per
    tensor, for rounds whose updates differ from the global model or from each other in dtype
    or broadcastable shape. ``old`` = per-tensor device tensors of the global model;
    ``pg`` = the pseudo-gradient folded so far (device tensors) or None."""

    def __init__(self, device, stream, old, pg=None):
        self.device = torch.device(device)
        self.stream = stream
        self.old = list(old)
        self.acc = None if pg is None else TensorFedAvg(device, stream, pg, owned=True)
        self.hold = []

    def add(self, ys, n, N):
        """One more update (device tensors, model order) into the pseudo-gradient."""
        splan = sub_plan(meta_of(ys), meta_of(self.old))
        fplan = None
        if self.acc is not None:
            fplan = fold_plan(self.acc.meta(), [(shape, d) for d, shape in splan], n, N)
        self.hold.append(ys)
        subs = []
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            for (d, shape), y, o in zip(splan, ys, self.old):
                td = ops.torch_dtype(d)
                yc, oc = _as(y, td, shape, self.stream), _as(o, td, shape, self.stream)
                s = torch.empty(shape, dtype=td, device=self.device)
                ops.elementwise("axpby", s.view(-1), yc.view(-1), oc.view(-1), 1.0, -1.0, stream=self.stream)
                subs.append(s)
        if self.acc is None:                     # fedopt.py:91: pg = subtract(next, old)
            self.acc = TensorFedAvg(self.device, self.stream, subs, owned=True)
        else:                                    # fedopt.py:93-94
            self.acc.fold(subs, n, N, plan=fplan)

    def server_step(self, m, v, params, fp32=False):
        """Apply adam / yogi / adagrad (fedopt.py:139-258) to the pseudo-gradient. ``m``, ``v``:
        the state as per-tensor device tensors or None. Returns (model host arrays, new m, new v).
        Inputs of different broadcastable shapes are broadcast to their common shape first (the
        state keeps that shape; every value is numpy's). ``fp32``: the fp32-state mode
        (aggregators.fedopt_f32state): for a tensor whose global model is float32, m, v and the new
        model are stored in float32 (the f64 step's results rounded once, fa_fedopt_step_ex), as
        the fused path stores them — the model's dtypes do not change with the round's path."""
        opt = params["serveropt"]
        if opt not in ("adam", "yogi", "adagrad"):
            raise ValueError(f"Unsupported server optimizer: {opt}")
        pg = self.acc.x
        L = min(len(pg), len(self.old), len(m) if m is not None else len(pg), len(v) if v is not None else len(pg))
        plan = []
        for i in range(L):
            p, o = pg[i], self.old[i]
            shapes = [tuple(p.shape), tuple(o.shape)]
            if m is not None:
                shapes.append(tuple(m[i].shape))
            if v is not None:
                shapes.append(tuple(v[i].shape))
            B = tuple(np.broadcast_shapes(*shapes))
            if p.dtype not in (torch.float16, torch.float32, torch.float64):
                raise TypeError(f"pseudo-gradient dtype {p.dtype} is not supported by the server step")
            # a half pg comes from half updates over a half model (numpy's half loops, the kernel's
            # CF16 step); otherwise a half model enters the step widened to f32, which is exact
            odt = o.dtype if p.dtype == torch.float16 or o.dtype != torch.float16 else torch.float32
            if np_dtype(odt) in _NARROW:         # old + f64 step: numpy widens the narrow model exactly
                odt = torch.float64
            if odt not in (torch.float16, torch.float32, torch.float64, torch.int32, torch.int64):
                raise TypeError(f"global-model dtype {o.dtype} is not supported by the server step")
            # the update dtype handed to fa_fedopt_step only fixes the pg dtype (K = 0)
            upd = odt if odt in (torch.int32, torch.int64) else p.dtype
            if ops.fedopt_dtypes(upd, odt, None)[0] != p.dtype:
                raise TypeError(f"pseudo-gradient {p.dtype} over a {o.dtype} global model is not supported")
            mdt = None if m is None else m[i].dtype
            if mdt is not None and mdt not in (torch.float16, torch.float32, torch.float64):
                raise TypeError(f"m dtype {mdt} is not supported")
            f32 = fp32 and o.dtype == torch.float32
            plan.append((B, odt, upd, torch.float32 if f32 else ops.fedopt_dtypes(upd, odt, mdt)[1],
                         torch.float32 if f32 else torch.float64))
        model, new_m, new_v = [], [], []
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            for i, (B, odt, upd, m_dt, sdt) in enumerate(plan):
                s = self.stream
                pb = _as(pg[i], pg[i].dtype, B, s)
                ob = _as(self.old[i], odt, B, s)
                mi = None if m is None else _as(m[i], m[i].dtype, B, s)
                vdt = torch.float64 if v is None or v[i].dtype != torch.float32 else torch.float32
                vi = None if v is None else _as(v[i], vdt, B, s)
                m_out = torch.empty(B, dtype=m_dt, device=self.device)
                v_out = torch.empty(B, dtype=sdt, device=self.device)
                out = torch.empty(B, dtype=sdt, device=self.device)
                fl = lambda t: None if t is None else t.view(-1)  # noqa: E731
                ops.fedopt_step(ob.view(-1), [], [], [], first=False, final=True, pg=pb.view(-1), m_in=fl(mi),
                                m_out=m_out.view(-1), v_in=fl(vi), v_out=v_out.view(-1), out=out.view(-1),
                                serveropt=opt, learning_rate=params["learning_rate"], beta1=params["beta1"],
                                beta2=params["beta2"], tau=params["tau"], stream=s, upd_dtype=upd)
                model.append(out)
                new_m.append(m_out)
                new_v.append(v_out)
        self.stream.synchronize()
        return [t.to("cpu").numpy() for t in model], new_m, new_v
