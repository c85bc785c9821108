"""Tensor-level entry points over the C ABI (device buffers are PyTorch-ROCm tensors).

These are thin: validate shapes/devices, collect raw pointers, call libfedagg on the
tensors' current HIP stream, raise :class:`FedAggError` on a nonzero status.

dtype rules mirror numpy's for the reference expressions:
see :func:`fold_result_dtype` and :func:`fedopt_dtypes`.
"""
import contextlib
import ctypes

import numpy as np
import torch

from . import _abi
from ._abi import FedAggError  # noqa: F401  (the status exception, re-exported for the pipelines)

_TORCH_TO_FA = {
    torch.float32: _abi.FA_F32,
    torch.float64: _abi.FA_F64,
    torch.bfloat16: _abi.FA_BF16,
    torch.float16: _abi.FA_F16,
    torch.int32: _abi.FA_I32,
    torch.int64: _abi.FA_I64,
    # narrow / unsigned integers: fa_cast and the IFOLD / NFOLD folds only (the per-tensor path)
    torch.int8: _abi.FA_I8,
    torch.int16: _abi.FA_I16,
    torch.uint8: _abi.FA_U8,
    torch.uint16: _abi.FA_U16,
    torch.uint32: _abi.FA_U32,
    torch.uint64: _abi.FA_U64,
}
_FA_TO_TORCH = {v: k for k, v in _TORCH_TO_FA.items()}
_NP_TO_TORCH = {
    np.dtype(np.float32): torch.float32,
    np.dtype(np.float64): torch.float64,
    np.dtype(np.float16): torch.float16,
    np.dtype(np.int32): torch.int32,
    np.dtype(np.int64): torch.int64,
    np.dtype(np.int8): torch.int8,
    np.dtype(np.int16): torch.int16,
    np.dtype(np.uint8): torch.uint8,
    np.dtype(np.uint16): torch.uint16,
    np.dtype(np.uint32): torch.uint32,
    np.dtype(np.uint64): torch.uint64,
    np.dtype(np.bool_): torch.bool,        # staged / returned as is; no kernel takes it (numpy never folds bool)
}
_TORCH_TO_NP = {v: k for k, v in _NP_TO_TORCH.items()}


def fa_dtype(t):
    dt = t.dtype if isinstance(t, torch.Tensor) else t
    if isinstance(dt, np.dtype) or (isinstance(dt, type) and issubclass(dt, np.generic)):
        dt = torch_dtype(dt)
    try:
        return _TORCH_TO_FA[dt]
    except KeyError:
        raise TypeError(f"dtype {dt} is not supported by libfedagg") from None


def torch_dtype(np_dtype):
    try:
        return _NP_TO_TORCH[np.dtype(np_dtype)]
    except KeyError:
        raise TypeError(f"numpy dtype {np_dtype} is not supported by libfedagg") from None


def numpy_dtype(torch_dt):
    if torch_dt == torch.bfloat16:
        raise TypeError("bfloat16 has no numpy dtype")
    return _TORCH_TO_NP[torch_dt]


def fold_result_dtype(agg_dt, upd_dt, nfolds=1):
    """dtype of ``np.add(x, n*(y-x)/N)`` for x: agg_dt, y: upd_dt (torch dtypes).

    bf16 (no numpy counterpart) accumulates in f32. Integer inputs become f64 on the
    first fold (numpy true_divide). ``nfolds == 0`` means "no fold yet" (plain alias).
    """
    if nfolds == 0:
        return upd_dt
    ints = (torch.int32, torch.int64)
    if agg_dt in ints or upd_dt in ints:
        return torch.float64
    if torch.float64 in (agg_dt, upd_dt):
        return torch.float64
    if agg_dt == torch.float16 and upd_dt == torch.float16:
        return torch.float16
    return torch.float32


def _stream_handle(t, stream):
    if stream is None:
        stream = torch.cuda.current_stream(t.device)
    return ctypes_stream(stream)


def ctypes_stream(stream):
    return int(stream.cuda_stream) if stream is not None else 0


def _check_dev(name, t, P, device):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be a device (cuda/hip) tensor, got {t.device}")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.numel() != P:
        raise ValueError(f"{name} has {t.numel()} elements, expected {P}")


def fedavg_fold(agg, updates, n, N, init, stream=None):
    """FedAvg fold on device (``fa_fedavg_fold``): numpyhelper.py:32 replayed in queue order.

    agg      flat device tensor (running model; written)
    updates  sequence of flat device tensors of the same length
    n, N     per-update num_examples and running totals (python numbers)
    init     True: agg := updates[0] then fold updates[1:]; False: fold all into agg
    """
    lib = _abi.load()
    K = len(updates)
    if len(n) != K or len(N) != K:
        raise ValueError("n and N must have one entry per update")
    P = agg.numel()
    dev = agg.device
    _check_dev("agg", agg, P, None)
    upd_dt = updates[0].dtype if K else agg.dtype
    for i, u in enumerate(updates):
        _check_dev(f"updates[{i}]", u, P, dev)
        if u.dtype != upd_dt:
            raise TypeError("all updates in one fold call must share a dtype")
    with _on(dev):        # launch on the tensors' device (multi-GPU processes)
        st = _stream_handle(agg, stream)
        rc = lib.fa_fedavg_fold(agg.data_ptr(), fa_dtype(agg), _abi.ptr_array([u.data_ptr() for u in updates]),
                                fa_dtype(upd_dt), _abi.double_array(n), _abi.double_array(N), K, P, int(bool(init)), st)
    _abi.check(rc)
    return agg


def fedavg_fold_ptrs(agg, ptrs, upd_dtype, n, N, init, stream=None):
    """:func:`fedavg_fold` with the client table given as device addresses (ints) of ``agg.numel()``
    elements of ``upd_dtype`` each, on ``agg``'s device: the pipelines' own staging buffers, whose
    extent they guarantee (no per-update tensor view or check)."""
    lib = _abi.load()
    K = len(ptrs)
    if len(n) != K or len(N) != K:
        raise ValueError("n and N must have one entry per update")
    P = agg.numel()
    _check_dev("agg", agg, P, None)
    args = (agg.data_ptr(), fa_dtype(agg), (ctypes.c_void_p * max(1, K))(*ptrs), fa_dtype(upd_dtype),
            (ctypes.c_double * max(1, K))(*n), (ctypes.c_double * max(1, K))(*N), K, P, int(bool(init)))
    if agg.device.index == torch.cuda.current_device():      # the common case: no device switch
        rc = lib.fa_fedavg_fold(*args, _stream_handle(agg, stream))
    else:
        with _on(agg.device):
            rc = lib.fa_fedavg_fold(*args, _stream_handle(agg, stream))
    _abi.check(rc)
    return agg


def weighted_sum(acc, updates, w, stream=None):
    """``acc[i] += updates[k][i] * w[k]`` for k in order (``fa_weighted_sum``): the loop of the
    reference's server-function example aggregate (server_functions.py:58-67), numpy rounding."""
    lib = _abi.load()
    K = len(updates)
    if len(w) != K:
        raise ValueError("w must have one entry per update")
    P = acc.numel()
    dev = acc.device
    _check_dev("acc", acc, P, None)
    upd_dt = updates[0].dtype if K else acc.dtype
    for i, u in enumerate(updates):
        _check_dev(f"updates[{i}]", u, P, dev)
        if u.dtype != upd_dt:
            raise TypeError("all updates in one weighted_sum call must share a dtype")
    with _on(dev):
        st = _stream_handle(acc, stream)
        rc = lib.fa_weighted_sum(acc.data_ptr(), fa_dtype(acc), _abi.ptr_array([u.data_ptr() for u in updates]),
                                 fa_dtype(upd_dt), _abi.double_array(w), K, P, st)
    _abi.check(rc)
    return acc


def running_mean(g, m, a, b, T, stream=None):
    """``g = (g*a + m*b)/T`` in place (``fa_running_mean``): one step of the reference's
    incremental server-function example (sf_incremental_aggregation.py:36-37)."""
    lib = _abi.load()
    P = g.numel()
    _check_dev("g", g, P, None)
    _check_dev("m", m, P, g.device)
    if m.dtype != g.dtype:
        raise TypeError(f"running_mean: model dtype {m.dtype} differs from the running model's {g.dtype}")
    with _on(g.device):
        st = _stream_handle(g, stream)
        rc = lib.fa_running_mean(g.data_ptr(), fa_dtype(g), m.data_ptr(), float(a), float(b), float(T), P, st)
    _abi.check(rc)
    return g


_OPTS = {"adam": _abi.FA_ADAM, "yogi": _abi.FA_YOGI, "adagrad": _abi.FA_ADAGRAD}


def promote(a, b):
    """numpy result dtype for the FedOpt elementwise pairs (torch dtypes; None = absent)."""
    if a is None:
        a, b = b, None
    if b is None:
        return torch.float32 if a == torch.bfloat16 else a
    a = torch.float32 if a == torch.bfloat16 else a
    b = torch.float32 if b == torch.bfloat16 else b
    if a == b:
        return a
    if torch.float64 in (a, b):
        return torch.float64
    return torch.float32


def fedopt_dtypes(upd_dt, old_dt, m_dt):
    """(pg dtype, m_out dtype) for fedopt.py's expressions; v and out are always f64.
    Integer updates: ``next*1.0 + old*(-1.0)`` is float64 in numpy (int array * python float)."""
    pg = torch.float64 if upd_dt in (torch.int32, torch.int64) else promote(upd_dt, old_dt)
    return pg, promote(m_dt, pg)


def fedopt_step(old, updates, n, N, *, first, final, pg=None, m_in=None, m_out=None, v_in=None, v_out=None,
                out=None, serveropt="adam", learning_rate=1e-3, beta1=0.9, beta2=0.99, tau=1e-4, stream=None,
                upd_dtype=None):
    """Fused FedOpt step on device (``fa_fedopt_step``), fedopt.py:74-118 + 151-258.

    ``upd_dtype``: dtype of the round's client updates; required when ``updates`` is empty
    (a server step on an accumulated ``pg``), because it fixes the pseudo-gradient dtype."""
    lib = _abi.load()
    if serveropt not in _OPTS:
        raise ValueError(f"Unsupported server optimizer: {serveropt}")
    K = len(updates)
    P = old.numel()
    dev = old.device
    _check_dev("old", old, P, None)
    if K:
        upd_dt = updates[0].dtype
    elif upd_dtype is not None:
        upd_dt = upd_dtype
    elif pg is not None and pg.dtype == torch.float64 and old.dtype != torch.float64:
        raise ValueError("fedopt_step without updates needs upd_dtype (pg is float64, old is not)")
    else:
        upd_dt = pg.dtype if pg is not None else old.dtype
    for i, u in enumerate(updates):
        _check_dev(f"updates[{i}]", u, P, dev)
        if u.dtype != upd_dt:
            raise TypeError("all updates in one call must share a dtype")
    if pg is not None and pg.dtype != fedopt_dtypes(upd_dt, old.dtype, None)[0]:
        raise TypeError(f"pg must be {fedopt_dtypes(upd_dt, old.dtype, None)[0]} for {upd_dt} updates over a "
                        f"{old.dtype} model")
    for name, t in (("pg", pg), ("m_in", m_in), ("m_out", m_out), ("v_in", v_in), ("v_out", v_out), ("out", out)):
        if t is not None:
            _check_dev(name, t, P, dev)
    if v_in is not None and v_in.dtype not in (torch.float64, torch.float32):
        raise TypeError("v must be float64 (fedopt.py:171: np.ones(...) * tau**2), or float32 (fp32-state mode)")
    # the storage dtype of the server state: out's (float64: the reference's flow; float32: the
    # fp32-state mode, fa_fedopt_step_ex — v and the model stored as f32, m as f32 or numpy's dtype)
    state_dt = out.dtype if out is not None else torch.float64
    if state_dt not in (torch.float64, torch.float32):
        raise TypeError("out must be float64 (the reference's model dtype) or float32 (fp32-state mode)")
    pg_dt, m_np = fedopt_dtypes(upd_dt, old.dtype, None if m_in is None else m_in.dtype)
    if final:
        if m_out is None or v_out is None or out is None:
            raise ValueError("final step needs m_out, v_out and out")
        if v_out.dtype != state_dt:
            raise TypeError(f"v_out must be {state_dt}, like out")
        if m_out.dtype != m_np and not (state_dt == torch.float32 and m_out.dtype == torch.float32):
            raise TypeError(f"output dtypes: m_out {m_np}" + (" or float32" if state_dt == torch.float32 else "") +
                            f", v_out/out {state_dt}")
    flags = (_abi.FA_PG_FIRST if first else 0) | (_abi.FA_PG_FINAL if final else 0)
    ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    with _on(dev):
        st = _stream_handle(old, stream)
        rc = lib.fa_fedopt_step_ex(
            old.data_ptr(), fa_dtype(old), _abi.ptr_array([u.data_ptr() for u in updates]), fa_dtype(upd_dt),
            _abi.double_array(n), _abi.double_array(N), K, ptr(pg), flags,
            ptr(m_in), _abi.FA_NONE if m_in is None else fa_dtype(m_in), ptr(m_out),
            fa_dtype(m_out) if m_out is not None else fa_dtype(m_np),
            ptr(v_in), _abi.FA_F64 if v_in is None else fa_dtype(v_in), ptr(v_out), ptr(out),
            fa_dtype(state_dt), _OPTS[serveropt], float(learning_rate), float(beta1), float(beta2), float(tau), P, st)
    _abi.check(rc)


def fedopt_step_raw(old_ptr, old_dt, upd_ptrs, upd_dt, n, N, P, *, first, final, pg_ptr=0, m_in=None, m_out=None,
                    v_in=None, v_out=None, out_ptr=0, state_dt=torch.float64, serveropt="adam", learning_rate=1e-3,
                    beta1=0.9, beta2=0.99, tau=1e-4, stream=None, device=None):
    """:func:`fedopt_step` with the global model, the client table, pg and the new model given as
    device addresses of ``P`` elements each — pinned host memory's device addresses included (a
    small round folded zero-copy, staging.FedOptPipeline) — and no tensor view per update; m / v
    are device tensors as in :func:`fedopt_step`. For the pipelines' own buffers, whose extents
    and dtypes they guarantee (the dtype rules are the same; the C ABI checks the pairs)."""
    if serveropt not in _OPTS:
        raise ValueError(f"Unsupported server optimizer: {serveropt}")
    K = len(upd_ptrs)
    if len(n) != K or len(N) != K:
        raise ValueError("fedopt_step_raw: one n and N per update")
    if final and (m_out is None or v_out is None or not out_ptr):
        raise ValueError("final step needs m_out, v_out and out")
    _, m_np = fedopt_dtypes(upd_dt, old_dt, None if m_in is None else m_in.dtype)
    flags = (_abi.FA_PG_FIRST if first else 0) | (_abi.FA_PG_FINAL if final else 0)
    ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    with _on(device):
        rc = _abi.load().fa_fedopt_step_ex(
            int(old_ptr), fa_dtype(old_dt), _abi.ptr_array([int(u) for u in upd_ptrs]), fa_dtype(upd_dt),
            _abi.double_array(n), _abi.double_array(N), K, int(pg_ptr), flags,
            ptr(m_in), _abi.FA_NONE if m_in is None else fa_dtype(m_in), ptr(m_out),
            fa_dtype(m_out.dtype if m_out is not None else m_np),
            ptr(v_in), _abi.FA_F64 if v_in is None else fa_dtype(v_in), ptr(v_out), int(out_ptr),
            fa_dtype(state_dt), _OPTS[serveropt], float(learning_rate), float(beta1), float(beta2), float(tau), int(P),
            ctypes_stream(stream))
    _abi.check(rc)


def cast(out, x, stream=None):
    """``out[...] = x`` broadcast to ``out.shape`` and widened to ``out.dtype`` (``fa_cast``):
    numpy's implicit operand preparation for a binary ufunc whose operands differ in dtype or
    broadcastable shape. ``out`` is contiguous; ``x`` any strided device tensor."""
    lib = _abi.load()
    if out.device != x.device:
        raise ValueError(f"cast: {x.device} -> {out.device}")
    if not out.is_contiguous():
        raise ValueError("cast: out must be contiguous")
    oshape = tuple(out.shape)
    xshape = tuple(x.shape)
    if len(xshape) > len(oshape):
        raise ValueError(f"cast: cannot broadcast {xshape} to {oshape}")
    # right-align x's dims to out's (numpy broadcasting); stride 0 where x has extent 1
    lead = len(oshape) - len(xshape)
    strides = [0] * lead
    for d, (xs, st) in enumerate(zip(xshape, x.stride())):
        os_ = oshape[lead + d]
        if xs == os_:
            strides.append(st if xs != 1 else 0)
        elif xs == 1:
            strides.append(0)
        else:
            raise ValueError(f"cast: cannot broadcast {xshape} to {oshape}")
    # drop extent-1 dims, then merge adjacent dims that are contiguous in both (keeps ndim
    # within the kernel's limit)
    dims = [(s, t) for s, t in zip(oshape, strides) if s != 1] or [(1, 0)]
    ms, mt = [dims[0][0]], [dims[0][1]]
    for s, t in dims[1:]:
        if mt[-1] == t * s:
            ms[-1] *= s
            mt[-1] = t
        else:
            ms.append(s)
            mt.append(t)
    if len(ms) > 8:
        raise ValueError(f"cast: {len(ms)} non-mergeable dimensions (kernel limit 8)")
    with _on(out.device):
        st = _stream_handle(out, stream)
        rc = lib.fa_cast(out.data_ptr(), fa_dtype(out), x.data_ptr(), fa_dtype(x), len(ms), _abi.int64_array(ms),
                         _abi.int64_array(mt), st)
    _abi.check(rc)
    return out


def _probe_lib():
    """The measurement entry points exist only in libfedagg_probe.so (include/fedagg_probe.h)."""
    lib = _abi.load()
    if lib is not _abi._probe:
        raise RuntimeError("measurement / tuning entry point: call fedn_amd._abi.use_probe() first "
                           "(libfedagg_probe.so; the product libfedagg.so has no knobs)")
    return lib


def stream_copy(dst, src, stream=None):
    lib = _probe_lib()
    st = _stream_handle(src, stream)
    _abi.check(lib.fa_stream_copy(dst.data_ptr(), src.data_ptr(), src.numel() * src.element_size(), st))


def stream_sum(out, bufs, stream=None):
    """Measurement: out = sum of bufs (fp32) with the FedAvg kernel's traversal."""
    lib = _probe_lib()
    st = _stream_handle(out, stream)
    _abi.check(lib.fa_stream_sum(out.data_ptr(), _abi.ptr_array([b.data_ptr() for b in bufs]), len(bufs),
                                 out.numel(), st))


def stream_read(src, sink, stream=None):
    lib = _probe_lib()
    st = _stream_handle(src, stream)
    _abi.check(lib.fa_stream_read(src.data_ptr(), src.numel() * src.element_size(), sink.data_ptr(), st))


def stream_read_sink(src):
    lib = _probe_lib()
    blocks = lib.fa_stream_read_blocks(src.numel() * src.element_size())
    return torch.empty(max(1, blocks) * 16, dtype=torch.uint8, device=src.device)


_KNOBS = {"strips": _abi.FA_TUNE_STRIPS, "unroll": _abi.FA_TUNE_UNROLL, "nt": _abi.FA_TUNE_NT,
          "fastdiv": _abi.FA_TUNE_FASTDIV, "lanetab": _abi.FA_TUNE_LANETAB,
          "grid": _abi.FA_TUNE_GRID, "read": _abi.FA_TUNE_READ,
          "block": _abi.FA_TUNE_BLOCK, "sum_nostore": _abi.FA_TUNE_SUM_NOSTORE,
          "nt_store": _abi.FA_TUNE_NT_STORE, "fastdiv64": _abi.FA_TUNE_FASTDIV64,
          "tilemap": _abi.FA_TUNE_TILEMAP, "opt_nt": _abi.FA_TUNE_OPT_NT, "opt_nostore": _abi.FA_TUNE_OPT_NOSTORE,
          "opt_store": _abi.FA_TUNE_OPT_STORE, "opt_coal": _abi.FA_TUNE_OPT_COAL, "narrow": _abi.FA_TUNE_NARROW,
          "lds": _abi.FA_TUNE_LDS, "wpe": _abi.FA_TUNE_WPE,
          "opt_mv": _abi.FA_TUNE_OPT_MV, "auto_geom": _abi.FA_TUNE_AUTO_GEOM,
          "opt_mix": _abi.FA_TUNE_OPT_MIX, "opt_burst": _abi.FA_TUNE_OPT_BURST,
          "opt_g": _abi.FA_TUNE_OPT_G, "opt_win_period": _abi.FA_TUNE_OPT_WIN_PERIOD, "opt_win_w": _abi.FA_TUNE_OPT_WIN_W,
          "opt_win_mode": _abi.FA_TUNE_OPT_WIN_MODE, "avg_win_period": _abi.FA_TUNE_AVG_WIN_PERIOD,
          "avg_win_w": _abi.FA_TUNE_AVG_WIN_W, "avg_win_mode": _abi.FA_TUNE_AVG_WIN_MODE,
          "opt_win_prod": _abi.FA_TUNE_OPT_WIN_PROD,
          "opt_quad": _abi.FA_TUNE_OPT_QUAD}


def tune(**knobs):
    """Set launch knobs (fa_tune): FedAvg strips, unroll, nt, fastdiv, ...; and fastdiv64 (CF64's division). Results never change (every setting is bit-identical)."""
    lib = _probe_lib()
    for k, v in knobs.items():
        _abi.check(lib.fa_tune(_KNOBS[k], int(v)))


_EW = {"axpby": _abi.FA_EW_AXPBY, "mul": _abi.FA_EW_MUL, "div": _abi.FA_EW_DIV, "sqrt": _abi.FA_EW_SQRT,
       "square": _abi.FA_EW_SQUARE, "sign": _abi.FA_EW_SIGN, "fill": _abi.FA_EW_FILL, "pow": _abi.FA_EW_POW,
       "ipow": _abi.FA_EW_IPOW, "ifold": _abi.FA_EW_IFOLD, "nfold": _abi.FA_EW_NFOLD}


def elementwise(op, out, x=None, y=None, a=0.0, b=0.0, stream=None):
    """numpyhelper primitive on device tensors (``fa_elementwise``); see include/fedagg.h."""
    lib = _abi.load()
    P = out.numel()
    _check_dev("out", out, P, None)
    for name, t in (("x", x), ("y", y)):
        if t is not None:
            _check_dev(name, t, P, out.device)
    if P == 0:                      # an empty tensor: nothing to compute (its buffers may be null)
        for t in (out, x, y):
            if t is not None:
                fa_dtype(t)         # the same dtype refusal as a non-empty call
        if op not in _EW:
            raise ValueError(f"unknown elementwise op {op}")
        return out
    with _on(out.device):
        st = _stream_handle(out, stream)
        rc = lib.fa_elementwise(_EW[op], out.data_ptr(), fa_dtype(out), 0 if x is None else x.data_ptr(),
                                fa_dtype(out) if x is None else fa_dtype(x), 0 if y is None else y.data_ptr(),
                                _abi.FA_NONE if y is None else fa_dtype(y), float(a), float(b), P, st)
    _abi.check(rc)
    return out


def norm1(x, matrix, stream=None):
    """np.linalg.norm(x, 1) of one device tensor (``fa_norm1``): a 0-dim f64 device tensor.
    ``matrix``: x is 2-D (max column sum of |x|), else the sum of |x| over all elements."""
    lib = _abi.load()
    if not x.is_contiguous():
        raise ValueError("norm1: x must be contiguous")
    rows, cols = (x.shape[0], x.shape[1]) if matrix else (1, x.numel())
    work = torch.empty(max(1, int(lib.fa_norm1_work(rows, cols, int(matrix)))), dtype=torch.float64, device=x.device)
    out = torch.empty((), dtype=torch.float64, device=x.device)
    with _on(x.device):
        st = _stream_handle(x, stream)
        rc = lib.fa_norm1(out.data_ptr(), x.data_ptr(), fa_dtype(x), rows, cols, int(matrix), work.data_ptr(), st)
    _abi.check(rc)
    return out


# ---- peer transport of the sliced all-gather (include/fedagg.h fa_ipc_* / fa_copy_async) ----------

def ipc_handle(t):
    """(handle bytes, byte offset) exporting device tensor ``t``'s memory to another process."""
    import ctypes
    lib = _abi.load()
    h = ctypes.create_string_buffer(_abi.IPC_HANDLE_BYTES)
    off = ctypes.c_uint64(0)
    with _on(t.device):
        _abi.check(lib.fa_ipc_get_handle(t.data_ptr(), h, ctypes.byref(off)))
    return h.raw, int(off.value)


def ipc_open(handle, offset, device):
    """Map a peer process's buffer on ``device``: (base, device pointer); unmap with ipc_close(base)."""
    import ctypes
    lib = _abi.load()
    if len(handle) != _abi.IPC_HANDLE_BYTES:
        raise ValueError(f"IPC handle must be {_abi.IPC_HANDLE_BYTES} bytes")
    base, ptr = ctypes.c_void_p(), ctypes.c_void_p()
    with _on(device):
        _abi.check(lib.fa_ipc_open(ctypes.create_string_buffer(handle, len(handle)), int(offset), ctypes.byref(base),
                                   ctypes.byref(ptr)))
    return int(base.value or 0), int(ptr.value or 0)


def ipc_close(base, device):
    lib = _abi.load()
    with _on(device):
        _abi.check(lib.fa_ipc_close(base))


def copy_async(dst_ptr, src, nbytes, stream):
    """``nbytes`` of device tensor ``src`` (from its start) to device address ``dst_ptr`` on ``stream``
    (an IPC mapping of a peer's buffer, or another device's tensor): the DMA engines drive the link."""
    lib = _abi.load()
    if nbytes > src.numel() * src.element_size():
        raise ValueError("copy_async: more bytes than the source holds")
    with _on(src.device):
        _abi.check(lib.fa_copy_async(int(dst_ptr), src.data_ptr(), int(nbytes), ctypes_stream(stream)))


def copy_ptr_async(dst_ptr, src_ptr, nbytes, stream, device):
    """``nbytes`` from address ``src_ptr`` to ``dst_ptr`` (host or device) on ``stream``: one
    hipMemcpyAsync, without a tensor per call."""
    with _on(device):
        _abi.check(_abi.load().fa_copy_async(int(dst_ptr), int(src_ptr), int(nbytes), ctypes_stream(stream)))


def fedavg_fold_push(agg_ptr, ptrs, n, N, P, init, dst_ptrs, stream, device, release_rec=None):
    """The fp32 fold of ``P`` elements into device address ``agg_ptr`` whose kernel also stores the
    result to every address in ``dst_ptrs`` (``fa_fedavg_fold_push``: fold and all-gather push in
    one pass); client table and destinations as device addresses, 16-B aligned. ``release_rec``: a
    :func:`release_record` tensor on ``device`` the release grid records its XCDs in (or None).
    Returns whether a release grid was launched (there were destinations and something to fold)."""
    K = len(ptrs)
    if len(n) != K or len(N) != K:
        raise ValueError("n and N must have one entry per update")
    nd = len(dst_ptrs)
    rec = _release_ptr(release_rec, device)
    with _on(device):
        _abi.check(_abi.load().fa_fedavg_fold_push(
            int(agg_ptr), (ctypes.c_void_p * max(1, K))(*ptrs), (ctypes.c_double * max(1, K))(*n),
            (ctypes.c_double * max(1, K))(*N), K, int(P), int(bool(init)),
            (ctypes.c_void_p * max(1, nd))(*[int(p) for p in dst_ptrs]), nd, rec, ctypes_stream(stream)))
    return K > 0 and P > 0 and nd > 0    # a release grid ran after the peer stores


def push(dst_ptrs, src, nbytes, stream, release_rec=None):
    """``nbytes`` of device tensor ``src`` (from its start) to every device address in ``dst_ptrs``
    on ``stream`` with ONE kernel (``fa_push``): the source is read once, each destination written
    over its own link (IPC mappings of peers' buffers, or other devices' buffers in-process).
    Returns whether a release grid was launched (something was stored)."""
    lib = _abi.load()
    if nbytes > src.numel() * src.element_size():
        raise ValueError("push: more bytes than the source holds")
    n = len(dst_ptrs)
    rec = _release_ptr(release_rec, src.device)
    with _on(src.device):
        _abi.check(lib.fa_push((ctypes.c_void_p * max(1, n))(*[int(p) for p in dst_ptrs]), n, src.data_ptr(),
                               int(nbytes), rec, ctypes_stream(stream)))
    return n > 0 and nbytes > 0          # a release grid ran after the stores (fa_push returns before one
    #                                      when there is nothing to store)


def release_record(device):
    """A zeroed release record (include/fedagg.h FA_RELEASE_WORDS uint32 on ``device``) for the
    release grids of :func:`push` / :func:`fedavg_fold_push` on one stream."""
    return torch.zeros(_abi.RELEASE_WORDS, dtype=torch.int32, device=device)


def _release_ptr(rec, device):
    if rec is None:
        return None
    if (rec.dtype != torch.int32 or rec.numel() < _abi.RELEASE_WORDS or not rec.is_contiguous()
            or rec.device != torch.device(device)):
        raise ValueError(f"release record must be {_abi.RELEASE_WORDS} contiguous int32 on {device}")
    return rec.data_ptr()


def read_release_record(rec):
    """The XCD-coverage record of the release grids (synchronises with its device): launches checked,
    launches that missed an XCD, the XCDs seen (mask) and the device's XCD mask."""
    v = [int(x) & 0xFFFFFFFF for x in rec.cpu().tolist()]
    return {"launches": v[_abi.FA_REL_LAUNCHES], "misses": v[_abi.FA_REL_MISSES], "seen_mask": v[_abi.FA_REL_SEEN],
            "expect_mask": v[_abi.FA_REL_EXPECT], "xcds_seen": bin(v[_abi.FA_REL_SEEN]).count("1")}


def device_xccs(device):
    """XCDs (each with its own L2) of ``device``."""
    out = ctypes.c_int(0)
    idx = torch.device(device).index or 0
    _abi.check(_abi.load().fa_device_xccs(int(idx), ctypes.byref(out)))
    return int(out.value)


_NULL_CTX = contextlib.nullcontext()


def _on(device):
    """``torch.cuda.device(device)`` unless it is already the current device (the per-round and
    per-update copy calls of the pipelines pay the context switch only when they need it)."""
    if device is None:
        return _NULL_CTX
    idx = device.index if isinstance(device, torch.device) else torch.device(device).index
    if idx is None or idx == torch.cuda.current_device():
        return _NULL_CTX
    return torch.cuda.device(device)


def peer_enable(dev, peer):
    """Direct access of device ``dev`` to device ``peer``'s memory (in-process multi-GPU)."""
    _abi.check(_abi.load().fa_peer_enable(int(dev), int(peer)))


def last_kernel():
    """The kernel family the calling thread's last fold / FedOpt launch ran (fa_last_kernel)."""
    v = _abi.load().fa_last_kernel()
    return v.decode() if v else ""


def host_device_ptr(host_ptr, device):
    """Device address of page-locked host memory at ``host_ptr`` (raises for pageable memory)."""
    out = ctypes.c_void_p()
    with _on(device):
        _abi.check(_abi.load().fa_host_device_ptr(int(host_ptr), ctypes.byref(out)))
    return int(out.value or 0)


def fedavg_fold_raw(out_ptr, out_dtype, P, ptrs, upd_dtype, n, N, init, stream, device):
    """:func:`fedavg_fold_ptrs` into ``P`` elements of ``out_dtype`` at device address ``out_ptr``
    (e.g. pinned host memory's device address: the model lands on the host with no D2H copy)."""
    K = len(ptrs)
    if len(n) != K or len(N) != K:
        raise ValueError("n and N must have one entry per update")
    with _on(device):
        _abi.check(_abi.load().fa_fedavg_fold(int(out_ptr), fa_dtype(out_dtype), (ctypes.c_void_p * max(1, K))(*ptrs),
                                              fa_dtype(upd_dtype), (ctypes.c_double * max(1, K))(*n),
                                              (ctypes.c_double * max(1, K))(*N), K, int(P), int(bool(init)),
                                              ctypes_stream(stream)))


def fedavg_fold_host(call, n, N):
    """A small round's whole fold (smallround.py): ``call(n, N)`` runs the native pack wait +
    ``fa_fedavg_fold_host`` + stream wait (``_fastpack.fold_host``) with the client table's ``n`` /
    ``N`` and returns its status; FedAggError on a failed one (the C-ABI wrapper level, as every
    fold op here), CodecError if the pack it waited for failed."""
    if len(n) != len(N):
        raise ValueError("n and N must have one entry per update")
    rc = call(n, N)
    if rc == -1:
        from . import codec
        raise codec.CodecError(f"fnpz_gather_wait: {codec.load_lib().fnpz_last_error().decode(errors='replace')}")
    _abi.check(rc)


def fedopt_step_host(call, n, N, *, first=True, final=True):
    """A small FedOpt round's whole step (smallround.SmallFedOptRound): ``call(n, N)`` runs the native
    pack wait + ``fa_fedopt_step_host`` (FIRST | FINAL) + stream wait with the client table's ``n`` /
    ``N``; FedAggError on a failed one (the state untouched: the step writes the buffers the state
    does not hold), CodecError if a pack failed."""
    if len(n) != len(N):
        raise ValueError("n and N must have one entry per update")
    if not (first and final):
        raise ValueError("fedopt_step_host: the one-call round is a FIRST | FINAL step")
    rc = call(n, N)
    if rc == -1:
        from . import codec
        raise codec.CodecError(f"fnpz_gather_wait: {codec.load_lib().fnpz_last_error().decode(errors='replace')}")
    _abi.check(rc)


def host_register(t):
    """Page-lock the memory of host tensor ``t`` (mapped by the caller, e.g. shared memory)."""
    _abi.check(_abi.load().fa_host_register(t.data_ptr(), t.numel() * t.element_size()))


def host_unregister(t):
    _abi.check(_abi.load().fa_host_unregister(t.data_ptr()))


def host_register_ptr(ptr, nbytes):
    """Page-lock ``nbytes`` of host memory at ``ptr`` in place (e.g. a decoded update's numpy array),
    so DMA reads it directly; undo with :func:`host_unregister_ptr` before the memory is freed."""
    _abi.check(_abi.load().fa_host_register(int(ptr), int(nbytes)))


def host_unregister_ptr(ptr):
    _abi.check(_abi.load().fa_host_unregister(int(ptr)))
