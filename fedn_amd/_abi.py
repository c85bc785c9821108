"""ctypes binding of ``libfedagg.so`` (C ABI declared in ``include/fedagg.h``).

The library is the product path: if it is missing or fails to load, every entry
point raises :class:`FedAggLibraryError`. There is no CPU fallback.

``torch`` is imported before the library is opened so the HIP runtime that
PyTorch-ROCm already loaded (SONAME ``libamdhip64.so.7``) is the one the library
binds to; streams and device pointers handed over from torch are then valid in it.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libfedagg.so"
LIB_PATH = os.path.join(_HERE, LIB_NAME)

# element type codes (enum fa_dtype)
FA_NONE, FA_F32, FA_F64, FA_BF16, FA_F16, FA_I32, FA_I64 = -1, 0, 1, 2, 3, 4, 5
FA_I8, FA_I16, FA_U8, FA_U16, FA_U32, FA_U64 = 6, 7, 8, 9, 10, 11
# status codes (enum fa_status)
FA_OK, FA_EINVAL, FA_EDTYPE, FA_EHIP = 0, 1, 2, 3
# server optimizers (enum fa_serveropt)
FA_ADAM, FA_YOGI, FA_ADAGRAD = 0, 1, 2
FA_PG_FIRST, FA_PG_FINAL = 1, 2
(FA_EW_AXPBY, FA_EW_MUL, FA_EW_DIV, FA_EW_SQRT, FA_EW_SQUARE, FA_EW_SIGN, FA_EW_FILL, FA_EW_POW, FA_EW_IPOW, FA_EW_IFOLD,
 FA_EW_NFOLD) = range(11)
(FA_TUNE_STRIPS, FA_TUNE_UNROLL, FA_TUNE_NT, FA_TUNE_FASTDIV, FA_TUNE_LANETAB, FA_TUNE_GRID, FA_TUNE_READ,
 FA_TUNE_BLOCK, FA_TUNE_SUM_NOSTORE, FA_TUNE_NT_STORE, FA_TUNE_FASTDIV64, FA_TUNE_TILEMAP, FA_TUNE_OPT_NT,
 FA_TUNE_OPT_NOSTORE, FA_TUNE_OPT_STORE, FA_TUNE_OPT_COAL, FA_TUNE_NARROW, FA_TUNE_LDS, FA_TUNE_WPE, FA_TUNE_OPT_MV, FA_TUNE_AUTO_GEOM,
 FA_TUNE_OPT_MIX, FA_TUNE_OPT_BURST, FA_TUNE_OPT_G, FA_TUNE_OPT_WIN_PERIOD, FA_TUNE_OPT_WIN_W, FA_TUNE_OPT_WIN_MODE,
 FA_TUNE_AVG_WIN_PERIOD, FA_TUNE_AVG_WIN_W, FA_TUNE_AVG_WIN_MODE, FA_TUNE_OPT_WIN_PROD,
 FA_TUNE_OPT_QUAD) = range(32)

EXPORTS = {
    # name: (restype, argtypes)
    "fa_abi_version": (ctypes.c_int, []),
    "fa_last_error": (ctypes.c_char_p, []),
    "fa_last_kernel": (ctypes.c_char_p, []),
    "fa_promote": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "fa_fedavg_fold": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int,                       # agg, agg_dtype
        ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,       # updates, upd_dtype
        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_int,  # n, N, K
        ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),     # P, init, stream
    "fa_fedavg_fold_host": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int,                       # agg (pinned host), agg_dtype
        ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,       # updates (pinned host), upd_dtype
        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_int,  # n, N, K
        ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),     # P, init, stream
    "fa_fedopt_step_host": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int,                       # old (pinned host), old_dtype
        ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,       # updates (pinned host), upd_dtype
        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_int,  # n, N, K
        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,  # m_in, m_in_dtype, m_out, m_out_dtype
        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,  # v_in, v_in_dt, v_out, out, state_dt
        ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,  # opt, lr, b1, b2, tau
        ctypes.c_int64, ctypes.c_void_p]),                   # P, stream
    "fa_fedopt_step": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int,                       # old, old_dtype
        ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,       # updates, upd_dtype
        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_int,  # n, N, K
        ctypes.c_void_p, ctypes.c_int,                       # pg, flags
        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,      # m_in, m_in_dtype, m_out
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,   # v_in, v_out, out
        ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,  # opt, lr, b1, b2, tau
        ctypes.c_int64, ctypes.c_void_p]),                   # P, stream
    "fa_fedopt_step_ex": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int,                       # old, old_dtype
        ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,       # updates, upd_dtype
        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_int,  # n, N, K
        ctypes.c_void_p, ctypes.c_int,                       # pg, flags
        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,  # m_in, m_in_dtype, m_out, m_out_dtype
        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,  # v_in, v_in_dt, v_out, out, state_dt
        ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,  # opt, lr, b1, b2, tau
        ctypes.c_int64, ctypes.c_void_p]),                   # P, stream
    "fa_weighted_sum": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int,                       # acc, acc_dtype
        ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,       # updates, upd_dtype
        ctypes.POINTER(ctypes.c_double), ctypes.c_int,       # w, K
        ctypes.c_int64, ctypes.c_void_p]),                   # P, stream
    "fa_running_mean": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,      # g, dtype, m
        ctypes.c_double, ctypes.c_double, ctypes.c_double,   # a, b, T
        ctypes.c_int64, ctypes.c_void_p]),                   # P, stream
    "fa_elementwise": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int64,
                                      ctypes.c_void_p]),
    "fa_norm1_work": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int]),
    "fa_norm1": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "fa_cast": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]),
    "fa_ipc_get_handle": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "fa_ipc_open": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_void_p)]),
    "fa_ipc_close": (ctypes.c_int, [ctypes.c_void_p]),
    "fa_copy_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "fa_push": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                               ctypes.c_void_p, ctypes.c_void_p]),           # ..., release_rec, stream
    "fa_fedavg_fold_push": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p]),  # release_rec, stream
    "fa_device_xccs": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "fa_peer_enable": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "fa_host_device_ptr": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "fa_host_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "fa_host_unregister": (ctypes.c_int, [ctypes.c_void_p]),
}
# measurement / tuning entry points: libfedagg_probe.so only (include/fedagg_probe.h)
PROBE_EXPORTS = {
    "fa_tune": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "fa_stream_sum": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int64,
                                     ctypes.c_void_p]),
    "fa_stream_copy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "fa_stream_read_blocks": (ctypes.c_int64, [ctypes.c_int64]),
    "fa_stream_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
}

ABI_VERSION = 8
IPC_HANDLE_BYTES = 64    # FA_IPC_HANDLE_BYTES
RELEASE_WORDS = 8        # FA_RELEASE_WORDS; enum fa_release_word:
FA_REL_MASK, FA_REL_ARRIVED, FA_REL_LAUNCHES, FA_REL_MISSES, FA_REL_SEEN, FA_REL_EXPECT = range(6)


class FedAggLibraryError(ImportError):
    """libfedagg.so is missing or unusable: the HIP path cannot run (no fallback)."""


class FedAggError(RuntimeError):
    """A libfedagg entry point returned a nonzero status."""

    def __init__(self, status, message):
        super().__init__(f"libfedagg status {status}: {message}")
        self.status = status


_lock = threading.Lock()
_lib = None
_probe = None
_active = None          # the probe library, while a tool or test measures with it (use_probe)
PROBE_PATH = os.path.join(_HERE, "libfedagg_probe.so")


def lib_path():
    return os.environ.get("FEDN_AMD_LIB", LIB_PATH)


def _open(path, exports):
    import torch  # noqa: F401  (binds the library to torch's HIP runtime)

    if not os.path.exists(path):
        raise FedAggLibraryError(
            f"{path} not found: build it first (python -c 'import __graft_entry__ as g; g.build()' "
            "or python -m fedn_amd.build). The HIP library is required; there is no CPU fallback.")
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:
        raise FedAggLibraryError(f"cannot load {path}: {e}") from e
    for name, (res, args) in exports.items():
        try:
            fn = getattr(lib, name)
        except AttributeError as e:
            raise FedAggLibraryError(f"{path} does not export {name}") from e
        fn.restype = res
        fn.argtypes = args
    ver = lib.fa_abi_version()
    if ver != ABI_VERSION:
        raise FedAggLibraryError(f"{path}: ABI version {ver}, expected {ABI_VERSION}; rebuild it")
    return lib


def load():
    """The library entry points run in: libfedagg.so (opened once, thread-safe), or the probe
    library while ``use_probe`` is in effect."""
    global _lib
    if _active is not None:
        return _active
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _lib = _open(lib_path(), EXPORTS)
        return _lib


def load_probe():
    """libfedagg_probe.so: the same kernels plus fa_tune and the probe kernels (measurement only)."""
    global _probe
    with _lock:
        if _probe is None:
            _probe = _open(PROBE_PATH, {**EXPORTS, **PROBE_EXPORTS})
        return _probe


class use_probe:
    """Route every ops.* call of this process to the probe library (tools/, A/B tests):
    ``_abi.use_probe()`` for the rest of the process, or ``with _abi.use_probe(): ...``."""

    def __init__(self):
        global _active
        self._prev = _active
        _active = load_probe()

    def __enter__(self):
        return _active

    def __exit__(self, *exc):
        global _active
        _active = self._prev


def check(status):
    if status != FA_OK:
        msg = load().fa_last_error()
        raise FedAggError(status, msg.decode(errors="replace") if msg else "")


def ptr_array(ptrs):
    arr = (ctypes.c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = ctypes.c_void_p(int(p))
    return arr


def int64_array(vals):
    arr = (ctypes.c_int64 * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr


def double_array(vals):
    arr = (ctypes.c_double * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = float(v)
    return arr
