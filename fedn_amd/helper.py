"""FEDn helper plug-in backed by the native npz codec and the GPU fold — drop-in for
``fedn.utils.helpers.plugins.numpyhelper.Helper`` (numpyhelper.py:10-212) on the methods
FEDn's ``HelperBase`` requires (helperbase.py:4-40) plus its file-type API:

  increment_average(m1, m2, n, N)  numpyhelper.py:18-32, computed by libfedagg (bit-exact)
  save(weights, path=None, file_type="npz")   numpyhelper.py:144-169: np.savez_compressed's
                                              bytes exactly (codec.save_npz; the block-parallel
                                              writer with FEDN_AMD_NPZ_WRITER=blocks)
  load(path, file_type="npz")                 numpyhelper.py:171-189: native inflate (parallel
                                              for archives this codec wrote), members of 8 MiB+
                                              into pinned memory for a multi-GPU combiner;
                                              raw_binary as FEDn
  add / subtract / multiply / divide / sqrt / sign / ones
                                              numpyhelper.py:34-142 on the GPU (fa_elementwise),
                                              numpy's dtype promotion and rounding, so FEDn's
                                              stock fedopt.py runs unchanged on this helper
Inputs may be numpy arrays (results come back as numpy arrays, like numpyhelper) or device
tensors (results stay on the device, so chains of primitives never leave HBM).
  power(m, a) / norm(m)                       numpyhelper.py:94-117 on the GPU (general exponents,
                                              integer powers; the matrix 1-norm for 2-D tensors)
FEDn selects helpers by module name (helpers.py:7-17); install with a shim module
``fedn/utils/helpers/plugins/fednamdhelper.py``.
"""
import os
import tempfile
from io import BytesIO

import numpy as np

from . import codec


# npz members at least this large are decoded into page-locked host memory (0 disables) when the
# combiner aggregates on several GPUs in one process (FEDN_AMD_DEVICES lists more than one; or always
# with FEDN_AMD_DECODE_PINNED=1, never with 0): the multi-device pipeline DMAs such a tensor slice by
# slice straight from where it lies instead of packing it into a pinned slot first
# (multidev.INPLACE_MIN_BYTES). The blocks come from torch's caching host allocator, so a session's
# rounds reuse them without pinning pages again (its blocks round up to a power of two and stay
# cached for the process). One device packs every update anyway, so plain arrays serve it.
DECODE_PINNED_MIN_BYTES = int(os.environ.get("FEDN_AMD_DECODE_PINNED_MIN_BYTES", str(8 << 20)))
_pinned_ok = None


def decode_pinned():
    """Whether :meth:`Helper.load` decodes large members into page-locked memory (see above)."""
    v = os.environ.get("FEDN_AMD_DECODE_PINNED", "auto")
    if v in ("0", "1"):
        return v == "1"
    from .aggregators.fedavg import env_devices
    return len(env_devices() or []) > 1


def pinned_empty(shape, dtype, order="C"):
    """An uninitialised C-ordered array in page-locked host memory (None: no GPU, a Fortran-ordered
    or small member — the caller allocates it as usual). The array keeps its pinned block alive."""
    global _pinned_ok
    dtype = np.dtype(dtype)
    nbytes = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
    if order != "C" or DECODE_PINNED_MIN_BYTES <= 0 or nbytes < DECODE_PINNED_MIN_BYTES:
        return None
    import torch
    if _pinned_ok is None:
        _pinned_ok = torch.cuda.is_available()
    if not _pinned_ok:
        return None
    blk = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    return blk.numpy().view(dtype).reshape(shape)


def npz_writer():
    """Helper.save's npz writer: "numpy" (default: np.savez_compressed's bytes, numpyhelper.py:162) or
    "blocks" (FEDN_AMD_NPZ_WRITER=blocks: the codec's block-parallel archive — np.load reads it, but
    its bytes are not numpy's)."""
    v = os.environ.get("FEDN_AMD_NPZ_WRITER", "numpy")
    if v not in ("numpy", "blocks"):
        raise ValueError(f"FEDN_AMD_NPZ_WRITER={v!r}: expected 'numpy' or 'blocks'")
    return v


def _device():
    from .aggregators.fedavg import default_device
    return default_device()


def _to_dev(x, dev):
    """(device tensor, came_from_numpy)"""
    import torch
    if isinstance(x, torch.Tensor):
        return x.contiguous(), False
    a = np.ascontiguousarray(x)
    if a.dtype.kind not in "fiu" or a.dtype.itemsize > 8:
        raise TypeError(f"fednamdhelper primitives support float and integer arrays, got {a.dtype}")
    return torch.from_numpy(a).to(dev), True


def _np_result(op, xdt, ydt, a, b):
    """numpy's result dtype of numpyhelper's expression for these operand dtypes (empty arrays,
    no data; python scalars are weak): ``x*a + y*b``, ``x*y`` / ``x*a``, ``x/y`` / ``x/a``,
    ``sqrt``, ``sign``; ``ones`` is float64."""
    ex = np.empty(0, xdt)
    ey = None if ydt is None else np.empty(0, ydt)
    with np.errstate(all="ignore"):
        if op == "axpby":
            return (ex * a + ey * b).dtype
        if op == "mul":
            return (ex * (a if ey is None else ey)).dtype
        if op == "div":
            return (ex / (a if ey is None else ey)).dtype
        if op == "sqrt":
            return np.sqrt(ex).dtype
        if op == "sign":
            return np.sign(ex).dtype
    return np.dtype(np.float64)


def _ew_one(op, xd, yd, a, b, dev):
    """One numpyhelper primitive on flat device tensors, numpy's dtypes and rounding.

    float32 / float64 operands run fa_elementwise directly, three float16 arrays in AXPBY its half
    loop. Otherwise (float16 with a scalar or another dtype, 8 / 16 / 32 / 64-bit integers) the op
    is computed in a WIDER float and rounded once to numpy's result dtype r: operands are widened
    exactly (integers to float64 as numpy converts them; float16 to float32), the single op is
    correctly rounded in the wide type (float32 for an r of float16, float64 otherwise) and
    narrowed to r by fa_cast — the same value as the op rounded once in r (a correctly rounded op
    rounded again is innocuous: 24 >= 2*11+2, 53 >= 2*24+2). A python scalar meets a float16 array
    as a float16 (numpy's weak scalar), so it is rounded to half first. AXPBY with one float16
    operand rounds that operand's product in half first (numpy's order), then adds in r. Integer
    results (integer multiply / sign) are not supported (FedAggError)."""
    import torch

    from . import ops
    from ._abi import FedAggError
    kf = (torch.float32, torch.float64)
    xdt = ops.numpy_dtype(xd.dtype)
    ydt = None if yd is None else ops.numpy_dtype(yd.dtype)
    if op == "fill":
        o = torch.empty(xd.numel(), dtype=torch.float64, device=dev)
        ops.elementwise("fill", o, None, None, a, b)
        return o
    if xd.dtype in kf and (yd is None or yd.dtype in kf):          # the direct kernels
        odt = ops.promote(xd.dtype, yd.dtype) if (op == "axpby" or (op in ("mul", "div") and yd is not None)) \
            else xd.dtype
        o = torch.empty(xd.numel(), dtype=odt, device=dev)
        ops.elementwise(op, o, xd, yd, a, b)
        return o
    if op == "axpby" and xd.dtype == torch.float16 and yd is not None and yd.dtype == torch.float16:
        o = torch.empty(xd.numel(), dtype=torch.float16, device=dev)
        ops.elementwise(op, o, xd, yd, a, b)
        return o
    r = _np_result(op, xdt, ydt, a, b)
    if r.kind != "f" or r not in (np.float16, np.float32, np.float64):
        raise FedAggError(2, f"fednamdhelper: {op} on {xdt}" + (f" / {ydt}" if ydt is not None else "") +
                             f" gives {r}; integer results are not supported on the GPU helper")
    rt = ops.torch_dtype(r)
    wide = torch.float32 if r == np.float16 else torch.float64

    def widen(t, to=None):
        to = to or wide
        return t if t.dtype == to else ops.cast(torch.empty(t.numel(), dtype=to, device=dev), t)

    def narrow(t):
        return t if t.dtype == rt else ops.cast(torch.empty(t.numel(), dtype=rt, device=dev), t)

    half = lambda v: float(np.float16(v))  # noqa: E731  (a python float meeting a half array)
    if op == "axpby":
        if rt not in kf:                    # a half result needs three half operands (handled above)
            raise FedAggError(2, f"fednamdhelper: add on {xdt} / {ydt} is not supported")
        # numpy's order: each product in its own dtype (operand * weak python float), then the sum
        # in r. A product whose dtype is r is left to the final kernel (operand widened exactly);
        # another (float16 or float32 beside a wider r) is rounded in its dtype first
        parts = []
        for t, c in ((xd, a), (yd, b)):
            pd = _np_result("mul", ops.numpy_dtype(t.dtype), None, c, 0)
            parts.append((t, c) if pd == r else (_ew_one("mul", t, None, c, 0, dev), 1.0))
        (px, ca), (py, cb) = parts
        o = torch.empty(xd.numel(), dtype=rt, device=dev)
        ops.elementwise("axpby", o, widen(px, rt), widen(py, rt), ca, cb)
        return o
    if yd is None and op in ("mul", "div") and xd.dtype == torch.float16:
        a = half(a)
    wx = widen(xd)
    wy = None if yd is None else widen(yd)
    o = torch.empty(xd.numel(), dtype=wide, device=dev)
    ops.elementwise(op, o, wx, wy, a, b)
    return narrow(o)


def _back(t, host, shape):
    return t.to("cpu").numpy().reshape(shape) if host else t.reshape(shape)


CACHED_LAYOUTS = 2     # model layouts whose staging slots increment_average keeps


class Helper:
    def __init__(self):
        self.name = "fednamdhelper"
        self._cache = {}

    def increment_average(self, m1, m2, n, N):
        """One FedAvg fold of two models on the GPU (same rounding and promotion as
        numpyhelper.py:32). Stock FEDn calls this once per client (fedavg.py:68), so the pinned /
        device staging slots and streams are kept per (device, model layout) and reused: a call
        allocates only its result block."""
        from .aggregators.fedavg import default_device
        from .layout import Layout
        from .staging import FedAvgPipeline

        m1, m2 = list(m1), list(m2)
        dev = default_device()
        key = (str(dev), Layout.of(m1).signature())
        slots, streams = self._cache.pop(key, (None, None))
        pipe = FedAvgPipeline(dev, m1, nslots=2, slots=slots, streams=streams, batch=False)
        pipe.add(m2, n, N)
        out = pipe.result()
        self._cache[key] = (pipe.slots, (pipe.copy, pipe.d2h))
        while len(self._cache) > CACHED_LAYOUTS:              # oldest layout out
            self._cache.pop(next(iter(self._cache)))
        return out

    # ---- numpyhelper primitives on the GPU (numpyhelper.py:34-142) ----------------------------
    def _ew(self, op, m1, m2=None, a=0.0, b=0.0):
        import torch

        from . import ops
        dev = _device()
        out = []
        for i, x in enumerate(m1):
            shape = tuple(x.shape)
            xd, host = _to_dev(x, dev)
            xd = xd.reshape(-1)
            y = None if m2 is None else m2[i]
            yd = None
            if isinstance(y, np.generic):          # numpy scalars (0-d results) are arrays here
                y = np.asarray(y)
            ai = a
            if y is not None and not isinstance(y, (int, float)):
                if tuple(y.shape) != shape:
                    raise ValueError(f"operands could not be broadcast together with shapes {shape} {tuple(y.shape)}")
                yd, yhost = _to_dev(y, dev)
                yd = yd.reshape(-1)
                host = host or yhost
            elif y is not None:
                ai = float(y)                    # multiply/divide by a python scalar (weak)
            out.append(_back(_ew_one(op, xd, yd, ai, b, dev), host, shape))
        return out

    def add(self, m1, m2, a=1.0, b=1.0):
        """m1*a + m2*b (numpyhelper.py:34-44)."""
        return self._ew("axpby", m1, m2, a, b)

    def subtract(self, m1, m2, a=1.0, b=1.0):
        """m1*a - m2*b (numpyhelper.py:46-56)."""
        return self.add(m1, m2, a, -b)

    def divide(self, m1, m2):
        return self._ew("div", m1, m2)

    def multiply(self, m1, m2):
        return self._ew("mul", m1, m2)

    def sqrt(self, m1):
        return self._ew("sqrt", m1)

    def power(self, m1, a):
        """np.power(x, a) per tensor (numpyhelper.py:94-104), numpy's dtype rules: a float array
        keeps its dtype for a python scalar a; an integer array with a non-negative python int
        stays integer (exponentiation by squaring, wrapping), with a float a becomes float64.
        a == 2 is x*x, numpy's exact result; other float exponents run the device pow (numpy's
        own float power comes from its host SIMD library and differs between hosts: parity is
        1e-6 relative for float32, 1e-15 for float64)."""
        import torch

        from . import ops
        dev = _device()
        out = []
        for x in m1:
            host = not isinstance(x, torch.Tensor)
            xa = np.asarray(x) if host else None
            xdt = xa.dtype if host else ops.numpy_dtype(x.dtype)
            shape = tuple(x.shape)
            if xdt.kind in "iu" and isinstance(a, (int, np.integer)) and a < 0:
                raise ValueError("Integers to negative integer powers are not allowed.")
            rdt = np.power(np.empty(0, xdt), a).dtype               # numpy's result dtype (no data)
            xd = torch.from_numpy(np.ascontiguousarray(xa).reshape(-1)).to(dev) if host else x.contiguous().reshape(-1)
            o = torch.empty(xd.numel(), dtype=ops.torch_dtype(rdt), device=dev)
            if rdt.kind in "iu":
                ops.elementwise("ipow", o, xd, None, float(a))
            elif o.dtype == torch.float16:
                # half power: x*x / pow computed in float32 from the exact widening, rounded once to
                # half (x*x is exact in float32: numpy's result; pow: numpy's libm, 1e-3 relative)
                w = xd if xd.dtype == torch.float32 else ops.cast(torch.empty(xd.numel(), dtype=torch.float32,
                                                                               device=dev), xd)
                t = torch.empty(xd.numel(), dtype=torch.float32, device=dev)
                ops.elementwise("square" if a == 2 else "pow", t, w, None, float(np.float16(a)))
                ops.cast(o, t)
            else:
                if xd.dtype != o.dtype:
                    xd = ops.cast(torch.empty(xd.numel(), dtype=o.dtype, device=dev), xd)
                ops.elementwise("square" if a == 2 else "pow", o, xd, None, float(a))
            out.append(_back(o, host, shape))
        return out

    def norm(self, m):
        """numpyhelper.norm (numpyhelper.py:106-117): the sum over tensors of np.linalg.norm(x, 1) —
        sum |x| of a vector, the max column sum of |x| of a matrix (the MATRIX 1-norm), a
        ValueError for 0-d or >2-d tensors — accumulated from a python 0.0 as the reference does
        (so float32 models give a numpy float32). Each tensor's norm is one device reduction in
        float64 (numpy sums float32 pairwise in float32: parity 1e-6 relative)."""
        import torch

        from . import ops
        dev = _device()
        n = 0.0
        for x in m:
            host = not isinstance(x, torch.Tensor)
            xa = np.asarray(x) if host else None
            xdt = xa.dtype if host else ops.numpy_dtype(x.dtype)
            nd = len(x.shape)
            if nd not in (1, 2):
                raise ValueError("Improper number of dimensions to norm.")
            if nd == 2 and x.shape[1] == 0:
                raise ValueError("zero-size array to reduction operation maximum which has no identity")
            xd = torch.from_numpy(np.ascontiguousarray(xa)).to(dev) if host else x.contiguous()
            if xd.dtype == torch.float16:              # summed from the exact float32 widening
                xd = ops.cast(torch.empty(tuple(xd.shape), dtype=torch.float32, device=dev), xd)
            val = float(ops.norm1(xd, nd == 2).item())
            rdt = xdt if xdt.kind == "f" else np.dtype(np.float64)   # numpy: non-inexact -> astype(float)
            n += rdt.type(val)
        return n

    def sign(self, m1):
        return self._ew("sign", m1)

    def ones(self, m1, a):
        """np.ones(shape) * a: float64 (numpyhelper.py:129-142)."""
        return self._ew("fill", m1, None, a)

    def save(self, weights, path=None, file_type="npz"):
        """numpyhelper.save (numpyhelper.py:144-169): np.savez_compressed's archive, written by the
        native writer (codec.savez_into: the same bytes). numpy's own file handling is kept: a path
        gets ".npz" appended unless it ends in it (the given path is returned, as the reference
        returns it); a file object is written from where it stands. zipfile's records hold offsets
        from the stream's start and switch to data descriptors on a stream it cannot seek, so a
        file object not at offset 0, not seekable or without ``read`` is handed to np.savez_compressed
        itself (which writes it, or raises, as the reference would)."""
        self.check_supported_file_type(file_type)
        if file_type == "npz":
            if not path:
                path = self.get_tmp_path()
            weights = list(weights)
            if hasattr(path, "write"):
                at = None
                if hasattr(path, "read"):           # numpy's zipfile_factory takes it as a file only then
                    try:
                        at = path.tell()
                        path.seek(at)
                    except (AttributeError, OSError):
                        at = None
                if at != 0 and npz_writer() != "blocks":
                    np.savez_compressed(path, **{str(i): w for i, w in enumerate(weights)})
                    return path
            if npz_writer() == "blocks":
                data = codec.save_npz_blocks(weights)
            else:
                try:
                    data = memoryview(codec.savez_into(weights))
                except MemoryError:
                    # the native writer holds the archive in memory (and, for a big member, a copy of
                    # it): where that does not fit, numpy itself streams the same bytes to the target
                    # in 16 MiB writes, as the reference does
                    np.savez_compressed(path, **{str(i): w for i, w in enumerate(weights)})
                    return path
            if hasattr(path, "write"):
                path.write(data)
            else:
                fn = os.fspath(path)
                with open(fn if fn.endswith(".npz") else fn + ".npz", "wb") as f:
                    f.write(data)
            return path
        if not path:
            path = self.get_tmp_path(suffix=".bin")
        np.concatenate(weights).tofile(path)
        return path

    def load(self, path, file_type="npz"):
        self.check_supported_file_type(file_type)
        if file_type == "npz":
            alloc = pinned_empty if decode_pinned() else None
            if isinstance(path, (bytes, bytearray, memoryview)):
                return codec.load_npz(path, alloc=alloc)
            if hasattr(path, "getbuffer"):
                return codec.load_npz(path.getbuffer(), alloc=alloc)
            if hasattr(path, "read"):
                return codec.load_npz(path.read(), alloc=alloc)
            with open(path, "rb") as f:
                return codec.load_npz(np.fromfile(f, dtype=np.uint8), alloc=alloc)
        if isinstance(path, BytesIO):
            return [np.frombuffer(path.read(), dtype=np.float64)]
        return [np.fromfile(path, dtype=np.float64)]

    def get_tmp_path(self, suffix=".npz"):
        fd, path = tempfile.mkstemp(suffix=suffix)
        os.close(fd)
        return path

    def check_supported_file_type(self, file_type):
        supported = ["npz", "raw_binary"]
        if file_type not in supported:
            raise ValueError("File type not supported. Supported types are: {}".format(supported))
        return True
