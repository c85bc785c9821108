"""Flat device layout of a FEDn model (``list[np.ndarray]``, numpyhelper's model format).

A model is a list of per-layer arrays (numpyhelper.py:171-189 loads them from an npz
in key order "0", "1", ...). The kernels work on flat buffers, so a model is packed
into ONE contiguous byte buffer with one region per element dtype ("group"): every
fp32 tensor back to back, then (if any) the int64 tensors, etc. Each region starts
on a 256-byte boundary so every group base is 16-B aligned for the vector path.
One H2D copy moves a whole update; one kernel launch per group folds it.
"""
import ctypes
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ALIGN = 256
# host pack: large tensors are copied into the pinned staging buffer by several threads
# (np.copyto releases the GIL), so the host memcpy keeps up with PCIe Gen5 H2D
PACK_THREADS = int(os.environ.get("FEDN_AMD_PACK_THREADS", "8"))
PACK_CHUNK = 16 << 20   # bytes per copy task (at most)
PACK_MIN_PARALLEL = 1 << 20   # updates smaller than this are packed inline (a task costs ~10 us)
_pool = None


def _native_gather(jobs):
    """The pack's copies in one call to libfednpz's gather (persistent native threads: no Python
    future per piece, ~3x the Python pool's rate on mid-size updates); False if the codec library
    is not built, in which case the Python pool copies (same bytes)."""
    for d, src in jobs:
        if d.dtype != src.dtype:
            raise TypeError(f"pack: {src.dtype} into a {d.dtype} region")   # np.copyto(casting="no")
        if not (d.flags.c_contiguous and src.flags.c_contiguous):
            return False
    try:
        from . import codec
        codec.gather(jobs, PACK_THREADS)
    except ImportError:
        return False
    return True


def run_pack_jobs(jobs):
    """Run (destination view, flat source) copies: inline below PACK_MIN_PARALLEL bytes in total,
    else in >= 1 MiB pieces on the native gather's threads (the Python pool if the codec library
    is not built)."""
    total = sum(d.nbytes for d, _ in jobs)
    if PACK_THREADS <= 1 or total < PACK_MIN_PARALLEL:
        for d, src in jobs:
            np.copyto(d, src, casting="no")
        return
    if _native_gather(jobs):
        return
    piece = max(1 << 20, min(PACK_CHUNK, -(-total // PACK_THREADS)))
    futs = []
    for d, src in jobs:
        step = max(1, piece // src.itemsize)
        for i in range(0, src.size, step):
            futs.append(_executor().submit(np.copyto, d[i:i + step], src[i:i + step], casting="no"))
    for f in futs:
        f.result()


def _in_window(dst_ptr, nbytes, window):
    lo, ln = window
    if dst_ptr < lo or dst_ptr + nbytes > lo + ln:
        raise ValueError(f"pack: {nbytes} bytes at offset {dst_ptr - lo} do not fit the {ln}-byte destination buffer")


def start_pack_into(layout, arrays, dst_ptr, window):
    """Queue the pack of ``arrays`` (already checked against ``layout``: shapes and dtypes) into the
    host bytes at address ``dst_ptr`` to the native gather thread; returns (ticket, the sources to
    keep referenced until :func:`wait_pack_jobs`). None as ticket: copied already (no codec library,
    or a non-contiguous source). ``window`` = (address, length) of the pinned buffer ``dst_ptr``
    points into: a pack that would not fit raises (the native gather checks it too, fednpz ABI 4)."""
    srcs = [arrays[i] for i, _, _ in layout.pack_plan]
    if not srcs:                                  # only empty tensors: nothing to copy
        return None, srcs
    if all(type(a) is np.ndarray and a.flags.c_contiguous for a in srcs):
        try:
            from . import codec
            return codec.gather_start_raw([dst_ptr + off for _, off, _ in layout.pack_plan],
                                          [a.ctypes.data for a in srcs], [n for _, _, n in layout.pack_plan],
                                          PACK_THREADS, window), srcs
        except ImportError:
            pass
    _in_window(dst_ptr, layout.nbytes, window)
    buf = np.ctypeslib.as_array((ctypes.c_uint8 * layout.nbytes).from_address(dst_ptr))
    layout.pack(arrays, buf)
    return None, srcs


_FAST = None          # (admit, address of fnpz_gather_start) once loaded; False: extension not built


def _fast():
    global _FAST
    if _FAST is None:
        try:
            from . import _fastpack, codec
            _FAST = (_fastpack.admit, ctypes.cast(codec.load_lib().fnpz_gather_start, ctypes.c_void_p).value)
        except ImportError:
            _FAST = False
    return _FAST


def fast_admission(layout):
    """``admit(arrays, dst_ptr, window) -> ticket | 0 | -1`` for ``layout`` (cached on it): the exact
    (shape, dtype, C-contiguous) test of a host update and the queueing of its pack into the pinned
    bytes at ``dst_ptr`` in ONE native call (``_fastpack``, csrc/fastpack.c); -1 leaves everything
    untouched (not this layout). ``window`` = (address, length) of the pinned buffer: a pack outside
    it raises CodecError (FNPZ_ENOSPC) with nothing copied. None if the extension or the codec
    library is not built."""
    f = getattr(layout, "_fast_admit", 0)
    if f == 0:
        f = None
        fast = _fast()
        if fast:
            from . import _fastpack
            admit, gstart = fast
            offs = {i: off for i, off, _ in layout.pack_plan}
            plan = _fastpack.plan([(tuple(sh), np.dtype(dt), offs.get(i, 0))
                                   for i, (sh, dt) in enumerate(zip(layout.shapes, layout.dtypes))])

            def f(arrays, dst_ptr, window, plan=plan, admit=admit, gstart=gstart):
                t = admit(plan, arrays, dst_ptr, gstart, PACK_THREADS, window[0], window[1])
                if t == -2:                     # the gather queue refused the job: its reason
                    from . import codec
                    why = codec.load_lib().fnpz_last_error().decode(errors="replace")
                    raise codec.CodecError(f"fnpz_gather_start: {why}")
                return t
        layout._fast_admit = f
    return f


def wait_pack_jobs(ticket):
    if ticket is not None:
        from . import codec
        codec.gather_wait(ticket)


def _executor():
    global _pool
    if _pool is None or _pool[0] != os.getpid():     # a forked child starts its own pool
        _pool = (os.getpid(), ThreadPoolExecutor(max_workers=PACK_THREADS, thread_name_prefix="fedn_amd_pack"))
    return _pool[1]


def parallel_copy(dst, src):
    """dst[:] = src for 1-D arrays of one dtype, split over the pack thread pool."""
    n = src.size
    step = max(1, PACK_CHUNK // max(1, src.itemsize))
    if PACK_THREADS <= 1 or n <= 2 * step:
        np.copyto(dst, src, casting="no")
        return
    if _native_gather([(dst, src)]):
        return
    futs = [_executor().submit(np.copyto, dst[i:i + step], src[i:i + step], casting="no") for i in range(0, n, step)]
    for f in futs:
        f.result()


# FEDN_AMD_DEVICES: a model is sliced over several GPUs of the process only when its packed size
# is at least this; a smaller one (every per-GPU slice a few MB at most) runs on the first GPU,
# where one copy and one launch per update beat one per GPU
MULTIDEV_MIN_BYTES = int(os.environ.get("FEDN_AMD_MULTIDEV_MIN_BYTES", str(64 << 20)))


def spread(devices, nbytes):
    """The devices a model of ``nbytes`` (packed) is sliced over: all of ``devices`` for a large
    model, only the first below MULTIDEV_MIN_BYTES (read at call time)."""
    if devices and len(devices) > 1 and nbytes < MULTIDEV_MIN_BYTES:
        return list(devices[:1])
    return list(devices) if devices else devices


def _round_up(x, a):
    return (x + a - 1) // a * a


class Layout:
    """Shapes, dtypes and group offsets of a model."""

    def __init__(self, shapes, dtypes):
        self.shapes = [tuple(s) for s in shapes]
        self.dtypes = [np.dtype(d) for d in dtypes]
        self.sizes = [int(np.prod(s, dtype=np.int64)) for s in self.shapes]
        # group key = dtype, in first-appearance order
        self.groups = []          # list of dtype
        self.members = {}         # dtype -> list of (tensor index, element offset)
        self.group_elems = {}     # dtype -> elements
        for i, (dt, sz) in enumerate(zip(self.dtypes, self.sizes)):
            if dt not in self.members:
                self.groups.append(dt)
                self.members[dt] = []
                self.group_elems[dt] = 0
            self.members[dt].append((i, self.group_elems[dt]))
            self.group_elems[dt] += sz
        self.group_byte_offset = {}
        off = 0
        for dt in self.groups:
            self.group_byte_offset[dt] = off
            off = _round_up(off + self.group_elems[dt] * dt.itemsize, ALIGN)
        self.nbytes = max(off, ALIGN)
        self.nparams = sum(self.sizes)
        # (tensor index, byte offset in the packed buffer, bytes) of every non-empty tensor: the
        # copies of a pack as plain integers (staging's arena packs need no numpy views)
        self.pack_plan = [(i, self.group_byte_offset[dt] + off * dt.itemsize, self.sizes[i] * dt.itemsize)
                          for dt in self.groups for i, off in self.members[dt] if self.sizes[i]]

    def shard_geometry(self, ndev):
        """Parameter-slice sharding over ``ndev`` devices (multidev.py, ingest.py):
        ``bounds[dt][d]`` = device d's [lo, hi) of group dt (4 KiB-aligned,
        sharded.shard_bounds), ``dev_off[d][dt]`` = byte offset of that slice in device d's
        buffer (each slice ALIGN-aligned), ``dev_bytes[d]`` = size of device d's buffer."""
        from .sharded import shard_bounds
        bounds = {dt: shard_bounds(self.group_elems[dt], ndev) for dt in self.groups}
        dev_off, dev_bytes = [], []
        for d in range(ndev):
            off, offs = 0, {}
            for dt in self.groups:
                lo, hi = bounds[dt][d]
                offs[dt] = off
                off += _round_up((hi - lo) * dt.itemsize, ALIGN)
            dev_off.append(offs)
            dev_bytes.append(max(off, ALIGN))
        return bounds, dev_off, dev_bytes

    _by_sig = {}                  # Layout.of: one Layout per (shapes, dtypes) seen (a session's rounds)

    @classmethod
    def of(cls, arrays):
        arrays = [np.asarray(a) for a in arrays]
        key = tuple((a.shape, a.dtype.str) for a in arrays)
        lay = cls._by_sig.get(key)
        if lay is None:
            lay = cls([a.shape for a in arrays], [a.dtype for a in arrays])
            if len(cls._by_sig) >= 64:
                cls._by_sig.clear()
            cls._by_sig[key] = lay
        return lay

    def signature(self):
        sig = self.__dict__.get("_signature")
        if sig is None:                 # a Layout never changes: computed once
            sig = self._signature = (tuple(self.shapes), tuple(str(d) for d in self.dtypes))
        return sig

    def check(self, arrays):
        """Raise (as numpy would, on a non-broadcastable mismatch) if ``arrays`` does not match."""
        if len(arrays) != len(self.shapes):
            raise ValueError(f"model has {len(arrays)} tensors, expected {len(self.shapes)}")
        for i, a in enumerate(arrays):
            a = np.asarray(a)
            if tuple(a.shape) != self.shapes[i]:
                raise ValueError(f"operands could not be combined: tensor {i} has shape {a.shape}, "
                                 f"expected {self.shapes[i]}")
            if a.dtype != self.dtypes[i]:
                raise TypeError(f"tensor {i} has dtype {a.dtype}, expected {self.dtypes[i]} "
                                "(mixed dtypes across client updates are not supported)")

    def check_layout(self, other):
        """Like :meth:`check` for an already-laid-out update (a staged model's Layout)."""
        if other is self or other.signature() == self.signature():
            return
        if len(other.shapes) != len(self.shapes):
            raise ValueError(f"model has {len(other.shapes)} tensors, expected {len(self.shapes)}")
        for i, (s, d) in enumerate(zip(other.shapes, other.dtypes)):
            if s != self.shapes[i]:
                raise ValueError(f"operands could not be combined: tensor {i} has shape {s}, expected {self.shapes[i]}")
            if d != self.dtypes[i]:
                raise TypeError(f"tensor {i} has dtype {d}, expected {self.dtypes[i]} "
                                "(mixed dtypes across client updates are not supported)")

    def group_view(self, buf_np_u8, dt):
        """numpy view of group ``dt`` inside a uint8 host buffer."""
        off = self.group_byte_offset[dt]
        n = self.group_elems[dt]
        return buf_np_u8[off:off + n * dt.itemsize].view(dt)

    def pack(self, arrays, buf_np_u8):
        """Copy the tensors of ``arrays`` into their group regions of a host uint8 buffer: inline
        for a small update; otherwise every tensor is cut into pieces (>= 1 MiB, at most
        PACK_CHUNK, ~1 per pack thread over the whole update) copied by the pack threads, so a
        model of many mid-size tensors is packed in parallel, not one tensor at a time."""
        run_pack_jobs(self.pack_jobs(arrays, buf_np_u8))

    def pack_range(self, arrays, dst_ptr, lo, hi):
        """(destination address, source address, bytes) copies that write bytes [lo, hi) of the packed
        update at ``dst_ptr`` (padding between groups untouched, as :meth:`pack`); None if a source
        overlapping the range is not a C-contiguous ndarray of its layout dtype (the caller packs
        whole instead). The caller keeps ``arrays`` alive until the copies ran."""
        out = []
        for i, off, nb in self.pack_plan:
            s0, s1 = max(lo, off), min(hi, off + nb)
            if s0 < s1:
                a = arrays[i]
                if type(a) is not np.ndarray or not a.flags.c_contiguous or a.dtype != self.dtypes[i]:
                    return None
                out.append((dst_ptr + s0, a.ctypes.data + (s0 - off), s1 - s0))
        return out

    def pack_jobs(self, arrays, buf_np_u8):
        """The (destination view, flat source) copies of :meth:`pack`, not run yet (a caller that
        packs many small updates runs them together: :func:`run_pack_jobs`)."""
        jobs = []
        for dt in self.groups:
            g = self.group_view(buf_np_u8, dt)
            for i, off in self.members[dt]:
                sz = self.sizes[i]
                if sz:
                    jobs.append((g[off:off + sz], np.ascontiguousarray(arrays[i]).reshape(-1)))
        return jobs

    def unpack_group(self, flat, dt, out, copy=True):
        """Scatter a group's flat host array back into per-tensor arrays. With copy=False
        the tensors are views of ``flat`` (the caller hands over ownership of it)."""
        for i, off in self.members[dt]:
            sz = self.sizes[i]
            v = flat[off:off + sz]
            out[i] = (np.array(v) if copy else v).reshape(self.shapes[i])
        return out
