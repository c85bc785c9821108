"""Native .npz codec (``libfednpz.so``, include/fednpz.h) — FEDn's model wire format.

FEDn serialises every model with ``np.savez_compressed`` and reads it back through a temp
file and ``np.load`` (numpyhelper.py:144-189, modelservice.py:57-75, 110-146). This module
decodes an archive held in memory straight into caller buffers — optionally one pinned
host buffer in the grouped flat layout the GPU pipelines stage from (layout.py) — and
encodes. Decoded arrays are byte-identical to ``np.load``. Two writers:

  save_npz         the bytes np.savez_compressed writes (numpyhelper.py:162), byte for byte
                   (fnpz_savez): what Helper.save produces by default
  save_npz_blocks  a block-parallel deflate with a private block index (fnpz_write): valid
                   npz files np.load reads, several times smaller/faster to write and decode
                   in parallel, but not numpy's bytes (opt-in: FEDN_AMD_NPZ_WRITER=blocks)
"""
import ctypes
import io
import os
import threading
import zlib

import numpy as np

from .layout import Layout

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfednpz.so")
MAX_DIMS = 64           # numpy 2.x NPY_MAXDIMS (include/fednpz.h FNPZ_MAX_DIMS)
FNPZ_ABI_VERSION = 7    # include/fednpz.h
THREADS = int(os.environ.get("FEDN_AMD_CODEC_THREADS", str(min(16, os.cpu_count() or 1))))


class Entry(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 256), ("descr", ctypes.c_char * 32), ("fortran_order", ctypes.c_int32),
                ("ndim", ctypes.c_int32), ("shape", ctypes.c_int64 * MAX_DIMS), ("nbytes", ctypes.c_int64),
                ("npy_header", ctypes.c_int64), ("data_offset", ctypes.c_int64), ("comp_size", ctypes.c_int64),
                ("uncomp_size", ctypes.c_int64), ("crc32", ctypes.c_uint32), ("method", ctypes.c_int32),
                ("index_offset", ctypes.c_int64), ("index_count", ctypes.c_int32), ("reserved", ctypes.c_int32)]


FNPZ_EFALLBACK = 5     # fnpz_deflate_exact: the input needs zlib itself (fednpz.h)
FNPZ_ENOMEM = 6        # memory or a worker thread ran out inside the call: raised as MemoryError


class CodecError(ValueError):
    pass


_lib = None
_lock = threading.Lock()


def load_lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(f"{LIB_PATH} not found: run python -m fedn_amd.build")
            lib = ctypes.CDLL(LIB_PATH)
            try:
                # the version first: a library from an older build may lack later symbols
                lib.fnpz_abi_version.restype = ctypes.c_int
                if lib.fnpz_abi_version() != FNPZ_ABI_VERSION:
                    raise ImportError(f"{LIB_PATH}: ABI version {lib.fnpz_abi_version()}, expected "
                                      f"{FNPZ_ABI_VERSION}; rebuild it (python -m fedn_amd.build)")
                lib.fnpz_last_error.restype = ctypes.c_char_p
                lib.fnpz_open.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(Entry), ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_int)]
                lib.fnpz_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(Entry), ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]
                lib.fnpz_write_bound.restype = ctypes.c_int64
                lib.fnpz_write_bound.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                                 ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32)]
                lib.fnpz_write.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.POINTER(ctypes.c_int64), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                           ctypes.POINTER(ctypes.c_int64)]
                lib.fnpz_savez.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
                lib.fnpz_stream_open.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
                lib.fnpz_stream_close.argtypes = [ctypes.c_void_p]
                lib.fnpz_stream_close.restype = None
                lib.fnpz_stream_feed.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
                lib.fnpz_stream_next.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                                 ctypes.POINTER(ctypes.c_int), ctypes.POINTER(Entry),
                                                 ctypes.POINTER(ctypes.c_int64)]
                lib.fnpz_gather.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.POINTER(ctypes.c_int64), ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_int64]          # destination buffer window
                lib.fnpz_inflate_raw.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                                 ctypes.c_int64, ctypes.POINTER(ctypes.c_int)]
                lib.fnpz_parallel_config.restype = None
                lib.fnpz_parallel_config.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                                     ctypes.POINTER(ctypes.c_int64)]
                lib.fnpz_crc32.restype = ctypes.c_uint32
                lib.fnpz_crc32.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int64]
                lib.fnpz_gather_start.restype = ctypes.c_int64
                lib.fnpz_gather_start.argtypes = lib.fnpz_gather.argtypes
                lib.fnpz_gather_wait.argtypes = [ctypes.c_int64]
                lib.fnpz_savez_zlib_expect.restype = None
                lib.fnpz_savez_zlib_expect.argtypes = [ctypes.c_char_p, ctypes.c_int]
                lib.fnpz_savez_zlib_status.argtypes = [ctypes.c_char_p, ctypes.c_int64]
                lib.fnpz_savez_stats.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
                # numpy's archive comes from the libz Python's zlib module runs: the exact writer's
                # parallel path is allowed only while this library's libz is that one (fednpz.h)
                lib.fnpz_savez_zlib_expect(zlib.ZLIB_RUNTIME_VERSION.encode(), -1)
            except AttributeError as e:      # a symbol include/fednpz.h declares is missing
                raise ImportError(f"{LIB_PATH}: {e}; rebuild it (python -m fedn_amd.build)") from e
            _lib = lib
    return _lib


def _check(rc):
    if rc:
        msg = f"fednpz status {rc}: {load_lib().fnpz_last_error().decode(errors='replace')}"
        if rc == FNPZ_ENOMEM:
            raise MemoryError(msg)
        raise CodecError(msg)


def gather_start_raw(dsts, srcs, nbytes, threads, window):
    """``nbytes[i]`` bytes from address ``srcs[i]`` to ``dsts[i]`` (lists of ints), queued to the native
    gather thread (``fnpz_gather_start``); returns the ticket for :func:`gather_wait`. ``window`` =
    (address, length) of the destination buffer: a segment outside it raises CodecError (FNPZ_ENOSPC)
    and nothing is copied. The caller keeps every source and destination alive until the ticket is done."""
    n = len(dsts)
    lo, ln = window
    t = load_lib().fnpz_gather_start(n, (ctypes.c_void_p * n)(*dsts), (ctypes.c_void_p * n)(*srcs),
                                     (ctypes.c_int64 * n)(*nbytes), max(1, threads), int(lo), int(ln))
    if t < 0:
        _check(-t)
    return t


def gather_wait(ticket):
    _check(load_lib().fnpz_gather_wait(ticket))


def gather_raw(jobs, threads, window):
    """``(dst address, src address, bytes)`` copies in one native call (``fnpz_gather``: 1 MiB+ pieces
    on the persistent thread pool, the GIL released); the caller keeps both ends alive. ``window`` =
    (address, length) of the destination buffer every copy must land in (else CodecError)."""
    n = len(jobs)
    if not n:
        return
    dsts, srcs, nb = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)(), (ctypes.c_int64 * n)()
    for i, (d, src, b) in enumerate(jobs):
        dsts[i], srcs[i], nb[i] = d, src, b
    lo, ln = window
    _check(load_lib().fnpz_gather(n, dsts, srcs, nb, int(threads), int(lo), int(ln)))


def gather(pairs, threads):
    """``dst[:] = src`` for each (dst, src) pair of C-contiguous numpy arrays of equal byte size, in
    one native call (``fnpz_gather``: 1 MiB+ pieces on a persistent thread pool; the GIL is released
    while it copies). The destination window is the span the destination arrays cover (numpy bounds
    each one)."""
    n = len(pairs)
    dsts, srcs, nb = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)(), (ctypes.c_int64 * n)()
    lo = hi = None
    for i, (d, src) in enumerate(pairs):
        if d.nbytes != src.nbytes:
            raise ValueError(f"gather: {d.nbytes} != {src.nbytes} bytes")
        if not (d.flags.c_contiguous and src.flags.c_contiguous):
            raise ValueError("gather: non-contiguous array")
        dsts[i], srcs[i], nb[i] = d.ctypes.data, src.ctypes.data, d.nbytes
        if d.nbytes:
            a, b = d.ctypes.data, d.ctypes.data + d.nbytes
            lo, hi = (a, b) if lo is None else (min(lo, a), max(hi, b))
    _check(load_lib().fnpz_gather(n, dsts, srcs, nb, int(threads), lo or 0, (hi - lo) if lo is not None else 0))


def _as_u8(buf):
    """A contiguous uint8 numpy view of bytes / bytearray / memoryview / ndarray (no copy)."""
    if isinstance(buf, np.ndarray):
        a = buf.reshape(-1).view(np.uint8)
    else:
        a = np.frombuffer(buf, dtype=np.uint8)
    return np.ascontiguousarray(a)


def open_archive(buf):
    """Parse an npz archive; returns (uint8 view, list of Entry) in archive order."""
    lib = load_lib()
    a = _as_u8(buf)
    n = ctypes.c_int(0)
    cap = 64
    while True:
        ents = (Entry * cap)()
        rc = lib.fnpz_open(a.ctypes.data, a.size, ents, cap, ctypes.byref(n))
        if rc == 4 and n.value > cap:     # FNPZ_ENOSPC: retry with room for every member
            cap = n.value
            continue
        _check(rc)
        return a, list(ents[:n.value])


def _dtype(e):
    dt = np.dtype(e.descr.decode())
    if dt.hasobject:
        raise CodecError("object arrays are not supported")
    return dt


def _shape(e):
    return tuple(e.shape[i] for i in range(e.ndim))


def read_entries(a, ents, dsts, threads=None):
    lib = load_lib()
    arr = (Entry * max(1, len(ents)))(*ents)
    ptrs = (ctypes.c_void_p * max(1, len(ents)))(*[d.ctypes.data if d.size else 0 for d in dsts])
    _check(lib.fnpz_read(a.ctypes.data, a.size, arr, len(ents), ptrs, threads or THREADS))


def inflate_raw(data, out_len, window=0):
    """Raw DEFLATE decode of ``data`` (bytes-like) into ``out_len`` bytes with the codec's decoder
    (fnpz_inflate_raw; ``window``: resume every that many output bytes). (bytes, stream_end);
    CodecError on an invalid or short stream."""
    lib = load_lib()
    src = np.frombuffer(data, dtype=np.uint8)
    out = np.empty(max(1, out_len), dtype=np.uint8)
    end = ctypes.c_int(0)
    _check(lib.fnpz_inflate_raw(src.ctypes.data if src.size else None, src.size, out.ctypes.data, out_len, window,
                                ctypes.byref(end)))
    return out[:out_len].tobytes(), bool(end.value)


def parallel_config(min_member=0, min_chunk=0):
    """Thresholds of the parallel decode of one large deflate stream (fnpz_parallel_config; 0 keeps
    a value); returns (decodes that went parallel, decodes that fell back) so far."""
    ok, fb = ctypes.c_int64(0), ctypes.c_int64(0)
    load_lib().fnpz_parallel_config(int(min_member), int(min_chunk), ctypes.byref(ok), ctypes.byref(fb))
    return ok.value, fb.value


def crc32(data, crc=0):
    """CRC-32 of ``data`` (zlib.crc32's value) with the codec's folded implementation."""
    a = np.frombuffer(data, dtype=np.uint8)
    return int(load_lib().fnpz_crc32(crc, a.ctypes.data if a.size else None, a.size))


def _ordered(ents):
    """numpyhelper.load order: keys "0", "1", ... (numpyhelper.py:180-182); KeyError otherwise."""
    by_name = {e.name.decode(): e for e in ents}
    return [by_name[str(i)] for i in range(len(ents))]


def load_npz(buf, threads=None, alloc=None):
    """Decode an npz archive to the list numpyhelper.Helper.load returns (new arrays).

    ``alloc(shape, dtype, order)``, when given, returns the array a member is decoded into (e.g. in
    page-locked memory, helper.pinned_empty) or None for a plain np.empty."""
    a, ents = open_archive(buf)
    ents = _ordered(ents)
    outs = []
    for e in ents:
        dt, shape, order = _dtype(e), _shape(e), "F" if e.fortran_order else "C"
        o = alloc(shape, dt, order) if alloc is not None else None
        outs.append(np.empty(shape, dtype=dt, order=order) if o is None else o)
    read_entries(a, ents, [o.reshape(-1, order="A").view(np.uint8) if o.size else o.view(np.uint8).reshape(-1)
                           for o in outs], threads)
    return outs


def npz_layout(buf):
    """The flat layout an npz archive decodes into (load_npz_into_layout), from its directory
    and .npy headers alone — no inflate; CodecError if it cannot be decoded that way."""
    _, ents = open_archive(buf)
    ents = _ordered(ents)
    if any(e.fortran_order for e in ents):
        raise CodecError("fortran-ordered members cannot be decoded into the flat layout")
    return Layout([_shape(e) for e in ents], [_dtype(e) for e in ents])


def load_npz_into_layout(buf, alloc, threads=None):
    """Decode straight into ONE buffer in the grouped flat layout of layout.py.

    ``alloc(nbytes)`` returns a uint8 host tensor/array to decode into (e.g. pinned
    memory); returns (layout, buffer). Fortran-ordered members are not supported here."""
    a, ents = open_archive(buf)
    ents = _ordered(ents)
    if any(e.fortran_order for e in ents):
        raise CodecError("fortran-ordered members cannot be decoded into the flat layout")
    layout = Layout([_shape(e) for e in ents], [_dtype(e) for e in ents])
    out = alloc(layout.nbytes)
    base = out.numpy() if hasattr(out, "numpy") else out
    dsts = []
    for i, e in enumerate(ents):
        dt = layout.dtypes[i]
        off = dict(layout.members[dt])[i] * dt.itemsize + layout.group_byte_offset[dt]
        dsts.append(base[off:off + e.nbytes])
    read_entries(a, ents, dsts, threads)
    return layout, out


STRATEGIES = {"auto": -1, "default": 0, "filtered": 1, "huffman": 2, "rle": 3, "fixed": 4}


class _NumpyOnly(Exception):
    """A member only numpy itself writes (pickled object arrays, user dtypes, zero itemsize)."""


def _npy_member(x):
    """(npy header bytes, payload array in numpy's write order, numpy's write size in bytes) for one
    member, as numpy.lib.format.write_array writes it into the zip member (numpy 2.x format.py:
    _write_array_header with version=None — the oldest version that holds the header — then
    16 MiB // itemsize elements per write, C order, or F order for a Fortran-contiguous array)."""
    fmt = np.lib.format
    if x.dtype.hasobject or not getattr(type(x.dtype), "_legacy", True) or x.itemsize == 0:
        raise _NumpyOnly
    bio = io.BytesIO()
    fmt._write_array_header(bio, fmt.header_data_from_array_1_0(x), None)
    if x.flags.f_contiguous and not x.flags.c_contiguous:
        data = x.ravel(order="K")               # memory order == F order (no copy)
    else:
        data = np.ascontiguousarray(x).reshape(-1)
    seg = max(16 * 1024 ** 2 // x.itemsize, 1) * x.itemsize
    return np.frombuffer(bio.getvalue(), dtype=np.uint8), data, seg


def savez_into(arrays, threads=None):
    """np.savez_compressed's archive of ``arrays`` under keys "0", "1", ... (numpyhelper.Helper.save,
    numpyhelper.py:158-162) as a uint8 numpy array (no copy out of the native buffer). Byte-identical
    to numpy's: fnpz_savez replays zipfile's deflate calls on the same libz and its headers. Members
    only numpy writes (object arrays: pickled) make the whole archive come from np.savez_compressed."""
    vals = [np.asanyarray(x) for x in arrays]
    try:
        members = [_npy_member(x) for x in vals]
    except _NumpyOnly:
        bio = io.BytesIO()
        np.savez_compressed(bio, **{str(i): x for i, x in enumerate(vals)})
        return np.frombuffer(bio.getbuffer(), dtype=np.uint8)
    lib = load_lib()
    n = len(members)
    m = max(1, n)
    names = [str(i).encode() for i in range(n)]
    hl = (ctypes.c_int64 * m)(*[h.size for h, _, _ in members])
    nb = (ctypes.c_int64 * m)(*[d.nbytes for _, d, _ in members])
    nl = (ctypes.c_int32 * m)(*[len(s) for s in names])
    seg = (ctypes.c_int64 * m)(*[s for _, _, s in members])
    cap = lib.fnpz_write_bound(n, hl, nb, nl)
    out = np.empty(cap, dtype=np.uint8)
    out_len = ctypes.c_int64(0)
    _check(lib.fnpz_savez(n, (ctypes.c_char_p * m)(*names),
                          (ctypes.c_void_p * m)(*[h.ctypes.data for h, _, _ in members]), hl,
                          (ctypes.c_void_p * m)(*[d.ctypes.data if d.size else 0 for _, d, _ in members]), nb, seg,
                          threads or THREADS, out.ctypes.data, cap, ctypes.byref(out_len)))
    return out[:out_len.value]


def savez_zlib_status():
    """(True, reason) when the exact writer's big members may take its parallel deflate (pdeflate.h,
    zlib 1.2.11's stream recomputed on every thread), else (False, reason): every member then goes
    through the process's libz, the bytes numpy writes with it (include/fednpz.h, ABI 7)."""
    buf = ctypes.create_string_buffer(512)
    on = load_lib().fnpz_savez_zlib_status(buf, len(buf))
    return bool(on), buf.value.decode(errors="replace")


def savez_force_zlib(force):
    """Test hook: ``True`` makes the exact writer act as on a libz it does not model (every member
    through libz); ``False`` restores the check."""
    load_lib().fnpz_savez_zlib_expect(None, 1 if force else 0)


SAVEZ_PHASES = ("copy", "parse", "sync", "sched", "plan", "encode", "crc", "assemble", "total")


def savez_stats():
    """Phase times (s) of the exact writer's last big member and its last call (fnpz_savez_stats)."""
    out = (ctypes.c_double * len(SAVEZ_PHASES))()
    k = load_lib().fnpz_savez_stats(out, len(SAVEZ_PHASES))
    return {name: out[i] for i, name in enumerate(SAVEZ_PHASES[:k])}


def save_npz(arrays, threads=None):
    """np.savez_compressed's bytes for ``arrays`` (keys "0", "1", ...): see :func:`savez_into`."""
    return savez_into(arrays, threads).tobytes()


def save_npz_blocks(arrays, level=6, threads=None, block=0, strategy="auto"):
    """Encode ``arrays`` with the block-parallel writer (keys "0", "1", ...); returns bytes. np.load
    reads the archive; its bytes are this codec's own, not numpy's (see :func:`save_npz`).

    ``strategy``: "auto" (fnpz_write's FNPZ_STRATEGY_AUTO: run-length matching per block, the default
    strategy at level 1 where that is smaller on very compressible blocks — as small as
    np.savez_compressed's level 6 or smaller on model weights and several times faster), or a zlib
    strategy by name ("default" = np.savez_compressed's). np.load reads every choice."""
    lib = load_lib()
    strat = STRATEGIES[strategy] if isinstance(strategy, str) else int(strategy)
    arrays = [np.asarray(x) for x in arrays]
    n = len(arrays)
    names, hdrs, datas = [], [], []
    for i, x in enumerate(arrays):
        if x.dtype.hasobject:
            raise CodecError("object arrays are not supported")
        bio = io.BytesIO()
        np.lib.format.write_array_header_1_0(bio, np.lib.format.header_data_from_array_1_0(x))
        hdrs.append(np.frombuffer(bio.getvalue(), dtype=np.uint8))
        data = x if x.flags.c_contiguous or x.flags.f_contiguous else np.ascontiguousarray(x)
        datas.append(data)
        names.append(str(i).encode())
    hl = (ctypes.c_int64 * max(1, n))(*[h.size for h in hdrs])
    nb = (ctypes.c_int64 * max(1, n))(*[d.nbytes for d in datas])
    nl = (ctypes.c_int32 * max(1, n))(*[len(s) for s in names])
    cap = lib.fnpz_write_bound(n, hl, nb, nl)
    out = np.empty(cap, dtype=np.uint8)
    out_len = ctypes.c_int64(0)
    _check(lib.fnpz_write(n, (ctypes.c_char_p * max(1, n))(*names),
                          (ctypes.c_void_p * max(1, n))(*[h.ctypes.data for h in hdrs]), hl,
                          (ctypes.c_void_p * max(1, n))(*[d.ctypes.data if d.size else 0 for d in datas]), nb,
                          level, strat, threads or THREADS, block, out.ctypes.data, cap, ctypes.byref(out_len)))
    return out[:out_len.value].tobytes()
