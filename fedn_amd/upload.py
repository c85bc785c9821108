"""Decode client updates WHILE they upload (ModelService.Upload).

In FEDn a client streams its update to the combiner in 1 MiB chunks (ModelService.Upload,
modelservice.py:196-220; upload_request_generator, :15-31), which only appends them to a temp
file; the npz is inflated later, when the update is loaded (updatehandler.py:90-117,
modelservice.py:110-125). A numpy-written npz (np.savez_compressed) is one deflate stream per
tensor, so inflating a 100 M-parameter update takes ~0.3 s on one core, and it starts only
after the last byte arrived. :class:`StreamingUpload` wraps the combiner's ModelService:
every chunk still goes to the original Upload unchanged, and a copy is fed to a decoder on a
worker thread (:class:`NpzStreamDecoder`: ZIP local headers + .npy headers parsed as they
arrive, deflate inflated incrementally with zlib, CRC-32 checked), so decoding overlaps the
network transfer. When the upload completes, the decoded update is handed to the
:class:`~fedn_amd.ingest.StagingUpdateHandler`, which copies it to HBM when the matching
``ModelUpdate`` arrives (SendModelUpdate) instead of decoding the file again. Anything the
decoder does not handle (non-npz helpers' bytes, Fortran-ordered or object arrays, a corrupt
stream) is simply not adopted: the update then takes the normal path.
"""
import io
import queue
import struct
import threading
import zlib
from collections import OrderedDict
from concurrent.futures import Future, ThreadPoolExecutor

import numpy as np

MODEL_STATUS_OK = 0            # fedn.proto:147-153 (ModelStatus)
MODEL_STATUS_IN_PROGRESS = 1

_LOCAL = b"PK\x03\x04"
_DESC = b"PK\x07\x08"
_END = (b"PK\x01\x02", b"PK\x05\x06", b"PK\x06\x06", b"PK\x06\x07")


class DecodeError(ValueError):
    pass


class _Member:
    __slots__ = ("name", "method", "flags", "crc", "csize", "usize", "zip64", "inflater", "consumed", "hdr",
                 "array", "view", "filled", "crc_run", "raw_left")


class NpzStreamDecoder:
    """Incremental decoder of an npz archive (a ZIP of ``.npy`` members, stored or deflated)
    fed in arbitrary chunks. ``alloc(nbytes)`` returns a writable uint8 numpy buffer for one
    member's array data (e.g. a view of pinned host memory); ``members()`` returns
    ``[(name, dtype, shape, uint8 buffer)]`` in archive order once ``finish()`` succeeded."""

    def __init__(self, alloc=None):
        self.alloc = alloc or (lambda n: np.empty(n, dtype=np.uint8))
        self.buf = bytearray()
        self.state = "header"
        self.cur = None
        self.done = []
        self.finished = False

    # -- feeding ------------------------------------------------------------------------
    def feed(self, data):
        if self.finished:
            return
        self.buf += data
        while self._step():
            pass

    def finish(self):
        """Check the archive ended cleanly; returns the decoded members."""
        while self._step():
            pass
        if not self.finished and not (self.state == "header" and not self.buf and self.done):
            raise DecodeError(f"archive truncated (state {self.state})")
        return self.done

    def _step(self):
        if self.state == "header":
            return self._header()
        if self.state == "data":
            return self._data()
        if self.state == "descriptor":
            return self._descriptor()
        return False

    # -- ZIP local file header ----------------------------------------------------------------
    def _header(self):
        if len(self.buf) < 4:
            return False
        sig = bytes(self.buf[:4])
        if sig in _END:                               # central directory: every member is in
            self.finished = True
            self.state = "end"
            self.buf = bytearray()
            return False
        if sig != _LOCAL:
            raise DecodeError("not a ZIP local file header")
        if len(self.buf) < 30:
            return False
        (_, _, flags, method, _, _, crc, csize, usize, nlen, xlen) = struct.unpack("<IHHHHHIIIHH", bytes(self.buf[:30]))
        if len(self.buf) < 30 + nlen + xlen:
            return False
        name = bytes(self.buf[30:30 + nlen]).decode("utf-8", "replace")
        extra = bytes(self.buf[30 + nlen:30 + nlen + xlen])
        zip64 = False
        p = 0
        while p + 4 <= len(extra):                    # zip64 extended information (0x0001)
            tag, size = struct.unpack("<HH", extra[p:p + 4])
            if tag == 0x0001:
                zip64 = True
                vals = extra[p + 4:p + 4 + size]
                q = 0
                if usize == 0xFFFFFFFF and q + 8 <= len(vals):
                    usize = struct.unpack("<Q", vals[q:q + 8])[0]
                    q += 8
                if csize == 0xFFFFFFFF and q + 8 <= len(vals):
                    csize = struct.unpack("<Q", vals[q:q + 8])[0]
            p += 4 + size
        if method not in (0, 8):
            raise DecodeError(f"member {name}: compression method {method}")
        if method == 0 and flags & 8:
            raise DecodeError(f"member {name}: stored with a data descriptor (size unknown)")
        del self.buf[:30 + nlen + xlen]
        m = _Member()
        m.name, m.method, m.flags, m.crc, m.csize, m.usize, m.zip64 = name, method, flags, crc, csize, usize, zip64
        m.inflater = zlib.decompressobj(-15) if method == 8 else None
        m.raw_left = csize if method == 0 else None
        m.hdr = bytearray()
        m.array = None
        m.view = None
        m.filled = 0
        m.crc_run = 0
        self.cur = m
        self.state = "data"
        return True

    # -- member payload ---------------------------------------------------------------------
    def _data(self):
        m = self.cur
        if not self.buf:
            return False
        if m.method == 0:
            take = min(len(self.buf), m.raw_left)
            out = bytes(self.buf[:take])
            del self.buf[:take]
            m.raw_left -= take
            ended = m.raw_left == 0
        else:
            out = m.inflater.decompress(bytes(self.buf))
            self.buf = bytearray()
            ended = m.inflater.eof
            if ended:
                self.buf = bytearray(m.inflater.unused_data)
        if out:
            m.crc_run = zlib.crc32(out, m.crc_run)
            self._emit(m, out)
        if not ended:
            return False
        self._end_member(m)
        return True

    def _emit(self, m, out):
        if m.array is None:                           # still inside the .npy header
            m.hdr += out
            hdr = self._npy_header(m)
            if hdr is None:
                return
            used, dtype, shape = hdr
            rest = bytes(m.hdr[used:])
            m.hdr = None
            nbytes = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
            m.view = self.alloc(nbytes)
            m.array = (dtype, tuple(shape))
            out = rest
        if out:
            n = len(out)
            if m.filled + n > m.view.size:
                raise DecodeError(f"member {m.name}: more data than its .npy header declares")
            m.view[m.filled:m.filled + n] = np.frombuffer(out, dtype=np.uint8)
            m.filled += n

    @staticmethod
    def _npy_header(m):
        h = bytes(m.hdr)
        if len(h) < 10:
            return None
        if h[:6] != b"\x93NUMPY":
            raise DecodeError(f"member {m.name} is not a .npy array")
        major = h[6]
        hl_size = 2 if major == 1 else 4
        if len(h) < 8 + hl_size:
            return None
        hlen = struct.unpack("<H" if hl_size == 2 else "<I", h[8:8 + hl_size])[0]
        used = 8 + hl_size + hlen
        if len(h) < used:
            return None
        f = io.BytesIO(h[:used])
        version = np.lib.format.read_magic(f)
        shape, fortran, dtype = np.lib.format._read_array_header(f, version)   # safe literal parse
        if dtype.hasobject:
            raise DecodeError(f"member {m.name}: object arrays are not decoded (allow_pickle=False)")
        if fortran and len(shape) > 1:
            raise DecodeError(f"member {m.name}: Fortran-ordered arrays take the normal path")
        return used, dtype, shape

    def _end_member(self, m):
        if m.array is None:
            raise DecodeError(f"member {m.name}: truncated .npy header")
        if m.filled != m.view.size:
            raise DecodeError(f"member {m.name}: {m.filled} of {m.view.size} bytes")
        if m.flags & 8:
            self.state = "descriptor"
        else:
            if (m.crc_run & 0xFFFFFFFF) != m.crc:
                raise DecodeError(f"member {m.name}: CRC-32 mismatch")
            self._push(m)
            self.state = "header"

    def _descriptor(self):
        m = self.cur
        has_sig = len(self.buf) >= 4 and bytes(self.buf[:4]) == _DESC
        size = (4 if has_sig else 0) + 4 + (16 if m.zip64 else 8)
        if len(self.buf) < size:
            return False
        o = 4 if has_sig else 0
        crc = struct.unpack("<I", bytes(self.buf[o:o + 4]))[0]
        del self.buf[:size]
        if (m.crc_run & 0xFFFFFFFF) != crc:
            raise DecodeError(f"member {m.name}: CRC-32 mismatch")
        self._push(m)
        self.state = "header"
        return True

    def _push(self, m):
        dtype, shape = m.array
        name = m.name[:-4] if m.name.endswith(".npy") else m.name
        self.done.append((name, dtype, shape, m.view))
        self.cur = None


class DecodedUpdate:
    """A fully decoded npz update in host memory: arrays in FEDn's key order ("0", "1", ...)."""

    __slots__ = ("arrays", "nbytes", "pinned")

    def __init__(self, members, pinned):
        by_name = {m[0]: m for m in members}
        try:                          # numpyhelper.load order: a[str(i)] (numpyhelper.py:180-182)
            members = [by_name[str(i)] for i in range(len(members))]
        except KeyError as e:
            raise DecodeError(f"npz keys are not 0..{len(members) - 1}: missing {e}") from None
        self.arrays = [view.view(dtype).reshape(shape) for _, dtype, shape, view in members]
        self.nbytes = sum(a.nbytes for a in self.arrays)
        self.pinned = pinned          # keeps the pinned blocks alive


class StreamingUpload:
    """Wrap a FEDn ``ModelService`` so uploads are decoded while they stream in.

    ``Upload`` passes every request to the wrapped service's ``Upload`` unchanged (the temp file
    is still written) and feeds the chunk bytes to a decoder worker. On the ``OK`` request the
    decoded update is offered to ``handler`` (:meth:`StagingUpdateHandler.adopt`). Decoded but
    unclaimed uploads (e.g. the combiner's own global models) are dropped beyond
    ``max_unclaimed_bytes``. Every other attribute is the wrapped service's."""

    def __init__(self, inner, handler, workers=4, pinned=True):
        self.inner = inner
        self.handler = handler
        self.pinned = pinned
        self._pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="fedn_amd_upload")

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def _alloc(self, keep):
        def alloc(nbytes):
            if self.pinned:
                import torch
                t = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
                keep.append(t)
                return t.numpy()[:nbytes]
            a = np.empty(nbytes, dtype=np.uint8)
            keep.append(a)
            return a
        return alloc

    def _decode(self, q, fut):
        keep = []
        dec = NpzStreamDecoder(self._alloc(keep))
        ended = False
        try:
            while True:
                chunk = q.get()
                if chunk is None:
                    ended = True
                    break
                dec.feed(chunk)
            fut.set_result(DecodedUpdate(dec.finish(), keep))
        except Exception as e:  # noqa: BLE001 — not adopted: the update takes the normal path
            keep.clear()
            fut.set_exception(e)
            while not ended:                           # drain to the end of the upload
                ended = q.get() is None

    def Upload(self, request_iterator, context):
        streams = {}

        def tee():
            try:
                for request in request_iterator:
                    rid = request.id
                    if request.status == MODEL_STATUS_IN_PROGRESS and request.data:
                        st = streams.get(rid)
                        if st is None and self.handler.wants_upload():
                            q, fut = queue.Queue(), Future()
                            self._pool.submit(self._decode, q, fut)
                            st = streams[rid] = (q, fut)
                        if st is not None:
                            st[0].put(bytes(request.data))
                    if request.status == MODEL_STATUS_OK and not request.data and rid in streams:
                        q, fut = streams.pop(rid)
                        q.put(None)
                        self.handler.adopt(rid, fut)
                    yield request
            finally:                                   # stream ended (or Upload gave up) without OK
                for q, _ in streams.values():
                    q.put(None)
                streams.clear()

        return self.inner.Upload(tee(), context)

    def close(self):
        self._pool.shutdown(wait=True)


class AdoptedUploads:
    """Decoded uploads waiting for their ModelUpdate, bounded by bytes (oldest dropped first)."""

    def __init__(self, max_bytes=16 << 30):
        self.max_bytes = max_bytes
        self._lock = threading.Lock()
        self._items = OrderedDict()       # id -> Future[DecodedUpdate]

    def put(self, rid, fut):
        with self._lock:
            self._items[rid] = fut
            total, drop = 0, []
            for k, f in reversed(self._items.items()):
                if f.done() and f.exception() is None:
                    total += f.result().nbytes
                    if total > self.max_bytes:
                        drop.append(k)
            for k in drop:
                self._items.pop(k, None)

    def pop(self, rid):
        with self._lock:
            return self._items.pop(rid, None)
