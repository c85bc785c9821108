"""Decode client updates WHILE they upload (ModelService.Upload).

In FEDn a client streams its update to the combiner in 1 MiB chunks (ModelService.Upload,
modelservice.py:196-220; upload_request_generator, :15-31), which only appends them to a temp
file; the npz is inflated later, when the update is loaded (updatehandler.py:90-117,
modelservice.py:110-125). A numpy-written npz (np.savez_compressed) is one deflate stream per
tensor, so inflating a 100 M-parameter update takes ~1 s on one core, and it starts only
after the last byte arrived. :class:`StreamingUpload` wraps the combiner's ModelService:
every chunk still goes to the original Upload unchanged, and a copy is fed to a decoder on a
worker thread (:class:`NpzStreamDecoder` over libfednpz's native streaming reader: ZIP local
headers and .npy headers parsed as they arrive, deflate inflated incrementally, CRC-32
checked), so decoding overlaps the network transfer. The payload is inflated into a small
ring of pinned slots that are copied to HBM as they fill (:class:`DeviceSink`), so the
update is already on the device when its upload completes. The decoded update is handed to
the :class:`~fedn_amd.ingest.StagingUpdateHandler`, which places it in the pipelines' layout
when the matching ``ModelUpdate`` arrives (SendModelUpdate) instead of decoding the file
again. Anything the decoder does not handle (non-npz helpers' bytes, Fortran-ordered or
object arrays, a corrupt stream) is simply not adopted: the update then takes the normal path.
"""
import ctypes
import os
import queue
import threading
import time
from collections import OrderedDict
from concurrent.futures import Future, ThreadPoolExecutor

import numpy as np

MODEL_STATUS_OK = 0            # fedn.proto:147-153 (ModelStatus)
MODEL_STATUS_IN_PROGRESS = 1

class DecodeError(ValueError):
    pass


EV_NEED_INPUT, EV_MEMBER, EV_DATA, EV_MEMBER_END, EV_END = range(5)     # include/fednpz.h (fnpz_event)


class HostSink:
    """Decoded payload into one host buffer per member (``alloc(nbytes)`` → uint8 numpy)."""

    def __init__(self, alloc=None):
        self.alloc = alloc or (lambda n: np.empty(n, dtype=np.uint8))

    def open(self, nbytes):
        return self.alloc(nbytes)

    def window(self, view, offset):
        """(address, bytes) the decoder may inflate the member's bytes from ``offset`` into."""
        return view.ctypes.data + offset, view.size - offset

    def commit(self, view, offset, n):
        pass

    def close(self, view):
        pass

    def finish(self):
        return None


class DeviceSink:
    """Decoded payload straight to HBM through a small ring of pinned slots: one device block
    per member; the decoder inflates into the current slot, and every full slot (and each
    member's end) is copied H2D on ``stream`` while the ring moves on (a slot is refilled
    only after its copy completed). Pinned memory per upload is ``ring * slot`` instead of
    the whole update, and the H2D runs while later chunks are still arriving. ``finish()``
    records the event that the last copy fired."""

    def __init__(self, device, stream, slot=8 << 20, ring=4, budget=None):
        import torch
        self.torch, self.device, self.stream, self.slot = torch, device, stream, slot
        # HBM admission (budget.HbmBudget of the staging handler): a member the budget cannot hold
        # ends this decode, and the update takes the normal path (staged or left host-side there)
        self.budget, self.reserved = budget, 0
        self.ring = [torch.empty(slot, dtype=torch.uint8, pin_memory=True) for _ in range(ring)]
        self.addr = [t.data_ptr() for t in self.ring]
        self.events = [None] * ring
        self.i = self.fill = 0
        self.cur, self.cur_off = None, 0

    def open(self, nbytes):
        n = max(nbytes, 1)
        if self.budget is not None:
            if not self.budget.reserve([(self.device, n)]):
                raise MemoryError("HBM budget full: the upload is not decoded into HBM")
            self.reserved += n
        torch = self.torch
        from . import reuse
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):   # allocated where it is written
            return reuse.watch(torch.empty(n, dtype=torch.uint8, device=self.device), self.stream)

    def window(self, blk, offset):
        if self.fill and (self.cur is not blk or self.cur_off + self.fill != offset):
            self._flush()
        if self.fill == 0:
            ev = self.events[self.i]
            if ev is not None:
                ev.synchronize()
            self.cur, self.cur_off = blk, offset
        return self.addr[self.i] + self.fill, self.slot - self.fill

    def commit(self, blk, offset, n):
        self.fill += n
        if self.fill == self.slot:
            self._flush()

    def _flush(self):
        if not self.fill:
            return
        torch = self.torch
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            self.cur[self.cur_off:self.cur_off + self.fill].copy_(self.ring[self.i][:self.fill], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.events[self.i] = ev
        self.i = (self.i + 1) % len(self.ring)
        self.fill, self.cur = 0, None

    def close(self, blk):
        self._flush()

    def finish(self):
        self._flush()
        torch = self.torch
        with torch.cuda.device(self.device):
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return ev


class NpzStreamDecoder:
    """Incremental decoder of an npz archive (a ZIP of ``.npy`` members, stored or deflated)
    fed in arbitrary chunks: the native streaming reader of libfednpz.so (fnpz_stream_*,
    include/fednpz.h) parses local headers and inflates each payload straight into the
    sink's window (no GIL held while it inflates, no intermediate Python bytes). Payload
    bytes go to a sink (:class:`HostSink` by default: ``alloc(nbytes)`` returns a writable
    uint8 numpy buffer for one member); ``finish()`` returns ``[(name, dtype, shape,
    handle)]`` in archive order once the archive ended cleanly."""

    def __init__(self, alloc=None, sink=None):
        from .codec import Entry, load_lib
        self.lib = load_lib()
        self.sink = sink if sink is not None else HostSink(alloc)
        self.h = ctypes.c_void_p()
        self._check(self.lib.fnpz_stream_open(ctypes.byref(self.h)))
        self.ent = Entry()
        self.ev = ctypes.c_int()
        self.n = ctypes.c_int64()
        self.cur = None           # [name, dtype, shape, handle, nbytes, filled]
        self.done = []
        self.finished = False

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            self.lib.fnpz_stream_close(h)

    def _check(self, rc):
        if rc:
            raise DecodeError(f"fednpz status {rc}: {self.lib.fnpz_last_error().decode(errors='replace')}")

    def feed(self, data):
        if self.finished:
            return
        self._check(self.lib.fnpz_stream_feed(self.h, bytes(data), len(data)))
        self._drain()

    def _drain(self):
        lib, ev, n = self.lib, self.ev, self.n
        while True:
            c = self.cur
            if c is not None and c[5] < c[4]:
                addr, cap = self.sink.window(c[3], c[5])
                cap = min(cap, c[4] - c[5])
            else:
                addr, cap = None, 0
            self._check(lib.fnpz_stream_next(self.h, addr, cap, ctypes.byref(ev), ctypes.byref(self.ent),
                                             ctypes.byref(n)))
            e = ev.value
            if e == EV_NEED_INPUT:
                return
            if e == EV_DATA:
                self.sink.commit(c[3], c[5], n.value)
                c[5] += n.value
            elif e == EV_MEMBER:
                self.cur = self._open_member()
            elif e == EV_MEMBER_END:
                self.sink.close(c[3])
                self.done.append((c[0], c[1], c[2], c[3]))
                self.cur = None
            elif e == EV_END:
                self.finished = True
                return

    def _open_member(self):
        ent = self.ent
        name = ent.name.decode(errors="replace")
        try:
            dtype = np.dtype(ent.descr.decode())
        except TypeError as exc:
            raise DecodeError(f"member {name}: dtype {ent.descr!r}: {exc}") from None
        if dtype.hasobject:
            raise DecodeError(f"member {name}: object arrays are not decoded (allow_pickle=False)")
        shape = tuple(ent.shape[d] for d in range(ent.ndim))
        if ent.fortran_order and len(shape) > 1:
            raise DecodeError(f"member {name}: Fortran-ordered arrays take the normal path")
        nbytes = int(ent.nbytes)
        if nbytes != int(np.prod(shape, dtype=np.int64)) * dtype.itemsize:
            raise DecodeError(f"member {name}: {nbytes} payload bytes for {dtype} {shape}")
        return [name, dtype, shape, self.sink.open(nbytes), nbytes, 0]

    def finish(self):
        """Check the archive ended cleanly; returns the decoded members."""
        if not self.finished:
            self._drain()
        if not self.finished:
            raise DecodeError("archive truncated before its central directory")
        return self.done


def _ordered(members):
    """numpyhelper.load order: a[str(i)] for i in range(len(files)) (numpyhelper.py:180-182)."""
    by_name = {m[0]: m for m in members}
    try:
        return [by_name[str(i)] for i in range(len(members))]
    except KeyError as e:
        raise DecodeError(f"npz keys are not 0..{len(members) - 1}: missing {e}") from None


class DecodedUpdate:
    """A fully decoded npz update in host memory: arrays in FEDn's key order ("0", "1", ...)."""

    __slots__ = ("arrays", "nbytes", "pinned")

    def __init__(self, members, pinned):
        self.arrays = [view.view(dtype).reshape(shape) for _, dtype, shape, view in _ordered(members)]
        self.nbytes = sum(a.nbytes for a in self.arrays)
        self.pinned = pinned          # keeps the pinned blocks alive


class DeviceDecodedUpdate:
    """An update decoded during its upload straight into HBM (:class:`DeviceSink`): one
    device block (uint8) per tensor in FEDn's key order, valid once ``ready`` has fired."""

    __slots__ = ("shapes", "dtypes", "blocks", "ready", "device", "nbytes", "budget_fin", "__weakref__")

    def __init__(self, members, ready, device):
        self.budget_fin = None            # the HBM budget's hold on the decode (budget.HbmBudget.take)
        members = _ordered(members)
        self.shapes = [tuple(shape) for _, _, shape, _ in members]
        self.dtypes = [dtype for _, dtype, _, _ in members]
        self.blocks = [blk for _, _, _, blk in members]
        self.ready, self.device = ready, device
        self.nbytes = sum(int(np.prod(sh, dtype=np.int64)) * dt.itemsize for sh, dt in zip(self.shapes, self.dtypes))


class StreamingUpload:
    """Wrap a FEDn ``ModelService`` so uploads are decoded while they stream in.

    ``Upload`` passes every request to the wrapped service's ``Upload`` unchanged (the temp file
    is still written) and feeds the chunk bytes to a decoder worker. On the ``OK`` request the
    decoded update is offered to ``handler`` (:meth:`StagingUpdateHandler.adopt`). Decoded but
    unclaimed uploads (e.g. the combiner's own global models) are dropped beyond
    ``max_unclaimed_bytes``. Every other attribute is the wrapped service's."""

    def __init__(self, inner, handler, workers=4, pinned=True, device_decode=True, slot=8 << 20, ring=4,
                 upload=None, max_queued_chunks=512, max_queued_bytes=None):
        self.inner = inner
        # bounded tee: at most 4 x workers uploads are decoded at once (a decoder waits for a worker
        # with at most max_queued_chunks chunks buffered; one that falls further behind is
        # abandoned), later ones take the normal path — the host memory the tee holds is bounded,
        # per stream and, over all streams, by max_queued_bytes (FEDN_AMD_TEE_MAX_BYTES, 2 GiB). A
        # decode slower than its upload (an inflate core does ~470 MB/s of input) lags instead of
        # giving up: the backlog left when the upload ends is much shorter than decoding it all then.
        self._free = threading.Semaphore(4 * workers)
        self.max_queued_chunks = max_queued_chunks
        self.max_queued_bytes = int(os.environ.get("FEDN_AMD_TEE_MAX_BYTES", str(2 << 30))) \
            if max_queued_bytes is None else int(max_queued_bytes)
        self._queued = 0                     # chunk bytes queued to decoders, all streams
        self._upload = upload if upload is not None else inner.Upload
        self.handler = handler
        self.pinned = pinned
        self.device_decode = device_decode and pinned
        self.slot, self.ring = slot, ring
        self._pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="fedn_amd_upload")
        self._streams = {}
        self._lock = threading.Lock()

    def _device(self):
        """Where the handler wants decoded uploads: a device (decode through DeviceSink) or
        None (host buffers, e.g. a multi-device handler that slices them itself)."""
        if not self.device_decode:
            return None
        get = getattr(self.handler, "upload_device", None)
        return get() if get is not None else None

    def _stream(self, device):
        import torch
        key = (threading.get_ident(), str(device))
        with self._lock:
            st = self._streams.get(key)
            if st is None:
                st = self._streams[key] = torch.cuda.Stream(device)
        return st

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

    def _decode(self, q, fut, device, stop):
        keep = []
        ended = False
        sink = None
        budget = getattr(self.handler, "budget", None)
        try:
            if device is not None:
                sink = DeviceSink(device, self._stream(device), self.slot, self.ring, budget)
            else:
                sink = HostSink(self._alloc(keep))
            dec = NpzStreamDecoder(sink=sink)
            while True:
                chunk = q.get()
                if chunk is None:
                    ended = True
                    break
                self._dequeued(len(chunk))
                if stop.is_set():
                    raise RuntimeError("decode abandoned: the upload outpaced the decoder")
                dec.feed(chunk)
            if stop.is_set():
                raise RuntimeError("decode abandoned: the upload outpaced the decoder")
            members = dec.finish()
            ready = sink.finish()
            if device is not None:
                upd = DeviceDecodedUpdate(members, ready, device)
                if sink.reserved:
                    budget.hold(upd, [(device, sink.reserved)])      # returned when the decode is dropped
                    sink.reserved = 0
                fut.set_result(upd)
            else:
                fut.set_result(DecodedUpdate(members, keep))
        except Exception as e:  # noqa: BLE001 — not adopted: the update takes the normal path
            if isinstance(sink, DeviceSink) and sink.reserved:
                budget.release([(device, sink.reserved)])
                sink.reserved = 0
            keep.clear()
            fut.set_exception(e)
            while not ended:                           # drain to the end of the upload
                chunk = q.get()
                ended = chunk is None
                if not ended:
                    self._dequeued(len(chunk))
        finally:
            self._free.release()

    def _dequeued(self, n):
        with self._lock:
            self._queued -= n

    def _enqueue(self, q, chunk):
        """Queue a chunk to its decoder: False (nothing queued) if its queue or the tee's byte
        budget is full."""
        with self._lock:
            if self._queued + len(chunk) > self.max_queued_bytes:
                return False
            try:
                q.put_nowait(chunk)
            except queue.Full:
                return False
            self._queued += len(chunk)
            return True

    def _start(self):
        """A decoder for a new upload, or None when too many are in flight (normal path)."""
        if not self.handler.wants_upload() or not self._free.acquire(blocking=False):
            return None
        q, fut, stop = queue.Queue(maxsize=self.max_queued_chunks), Future(), threading.Event()
        self._pool.submit(self._decode, q, fut, self._device(), stop)
        return q, fut, stop

    def Upload(self, request_iterator, context):
        if context is self.inner or context is self:
            # the service uploading to itself: ModelService.set_model passes the service as
            # the context (modelservice.py:184-195), for the combiner's own global models,
            # which no ModelUpdate will claim
            return self._upload(request_iterator, context)
        streams = {}

        def tee():
            try:
                for request in request_iterator:
                    rid = request.id
                    if request.status == MODEL_STATUS_IN_PROGRESS and request.data:
                        if rid not in streams:
                            streams[rid] = self._start()
                        st = streams[rid]
                        if st is not None and not self._enqueue(st[0], bytes(request.data)):
                            st[2].set()                 # decoder too far behind: give this upload up
                            try:                        # drop the backlog (never block the upload)
                                while True:
                                    c = st[0].get_nowait()
                                    if c is not None:
                                        self._dequeued(len(c))
                            except queue.Empty:
                                pass
                            st[0].put_nowait(None)
                            streams[rid] = None
                    if request.status == MODEL_STATUS_OK and not request.data and streams.get(rid) is not None:
                        q, fut, _ = streams.pop(rid)
                        q.put(None)
                        self.handler.adopt(rid, fut)
                    yield request
            finally:                                   # stream ended (or Upload gave up) without OK
                for st in streams.values():
                    if st is not None:
                        st[0].put(None)
                streams.clear()

        return self._upload(tee(), context)

    def close(self):
        self._pool.shutdown(wait=True)


class StreamingUploadMixin:
    """The same, as a mixin of FEDn's ``ModelService`` (the gRPC server registers the model
    servicer only if it IS a ``ModelServiceServicer``, grpc/server.py:57-58)::

        class StreamingModelService(StreamingUploadMixin, ModelService): pass

    ``attach(handler)`` starts decoding uploads for that handler; until then, and after
    ``detach()``, ``Upload`` is the base class's unchanged."""

    _streaming = None

    def attach(self, handler, **kw):
        base = super(StreamingUploadMixin, self).Upload
        self._streaming = StreamingUpload(self, handler, upload=base, **kw)
        return self._streaming

    def detach(self):
        s, self._streaming = self._streaming, None
        if s is not None:
            s.close()

    def Upload(self, request_iterator, context):
        s = self._streaming
        if s is None:
            return super().Upload(request_iterator, context)
        return s.Upload(request_iterator, context)


class AdoptedUploads:
    """Decoded uploads waiting for their ModelUpdate, bounded by bytes (oldest dropped first) and
    by age: an upload whose ModelUpdate never arrives (the client died after uploading, or the
    update was rejected) is dropped after ``ttl`` seconds, so its host / HBM blocks are freed."""

    def __init__(self, max_bytes=16 << 30, ttl=3600.0):
        self.max_bytes = max_bytes
        self.ttl = ttl
        self._lock = threading.Lock()
        self._items = OrderedDict()       # id -> Future[DecodedUpdate]
        self._born = {}

    def put(self, rid, fut):
        now = time.monotonic()
        with self._lock:
            self._items[rid] = fut
            self._born[rid] = now
            for k in [k for k, t in self._born.items() if now - t > self.ttl]:
                self._items.pop(k, None)
                self._born.pop(k, None)
            total, drop = 0, []
            for k, f in reversed(self._items.items()):
                if f.done() and f.exception() is None:
                    total += f.result().nbytes
                    if total > self.max_bytes:
                        drop.append(k)
            for k in drop:
                self._items.pop(k, None)
                self._born.pop(k, None)

    def pop(self, rid):
        with self._lock:
            self._born.pop(rid, None)
            return self._items.pop(rid, None)
