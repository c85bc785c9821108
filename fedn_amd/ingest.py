"""Streaming ingest: stage client updates into HBM when they
ARRIVE, not when the round aggregates.

In FEDn an update reaches the combiner through ``ModelService.Upload`` (modelservice.py:
198-221) and ``UpdateHandler.on_model_update`` (updatehandler.py:46-70), which only
validates and enqueues it; decoding (npz inflate, updatehandler.py:90-117) and all
arithmetic happen later, serially, inside ``combine_models`` (fedavg.py:56, 68). Here
:class:`StagingUpdateHandler` wraps the combiner's UpdateHandler: ``on_model_update``
enqueues the update in arrival order exactly as before AND hands it to a worker pool
that decodes it (the wrapped handler's own ``load_model_update`` with the round's
helper) and copies it into a device buffer on its own HIP stream. When the aggregator
later calls ``load_model_update`` it receives a :class:`StagedModel` (already in HBM),
which the pipelines in staging.py fold without any host work. FIFO order, metadata
handling and error semantics are unchanged: a decode that fails re-raises from
``load_model_update``, where the aggregator's per-update error handling (fedavg.py:
137-140) logs and skips it, as FEDn would.
"""
import json
import os
import queue
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from . import reuse
from .budget import HbmBudget
from .layout import Layout, spread


class _HostSide(Exception):
    """The HBM budget cannot hold this update: leave it host-side (folded through the host path)."""


class StagedModel:
    """One decoded client update resident in HBM: flat grouped layout (layout.py) in
    ``dev`` (uint8), ready once ``ready`` (an event on the staging stream) has fired.
    ``host`` returns the update as host arrays (needed only when it is the round's sole
    update, fedavg.py:65-66): the decoded arrays if they were kept, else a D2H copy."""

    __slots__ = ("layout", "dev", "ready", "_host", "__weakref__")

    def __init__(self, layout, dev, ready, host=None):
        self.layout, self.dev, self.ready, self._host = layout, dev, ready, host

    @property
    def host(self):
        if self._host is None:
            self.ready.synchronize()
            flat = self.dev.to("cpu").numpy()
            out = [None] * len(self.layout.shapes)
            for dt in self.layout.groups:
                self.layout.unpack_group(self.layout.group_view(flat, dt), dt, out, copy=False)
            self._host = out
        return self._host

    # list-like access to the host arrays, so code written for list[np.ndarray] still works
    def __len__(self):
        return len(self.layout.shapes)

    def __getitem__(self, i):
        return self.host[i]

    def __iter__(self):
        return iter(self.host)


class ShardedStagedModel:
    """One decoded client update resident in HBM as parameter slices over several devices
    (Layout.shard_geometry, the layout of multidev.py): ``bufs[d]`` holds device d's [lo, hi)
    of every dtype group, ready once ``ready[d]`` has fired. The multi-device pipelines fold it
    in place; ``host`` reassembles host arrays only when needed (a round's sole update)."""

    __slots__ = ("layout", "devices", "bounds", "dev_off", "bufs", "ready", "_host", "__weakref__")

    def __init__(self, layout, devices, bufs, ready, host=None):
        self.layout, self.devices, self.bufs, self.ready, self._host = layout, list(devices), bufs, ready, host
        self.bounds, self.dev_off, _ = layout.shard_geometry(len(self.devices))

    def view(self, d, dt):
        """Device d's slice of group ``dt`` (flat torch view)."""
        lo, hi = self.bounds[dt][d]
        off = self.dev_off[d][dt]
        return self.bufs[d][off:off + (hi - lo) * dt.itemsize].view(_torch_dtype(dt))

    @property
    def host(self):
        if self._host is None:
            out = [None] * len(self.layout.shapes)
            for dt in self.layout.groups:
                flat = np.empty(self.layout.group_elems[dt], dtype=dt)
                for d in range(len(self.devices)):
                    lo, hi = self.bounds[dt][d]
                    if hi > lo:
                        self.ready[d].synchronize()
                        flat[lo:hi] = self.view(d, dt).cpu().numpy()
                self.layout.unpack_group(flat, dt, out, copy=False)
            self._host = out
        return self._host

    def __len__(self):
        return len(self.layout.shapes)

    def __getitem__(self, i):
        return self.host[i]

    def __iter__(self):
        return iter(self.host)


def _torch_dtype(dt):
    from .ops import torch_dtype
    return torch_dtype(dt)


def stage_sharded(layout, pinned, devices, streams, host=None):
    """Copy each device's slices of a pinned, layout-packed update (``pinned``: uint8 tensor)
    to that device on ``streams[d]`` (every device over its own link, concurrently); returns a
    :class:`ShardedStagedModel` once the copies no longer read ``pinned``."""
    bounds, dev_off, dev_bytes = layout.shard_geometry(len(devices))
    bufs, ready = [], []
    for d, dv in enumerate(devices):
        with torch.cuda.device(dv):
            with torch.cuda.stream(streams[d]):   # allocated on the stream that writes it
                buf = reuse.watch(torch.empty(dev_bytes[d], dtype=torch.uint8, device=dv), streams[d])
                for dt in layout.groups:
                    lo, hi = bounds[dt][d]
                    if hi > lo:
                        g0, o = layout.group_byte_offset[dt], dev_off[d][dt]
                        buf[o:o + (hi - lo) * dt.itemsize].copy_(
                            pinned[g0 + lo * dt.itemsize:g0 + hi * dt.itemsize], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(streams[d])
        bufs.append(buf)
        ready.append(ev)
    for ev in ready:
        ev.synchronize()
    return ShardedStagedModel(layout, devices, bufs, ready, host)


def stage_arrays(arrays, device, stream):
    """Pack host ``arrays`` into pinned memory and copy them to a new device buffer on
    ``stream``; returns a :class:`StagedModel` (the H2D may still be in flight)."""
    arrays = [np.asarray(a) for a in arrays]
    layout = Layout.of(arrays)
    pinned = torch.empty(layout.nbytes, dtype=torch.uint8, pin_memory=True)
    layout.pack(arrays, pinned.numpy())
    ready = torch.cuda.Event()
    with torch.cuda.stream(stream):                 # allocated on the stream that writes it
        dev = reuse.watch(torch.empty(layout.nbytes, dtype=torch.uint8, device=device), stream)
        dev.copy_(pinned, non_blocking=True)
        ready.record(stream)
    # the pinned block returns to torch's caching host allocator only after the copy
    ready.synchronize()
    del pinned
    return StagedModel(layout, dev, ready, arrays)


def stage_npz(data, device, stream):
    """Inflate an npz update (native codec) straight into a pinned buffer laid out for the
    pipelines, then copy it to HBM on ``stream``: no temp file, no numpy arrays, no pack."""
    from . import codec

    layout, pinned = codec.load_npz_into_layout(
        data, lambda nbytes: torch.empty(nbytes, dtype=torch.uint8, pin_memory=True))
    return stage_pinned(layout, pinned, device, stream)


def stage_pinned(layout, pinned, device, stream, host=None):
    """Copy a pinned, layout-packed update (uint8 tensor) to a new device buffer on ``stream``."""
    ready = torch.cuda.Event()
    with torch.cuda.stream(stream):                 # allocated on the stream that writes it
        dev = reuse.watch(torch.empty(layout.nbytes, dtype=torch.uint8, device=device), stream)
        dev.copy_(pinned, non_blocking=True)
        ready.record(stream)
    ready.synchronize()
    return StagedModel(layout, dev, ready, host)


def _member_spans(layout, dt, lo, hi):
    """(tensor index, first element within the tensor, element count, element offset from
    ``lo``) for every tensor of group ``dt`` that overlaps the group range [lo, hi)."""
    out = []
    for i, off in layout.members[dt]:
        a, b = max(lo, off), min(hi, off + layout.sizes[i])
        if b > a:
            out.append((i, a - off, b - a, a - lo))
    return out


def stage_decoded(decoded, device, stream):
    """Copy an update decoded during its upload into a new device buffer in the pipelines'
    layout on ``stream``, tensor by tensor: from HBM (upload.DeviceDecodedUpdate, decoded
    through DeviceSink: a D2D copy per tensor once its H2D copies have landed) or from one
    pinned block per tensor (upload.DecodedUpdate): no pack, no second host copy."""
    from .upload import DeviceDecodedUpdate
    if isinstance(decoded, DeviceDecodedUpdate):
        layout = Layout(decoded.shapes, decoded.dtypes)
        ready = torch.cuda.Event()
        with torch.cuda.stream(stream):
            dev = reuse.watch(torch.empty(layout.nbytes, dtype=torch.uint8, device=device), stream)
            stream.wait_event(decoded.ready)
            for dt in layout.groups:
                g0 = layout.group_byte_offset[dt]
                for i, e0, n, o in _member_spans(layout, dt, 0, layout.group_elems[dt]):
                    dev[g0 + o * dt.itemsize:g0 + (o + n) * dt.itemsize].copy_(
                        decoded.blocks[i][e0 * dt.itemsize:(e0 + n) * dt.itemsize], non_blocking=True)
            ready.record(stream)
        ready.synchronize()               # the per-tensor blocks are released after the copies
        return StagedModel(layout, dev, ready)
    layout = Layout.of(decoded.arrays)
    ready = torch.cuda.Event()
    with torch.cuda.stream(stream):
        dev = reuse.watch(torch.empty(layout.nbytes, dtype=torch.uint8, device=device), stream)
        for dt in layout.groups:
            g0 = layout.group_byte_offset[dt]
            for i, e0, n, o in _member_spans(layout, dt, 0, layout.group_elems[dt]):
                src = torch.from_numpy(decoded.arrays[i].reshape(-1).view(np.uint8))
                dev[g0 + o * dt.itemsize:g0 + (o + n) * dt.itemsize].copy_(src, non_blocking=True)
        ready.record(stream)
    ready.synchronize()
    return StagedModel(layout, dev, ready)


def stage_decoded_sharded(decoded, devices, streams):
    """:func:`stage_decoded` for the multi-device layout: device d receives only the parts of
    each tensor inside its parameter slices (Layout.shard_geometry), over its own link."""
    layout = Layout.of(decoded.arrays)
    bounds, dev_off, dev_bytes = layout.shard_geometry(len(devices))
    flat = {i: torch.from_numpy(a.reshape(-1).view(np.uint8)) for i, a in enumerate(decoded.arrays)}
    bufs, ready = [], []
    for d, dv in enumerate(devices):
        with torch.cuda.device(dv):
            with torch.cuda.stream(streams[d]):   # allocated on the stream that writes it
                buf = reuse.watch(torch.empty(dev_bytes[d], dtype=torch.uint8, device=dv), streams[d])
                for dt in layout.groups:
                    lo, hi = bounds[dt][d]
                    base, isz = dev_off[d][dt], dt.itemsize
                    for i, e0, n, o in _member_spans(layout, dt, lo, hi):
                        buf[base + o * isz:base + (o + n) * isz].copy_(flat[i][e0 * isz:(e0 + n) * isz],
                                                                       non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(streams[d])
        bufs.append(buf)
        ready.append(ev)
    for ev in ready:
        ev.synchronize()
    return ShardedStagedModel(layout, devices, bufs, ready)


class Reaper:
    """One daemon thread that drops the references it is handed: a large free (munmap of a host
    block, hipHostUnregister, the caching allocators' bookkeeping) happens there instead of on the
    round thread. ``close()`` waits until everything handed over is gone."""

    def __init__(self):
        self._q = queue.Queue()
        self._t = None
        self._lock = threading.Lock()

    def drop(self, obj):
        with self._lock:
            if self._t is None:
                self._t = threading.Thread(target=self._run, name="fedn_amd_reaper", daemon=True)
                self._t.start()
        self._q.put(obj)

    def _run(self):
        while True:
            obj = self._q.get()
            del obj
            self._q.task_done()

    def close(self):
        if self._t is not None:
            self._q.join()


class StagingUpdateHandler:
    """Drop-in wrapper of a FEDn ``UpdateHandler`` that decodes + stages updates on arrival.

    helper   the round's helper (FEDn: ``get_helper(config["helper_type"])``); used for decoding
             when the update is not available as raw npz bytes
    workers  decode/H2D threads (each with its own HIP stream)
    native_decode  take the raw npz bytes (UpdateHandler.load_model_update_byte,
             updatehandler.py:119-144) and inflate them with fedn_amd.codec straight into
             pinned memory in the pipelines' layout
    devices  several devices (argument or FEDN_AMD_DEVICES, as the aggregators use): every
             update is staged as parameter slices over them (ShardedStagedModel), each device
             receiving only its slice over its own link, for multidev.py's pipelines
    hbm_budget  budget.HbmBudget (default: FEDN_AMD_HBM_BUDGET, else 3/4 of the free HBM): an
             update that would exceed it stays host-side and is loaded by the aggregator through
             the wrapped handler (decoded then, as FEDn does) — never an OOM, never a dropped client
    Every attribute not defined here (``model_updates``, ``next_model_update``, ``load_model``,
    ``waitforit``, ...) is the wrapped handler's.
    """

    stages_on_arrival = True       # aggregatorbase.queued_updates: loads are already done

    def __init__(self, inner, helper=None, device=None, workers=4, native_decode=True, devices=None,
                 max_unclaimed_upload_bytes=16 << 30, hbm_budget=None, delete_workers=None):
        from .upload import AdoptedUploads
        self.inner = inner
        # HBM admission control (budget.py): an update the budget cannot hold is not staged; the
        # aggregator loads and folds it from the host at its place in the FIFO
        self.budget = hbm_budget if hbm_budget is not None else HbmBudget()
        self.host_side = 0              # updates left host-side by the budget (or an HBM OOM)
        self._uploads = AdoptedUploads(max_unclaimed_upload_bytes)
        if devices is None:
            from .aggregators.fedavg import env_devices
            devices = env_devices()
        self.devices = [torch.device(d) for d in devices] if devices and len(devices) > 1 else None
        self.native_decode = native_decode
        self.helper = helper
        self.device = torch.device(device) if device is not None else None
        self._pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="fedn_amd_ingest")
        self._streams = {}
        self._lock = threading.Lock()
        self._staged = {}
        self._reaper = Reaper()
        # the wrapped store's deletes of one round run concurrently on this many threads and have all
        # completed when combine_models returns (finish_deletes); 0 = one after another inline
        if delete_workers is None:
            delete_workers = int(os.environ.get("FEDN_AMD_DELETE_WORKERS", "8"))
        self.delete_workers = max(0, int(delete_workers))
        self._deleter = None
        self._deletes = []                # (model_update, future) not waited for yet
        self._in_round = False            # begin_deletes .. finish_deletes: store deletes side by side
        self.delete_times = {"plugin_s": 0.0, "store_s": 0.0, "wait_s": 0.0, "count": 0}

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def _device(self):
        if self.device is None:
            from .aggregators.fedavg import default_device
            self.device = default_device()
        return self.device

    def _stream(self, dev=None):
        dev = dev if dev is not None else self._device()
        key = (threading.get_ident(), str(dev))
        with self._lock:
            st = self._streams.get(key)
            if st is None:
                st = self._streams[key] = torch.cuda.Stream(dev)
        return st

    # -- updates decoded while they uploaded (upload.StreamingUpload) -------------------------
    def wants_upload(self):
        """Whether uploads should be decoded as they stream in: npz helpers only (binaryhelper
        holds raw float64 bytes; androidhelper updates are folded from the host)."""
        from .staging import helper_kind
        return self.native_decode and helper_kind(self.helper, strict=False) not in ("binaryhelper", "androidhelper", "unknown")

    def upload_device(self):
        """The device uploads are decoded into (upload.DeviceSink), or None when updates are
        staged as parameter slices over several devices (decoded to host, sliced at staging)."""
        return None if self.devices else self._device()

    def adopt(self, model_id, fut):
        """Hold the decode of upload ``model_id`` (Future of upload.DecodedUpdate) for the
        ModelUpdate that names it (model_update_id == the upload's request id)."""
        self._uploads.put(model_id, fut)

    def _decoded_upload(self, model_update):
        fut = self._uploads.pop(model_update.model_update_id)
        if fut is None:
            return None
        try:
            return fut.result()
        except Exception:  # noqa: BLE001 — not decodable while streaming: take the normal path
            return None

    def _metadata(self, model_update):
        """training_metadata as UpdateHandler.load_model_update returns it (updatehandler.py:106-116)."""
        metadata = json.loads(model_update.meta)
        config = json.loads(metadata["config"]) if "config" in metadata else json.loads(model_update.config)
        training_metadata = metadata["training_metadata"]
        if "round_id" in config:
            training_metadata["round_id"] = config["round_id"]
        return training_metadata

    def _stage_sharded(self, model_update, parts):
        """Stage as parameter slices over the devices — or on the first one alone when the model
        is small (layout.spread: the rule the aggregators apply to pick their pipeline)."""
        decoded = self._decoded_upload(model_update)
        if decoded is not None and hasattr(decoded, "arrays"):
            devs = spread(self.devices, Layout.of(decoded.arrays).nbytes)
            self._admit(Layout.of(decoded.arrays), devs, parts)
            if len(devs) == 1:
                with torch.cuda.device(devs[0]):
                    return stage_decoded(decoded, devs[0], self._stream(devs[0])), self._metadata(model_update)
            return stage_decoded_sharded(decoded, devs, [self._stream(dv) for dv in devs]), \
                self._metadata(model_update)
        if self._native():
            try:
                data, metadata = self.inner.load_model_update_byte(model_update)
            except Exception:  # noqa: BLE001 — not held as bytes: decode through the helper
                data = None
            if data is not None:
                from . import codec
                try:
                    lay = codec.npz_layout(data)          # directory only: admit before decoding
                    self._admit(lay, spread(self.devices, lay.nbytes), parts)
                    layout, pinned = codec.load_npz_into_layout(
                        data, lambda nbytes: torch.empty(nbytes, dtype=torch.uint8, pin_memory=True))
                    return self._stage_packed(layout, pinned), metadata
                except codec.CodecError:
                    pass     # e.g. Fortran-ordered members: decode through the helper (np.load) below
        arrays, metadata = self.inner.load_model_update(model_update, self.helper)
        arrays = [np.asarray(a) for a in arrays]
        layout = Layout.of(arrays)
        if not parts:
            self._admit(layout, spread(self.devices, layout.nbytes), parts)
        pinned = torch.empty(layout.nbytes, dtype=torch.uint8, pin_memory=True)
        layout.pack(arrays, pinned.numpy())
        return self._stage_packed(layout, pinned, arrays), metadata

    def _stage_packed(self, layout, pinned, host=None):
        devs = spread(self.devices, layout.nbytes)
        if len(devs) == 1:
            with torch.cuda.device(devs[0]):
                return stage_pinned(layout, pinned, devs[0], self._stream(devs[0]), host)
        return stage_sharded(layout, pinned, devs, [self._stream(dv) for dv in devs], host)

    def _native(self):
        """Raw-bytes decode applies to npz (numpyhelper / fednamdhelper); binaryhelper's raw
        float64 bytes go through the helper's own load."""
        from .staging import helper_kind
        return self.native_decode and helper_kind(self.helper, strict=False) not in ("binaryhelper", "unknown") and \
            hasattr(self.inner, "load_model_update_byte")

    def _admit(self, layout, devs, parts):
        """Reserve HBM for ``layout`` on ``devs`` (its slices when several) or raise _HostSide."""
        if len(devs) == 1:
            want = [(devs[0], layout.nbytes)]
        else:
            _, _, dev_bytes = layout.shard_geometry(len(devs))
            want = list(zip(devs, dev_bytes))
        self._admit_bytes(want, parts)

    def _admit_bytes(self, want, parts):
        if not self.budget.reserve(want):
            raise _HostSide()
        parts.extend(want)

    def _stage(self, model_update):
        """Stage one update within the HBM budget: (StagedModel, metadata), or None when it stays
        host-side (the budget is full, or HBM ran out): load_model_update then takes it from the
        wrapped handler."""
        parts = []
        try:
            staged, metadata = self._stage_device(model_update, parts)
        except _HostSide:
            self.budget.release(parts)        # a decode's reservation taken over before the refusal
            with self._lock:
                self.host_side += 1
            return None
        except torch.cuda.OutOfMemoryError:
            self.budget.release(parts)
            with self._lock:
                self.host_side += 1
            return None
        except BaseException:
            self.budget.release(parts)
            raise
        if parts:
            self.budget.hold(staged, parts)
        return staged, metadata

    def _stage_device(self, model_update, parts):
        if self.devices:
            return self._stage_sharded(model_update, parts)
        dev = self._device()
        decoded = self._decoded_upload(model_update)
        if decoded is not None:
            from .upload import DeviceDecodedUpdate
            if isinstance(decoded, DeviceDecodedUpdate):
                lay = Layout(decoded.shapes, decoded.dtypes)
                # the decode's own reservation becomes the staged copy's: only the difference (the
                # layout's alignment padding) is reserved anew, so a decoded update is not counted
                # twice against the budget while it is copied into the pipelines' layout
                moved = sum(n for _, n in self.budget.take(decoded))      # reserved on dev by the sink
                if lay.nbytes > moved:
                    try:
                        self._admit_bytes([(dev, lay.nbytes - moved)], [])
                    except _HostSide:
                        self.budget.release([(dev, moved)])
                        raise
                elif moved > lay.nbytes:
                    self.budget.release([(dev, moved - lay.nbytes)])
                parts.append((dev, lay.nbytes))
            else:
                lay = Layout.of(decoded.arrays)
                self._admit(lay, [dev], parts)
            with torch.cuda.device(dev):
                return stage_decoded(decoded, dev, self._stream()), self._metadata(model_update)
        if self._native():
            try:
                data, metadata = self.inner.load_model_update_byte(model_update)
            except Exception:  # noqa: BLE001 — not held as bytes: decode through the helper
                data = None
            if data is not None:
                from . import codec
                try:
                    self._admit(codec.npz_layout(data), [dev], parts)   # directory only: before decoding
                    with torch.cuda.device(dev):
                        return stage_npz(data, dev, self._stream()), metadata
                except codec.CodecError:
                    pass     # e.g. Fortran-ordered members: decode through the helper (np.load) below
        arrays, metadata = self.inner.load_model_update(model_update, self.helper)
        if not parts:
            self._admit(Layout.of([np.asarray(a) for a in arrays]), [dev], parts)
        with torch.cuda.device(dev):
            return stage_arrays(arrays, dev, self._stream()), metadata

    def on_model_update(self, model_update):
        """Validate as FEDn does (updatehandler.py:72-88), start staging, then enqueue."""
        try:
            json.loads(model_update.meta)["training_metadata"]["num_examples"]
            valid = True
        except (KeyError, TypeError, ValueError):
            valid = False
        from .staging import helper_kind
        if valid and helper_kind(self.helper, strict=False) in ("androidhelper", "unknown"):
            # one flat array with its own fold rule (or a helper the aggregators refuse): the
            # aggregator takes it from the host
            valid = False
        if valid:
            self._device()
            with self._lock:
                self._staged[model_update.model_update_id] = self._pool.submit(self._stage, model_update)
        else:
            self._uploads.pop(model_update.model_update_id)   # FEDn drops the update: free its decode
        return self.inner.on_model_update(model_update)

    def load_model_update(self, model_update, helper):
        with self._lock:
            fut = self._staged.pop(model_update.model_update_id, None)
        if fut is None:                       # arrived before the wrapper was installed
            return self.inner.load_model_update(model_update, helper)
        res = fut.result()
        if res is None:                       # left host-side by the HBM budget: FEDn's own load
            return self.inner.load_model_update(model_update, helper)
        return res

    def delete_model(self, model_update):
        """FEDn's per-update delete (updatehandler.py:31-33, called in the aggregation loop,
        fedavg.py:73-74). This handler's own copies of the update (a staged future, a decoded
        upload) are handed to the reaper thread, so freeing their host / device memory never stalls
        the round. The wrapped handler's delete (the store's: ``os.remove`` of the update's file,
        tempmodelstorage.py:66-76, 25-40 ms for 400 MB) runs on a small pool, the round's deletes
        side by side, and :meth:`finish_deletes` — called by the aggregators before
        ``combine_models`` returns — waits for all of them: every folded update is deleted by then,
        as in the reference, and an exception from one is logged as the reference logs it
        (fedavg.py:75-78). ``delete_workers=0`` (FEDN_AMD_DELETE_WORKERS=0) runs them inline.
        ``delete_times`` accumulates the parts (seconds: plug-in, store, waiting) and the count."""
        t0 = time.perf_counter()
        with self._lock:
            staged = self._staged.pop(model_update.model_update_id, None)
        upload = self._uploads.pop(model_update.model_update_id)
        if staged is not None or upload is not None:
            self._reaper.drop((staged, upload))
        del staged, upload
        t1 = time.perf_counter()
        d = self.delete_times
        d["plugin_s"] += t1 - t0
        d["count"] += 1
        if self.delete_workers == 0 or not self._in_round:
            # inline (as the reference) unless inside an aggregator's round: a delete made outside
            # combine_models (a hook's own loop) would otherwise be waited for by nobody
            ok = self.inner.delete_model(model_update)
            d["store_s"] += time.perf_counter() - t1
            return ok
        if self._deleter is None:
            self._deleter = ThreadPoolExecutor(max_workers=self.delete_workers, thread_name_prefix="fedn_amd_delete")
        self._deletes.append((model_update, self._deleter.submit(self._timed_delete, model_update)))
        return None

    def _timed_delete(self, model_update):
        t = time.perf_counter()
        try:
            return self.inner.delete_model(model_update)
        finally:
            with self._lock:
                self.delete_times["store_s"] += time.perf_counter() - t

    def begin_deletes(self):
        """An aggregator's round starts: its store deletes may run side by side until
        :meth:`finish_deletes` (which the aggregator calls however the round ends)."""
        self._in_round = True

    def finish_deletes(self):
        """Wait for every store delete handed to the pool; returns [(model_update, exception)] of
        the ones that raised (the aggregator logs them as the reference logs a failed update).
        Deletes after this run inline again until the next :meth:`begin_deletes`."""
        self._in_round = False
        pending, self._deletes = self._deletes, []
        t = time.perf_counter()
        failed = []
        for mu, fut in pending:
            try:
                fut.result()
            except Exception as e:  # noqa: BLE001 — fedavg.py:75-78 logs it and goes on
                failed.append((mu, e))
        self.delete_times["wait_s"] += time.perf_counter() - t
        return failed

    def close(self):
        self.finish_deletes()
        if self._deleter is not None:
            self._deleter.shutdown(wait=True)
        self._pool.shutdown(wait=True)
        self._reaper.close()
