"""Device pipelines behind the aggregator plug-ins: pinned H2D staging overlapped with the fold.

FEDn hands the aggregator one client update at a time, in FIFO order, as host
``list[np.ndarray]`` (UpdateHandler.load_model_update, updatehandler.py:90-117). That
order IS the fold order, so each update is folded on arrival:

    host: pack update k+1 into pinned slot  |  copy stream: H2D slot k+1  |  compute stream: fold k

A ring of pinned-host/device slot pairs decouples the three: the host waits only for
the H2D that last read a pinned slot; the copy stream waits (GPU-side event) only for
the fold that last read a device slot. The running aggregate (and FedOpt's pseudo-
gradient, m and v) never leaves HBM until the round's result is copied back.

Updates that are ALREADY in HBM when the aggregator sees them (a StagedModel from the
streaming ingest, ingest.py — the normal case at round end) are not folded one launch each:
they queue and fold together in one multi-client launch (up to BATCH per flush), which reads
each update once and the running aggregate once per batch instead of once per update
(FedAvg 64 x 100 M: 26 GB instead of 77 GB; FedOpt: the fused pseudo-gradient + server step,
P*(4K+48) bytes, instead of ~P*(28K) with pg through HBM per update). The result's D2H
overlaps that final fold chunk by chunk. The fold order, and so every bit, is unchanged:
a multi-client launch replays the same recurrence (tests/test_gpu_parity.py).
"""
import os
import time

import numpy as np
import torch

from . import mixed, ops, reuse
from .ingest import StagedModel
from .layout import Layout, fast_admission, parallel_copy, start_pack_into, wait_pack_jobs


BATCH = 64                    # device-resident updates folded per launch (the kernarg client table)
MAX_CHUNKS = int(os.environ.get("FEDN_AMD_MAX_CHUNKS", "16"))  # the round's last launch is split into at most this many chunks, each
MIN_CHUNK_BYTES = 8 << 20     # chunk's D2H (and FedOpt's old-model H2D) overlapping the next chunk
RING_BYTES = 64 << 20         # pinned ring piece for host -> device streaming of the global model
# host updates of at most SMALL_UPDATE_BYTES (a packed model) are batched: packed on arrival into a
# pinned arena of up to BATCH updates / ARENA_BYTES, which reaches HBM in ONE copy right before ONE
# multi-client launch folds them all — for small models the per-update H2D, events and launch
# (~0.1 ms of host work each) cost far more than the bytes; larger updates fold on arrival
SMALL_UPDATE_BYTES = 4 << 20
ARENA_BYTES = 64 << 20
ARENA_UPLOAD_EVERY = 16       # an arena's packed updates go to HBM in parts of this many, while later ones load
# a large host update is packed into its pinned slot in pieces of STAGE_PIECE bytes, each piece's
# H2D enqueued as soon as it is packed: the pack of piece j + 1 overlaps the DMA of piece j, so a
# round's first update no longer waits for its whole pack, and a FedAvg round's LAST fold runs
# chunk by chunk behind the pieces with the result's D2H (full duplex) — see FedAvgPipeline.result
STAGE_PIECE = 32 << 20
STAGE_PIECES_MIN = 64 << 20
# a FedAvg round whose updates all wait in one arena, not yet uploaded, and hold at most this many
# bytes in total folds them straight from the pinned arena into the caller's pinned result block:
# the kernel reads and writes host memory over PCIe, with no H2D / D2H copy to enqueue and order
ZERO_COPY_BYTES = int(os.environ.get("FEDN_AMD_ZERO_COPY_BYTES", str(4 << 20)))


def _have_codec():
    """Whether libfednpz (the native gather the piecewise stage packs with) is built."""
    try:
        from . import codec
        codec.load_lib()
        return True
    except ImportError:
        return False


def chunks(n, itemsize):
    """[lo, hi) element ranges: at most MAX_CHUNKS, each >= MIN_CHUNK_BYTES, 1024-aligned."""
    if n <= 0:
        return []
    C = max(-(-n // MAX_CHUNKS), MIN_CHUNK_BYTES // itemsize)
    C = -(-C // 1024) * 1024
    return [(lo, min(n, lo + C)) for lo in range(0, n, C)]


class HostStreamer:
    """Host -> device streaming of host arrays through a small ring of pinned pieces filled by
    the pack threads: no whole-buffer concatenation or pinning (both cost more than the DMA
    for a multi-GB global model)."""

    def __init__(self, nbuf=3, nbytes=RING_BYTES):
        self.nbuf, self.nbytes = nbuf, nbytes
        self.ring, self.ev, self.i = [], [None] * nbuf, 0

    def h2d(self, parts, odt, lo, hi, dst, stream):
        """Enqueue on ``stream`` the copy of elements [lo, hi) of the concatenation of ``parts``
        ((flat host array, element offset) pairs of dtype ``odt``) into the device tensor
        ``dst`` (hi - lo elements); returns an event recorded after it."""
        if not self.ring:
            self.ring = [torch.empty(self.nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(self.nbuf)]
        isz = np.dtype(odt).itemsize
        step = self.nbytes // isz
        with torch.cuda.device(dst.device):
            for plo in range(lo, hi, step):
                phi = min(hi, plo + step)
                i = self.i
                self.i = (i + 1) % self.nbuf
                if self.ev[i] is not None:
                    self.ev[i].synchronize()            # the piece's previous H2D has read it
                buf = self.ring[i][:(phi - plo) * isz]
                view = buf.numpy().view(odt)
                for a, off in parts:                    # members overlapping [plo, phi)
                    s0, s1 = max(plo, off), min(phi, off + a.size)
                    if s0 < s1:
                        parallel_copy(view[s0 - plo:s1 - plo], a[s0 - off:s1 - off])
                with torch.cuda.stream(stream):
                    dst[plo - lo:phi - lo].copy_(buf.view(dst.dtype), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
                self.ev[i] = ev
            done = torch.cuda.Event()
            done.record(stream)
        return done


class StagingCache:
    """Staging resources an aggregator keeps from one round of a session to the next: the pinned
    host / device update slots, the small-update arenas, the copy and D2H streams and FedOpt's
    pinned ring, per (device, packed update size). A round's pipeline takes them when it is built
    and gives them back when the round's result is on the host (``_Pipeline.release``), so a
    session's later rounds allocate, pin and create nothing (at most ``keep`` layouts are kept)."""

    def __init__(self, keep=2):
        self.keep = keep
        self._res = {}

    def take(self, device, nbytes):
        return self._res.pop((str(device), nbytes), None)

    def give(self, device, nbytes, res):
        self._res.pop((str(device), nbytes), None)
        self._res[(str(device), nbytes)] = res
        while len(self._res) > self.keep:
            self._res.pop(next(iter(self._res)))


class _Slot:
    __slots__ = ("host", "host_np", "dev", "h2d_start", "h2d_done", "consumed", "used", "reserved", "pieces")

    def __init__(self, nbytes, device):
        self.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.host_np = self.host.numpy()
        self.dev = reuse.watch(torch.empty(nbytes, dtype=torch.uint8, device=device))
        self.h2d_start = torch.cuda.Event(enable_timing=True)
        self.h2d_done = torch.cuda.Event(enable_timing=True)
        self.consumed = torch.cuda.Event()
        self.used = False
        self.reserved = False
        self.pieces = None          # [(lo, hi, event after that byte range's H2D)] of a piecewise stage


class _Arena:
    """Pinned host + device bytes for up to ``cap`` packed small updates (see SMALL_UPDATE_BYTES);
    ``uploaded`` of them already sent to HBM (partial uploads every ARENA_UPLOAD_EVERY updates)."""
    __slots__ = ("host", "host_np", "host_ptr", "dev", "dev_ptr", "cap", "count", "uploaded", "done", "used",
                 "host_dev")

    def __init__(self, cap, nbytes, device):
        self.host = torch.empty(cap * nbytes, dtype=torch.uint8, pin_memory=True)
        self.host_np = self.host.numpy()
        self.host_ptr = self.host.data_ptr()
        self.dev = reuse.watch(torch.empty(cap * nbytes, dtype=torch.uint8, device=device))
        self.dev_ptr = self.dev.data_ptr()
        self.cap, self.count, self.uploaded, self.used = cap, 0, 0, False
        self.done = None
        self.host_dev = None          # device address of ``host`` (zero-copy rounds), once asked for


class _ArenaRef:
    """One update's bytes inside an arena: ``ptr`` is the device address the batch's fold reads
    (``dev``, the tensor view, is made only when a path needs one)."""
    __slots__ = ("ptr", "_arena", "_lo", "_hi")

    def __init__(self, arena, lo, hi):
        self.ptr = arena.dev_ptr + lo
        self._arena, self._lo, self._hi = arena, lo, hi

    @property
    def dev(self):
        return self._arena.dev[self._lo:self._hi]


def _addr(src):
    """Device address of a staged update's bytes (an arena piece, a slot or a StagedModel)."""
    return src.ptr if type(src) is _ArenaRef else src.dev.data_ptr()


NO_SNAPSHOT = object()   # _snapshot could not copy the aggregate aside (HBM full)


class _Pipeline:
    def __init__(self, device, layout, nslots, slots=None, streams=None, cache=None, batch=True):
        self.device = torch.device(device)
        self.layout = layout
        self.compute = torch.cuda.current_stream(self.device)
        # a session's earlier round left its staging resources in the aggregator's cache
        self.cache = cache
        kept = cache.take(self.device, layout.nbytes) if cache is not None else None
        if kept is not None:
            slots, streams = kept["slots"], kept["streams"]
        # H2D (update slots, FedOpt's global model) and D2H of the result (full duplex with H2D)
        self.copy, self.d2h = streams if streams is not None else (torch.cuda.Stream(self.device),
                                                                   torch.cuda.Stream(self.device))
        self.nslots = nslots
        # created on first use (staged inputs need none); a caller that folds many models of one
        # layout (helper.Helper.increment_average) hands the same slots to every pipeline
        self.slots = slots if slots is not None else []
        for sl in self.slots:
            sl.reserved = False
        self._next = 0
        self._h2d = []
        self._kern = []
        self.time_pack = 0.0
        self.time_d2h = 0.0
        self._hold = []
        self.pending = []                        # device-resident updates not folded yet: (staged, n, N)
        # small host updates are batched through arenas; ``batch=False`` on the helper path
        # (helper.Helper.increment_average folds ONE pair per pipeline: an arena there would be
        # allocated for a single update and never reused)
        self.batch_host = batch and layout.nbytes <= SMALL_UPDATE_BYTES
        self._arenas, self._arena, self._arena_i = (kept["arenas"] if kept else []), None, 0
        self._pack_jobs = []                     # copies into the arena being filled (kept referenced)
        self._pack_ticket = None                 # the last of them queued to the native gather thread
        # the fused path's fast admission of host updates: exact (shape, dtype) per tensor (computed
        # once per layout: Layout.of returns one object per signature)
        fast = getattr(layout, "_fast_admission", None)
        if fast is None:
            sig = [(tuple(sh), np.dtype(dt)) for sh, dt in zip(layout.shapes, layout.dtypes)]
            plain = not mixed.per_tensor_dtypes(layout.dtypes) and not any(np.dtype(d).kind == "i"
                                                                            for d in layout.dtypes)
            try:
                for dt in layout.groups:
                    ops.fa_dtype(ops.torch_dtype(dt))
            except (TypeError, KeyError):
                plain = False
            fast = layout._fast_admission = (sig, plain)
        self._sig, self._plain = fast
        # the same test and the pack's queueing in one native call (layout.fast_admission)
        self._admit = fast_admission(layout) if self.batch_host and self._plain else None
        self._d2h_on_compute = False             # a small result was copied back on the compute stream
        self._synced = False                     # the result is on the host: every recorded event fired
        self._kern_wall = 0.0                    # zero-copy rounds: launch-to-sync wall time (no events)
        self._copy_used = False                  # work was enqueued on the copy stream this round
        self._d2h_used = False                   # ... on the d2h stream
        self.streamer = kept["streamer"] if kept else HostStreamer()
        # per-update failure isolation (fedavg.py:75-78, fedopt.py:103-106): updates admitted into a
        # batch whose multi-client launch failed are refolded one at a time; (tag, exception) of each
        # one whose own fold failed, for the aggregator to log, uncount and keep in storage
        self.skipped = []
        self.broken = None                       # a batch lost beyond recovery: result() raises it

    def take_skipped(self):
        """(tag, exception) of the updates skipped since the last call (see ``skipped``)."""
        out, self.skipped = self.skipped, []
        return out

    def unsettled(self):
        """How many of the most recently added updates are admitted but not folded yet (the pending
        batch): their fold may still fail, so the aggregator keeps them in storage until then."""
        return len(self.pending)

    def _check_broken(self):
        if self.broken is not None:
            raise RuntimeError(f"a batched fold failed and could not be recovered: {self.broken}") from self.broken

    def quiesce(self):
        """Wait for the packs still queued to the native gather thread: its copies read the update
        arrays (kept alive only by ``_pack_jobs``) and write the arenas. A round abandoned between a
        put and the batch's upload (an exception out of combine_models, a server step refused) must
        not free either while the thread still copies."""
        if self._pack_ticket is not None:
            wait_pack_jobs(self._pack_ticket)
        self._pack_ticket, self._pack_jobs = None, []

    def release(self):
        """Give the staging resources to the cache for the session's next round (call once the
        round's result is on the host; the pipeline stages nothing afterwards)."""
        self.quiesce()
        if self.cache is not None:
            self.cache.give(self.device, self.layout.nbytes,
                            {"slots": self.slots, "arenas": self._arenas, "streams": (self.copy, self.d2h),
                             "streamer": self.streamer})
            self.cache = None

    # ---- staging ---------------------------------------------------------------------
    def _take_slot(self):
        if not self.slots:
            self.slots = [_Slot(self.layout.nbytes, self.device) for _ in range(self.nslots)]
        for _ in range(len(self.slots)):
            s = self.slots[self._next]
            self._next = (self._next + 1) % len(self.slots)
            if not s.reserved:
                return s
        raise RuntimeError("no free staging slot")

    def stage(self, arrays, wait=True):
        """Pack host ``arrays`` into a pinned slot and start its H2D copy; returns the slot. A large
        update (>= STAGE_PIECES_MIN bytes) is packed and copied piece by piece (``slot.pieces``).
        ``wait``: the compute stream waits for the whole H2D (else the caller orders its folds)."""
        s = self._take_slot()
        if s.used:
            s.h2d_done.synchronize()            # pinned bytes no longer read by the DMA
            self.copy.wait_event(s.consumed)    # device bytes no longer read by a fold
        else:
            # a fresh slot's HBM came from the compute stream's pool: its previous owner's queued work
            # there must run before this stream's H2D overwrites it
            self.copy.wait_stream(self.compute)
        self._copy_used = True
        tic = time.perf_counter()
        nb = self.layout.nbytes
        jobs = None
        if nb >= STAGE_PIECES_MIN and _have_codec():
            host_ptr = s.host.data_ptr()
            spans = [(lo, min(nb, lo + STAGE_PIECE)) for lo in range(0, nb, STAGE_PIECE)]
            jobs = [self.layout.pack_range(arrays, host_ptr, lo, hi) for lo, hi in spans]
            if any(j is None for j in jobs):
                jobs = None
        s.pieces = None
        if jobs is None:
            self.layout.pack(arrays, s.host_np)
            self.time_pack += time.perf_counter() - tic
            with torch.cuda.stream(self.copy):
                s.h2d_start.record(self.copy)
                s.dev.copy_(s.host, non_blocking=True)
                s.h2d_done.record(self.copy)
        else:
            from . import codec
            from .layout import PACK_THREADS
            dev_ptr = s.dev.data_ptr()
            s.h2d_start.record(self.copy)
            s.pieces = []
            for (lo, hi), job in zip(spans, jobs):
                t0 = time.perf_counter()
                codec.gather_raw(job, PACK_THREADS, (host_ptr, s.host.numel()))
                self.time_pack += time.perf_counter() - t0
                ops.copy_ptr_async(dev_ptr + lo, host_ptr + lo, hi - lo, self.copy, self.device)
                ev = torch.cuda.Event()
                ev.record(self.copy)
                s.pieces.append((lo, hi, ev))
            s.h2d_done.record(self.copy)
        self._h2d.append((s.h2d_start, s.h2d_done))
        if wait:
            self.compute.wait_event(s.h2d_done)
        s.used = True
        return s

    def wait_bytes(self, slot, lo, hi):
        """The compute stream waits for the H2D of bytes [lo, hi) of ``slot`` (its pieces that overlap
        the range, or the whole copy)."""
        if slot.pieces is None:
            self.compute.wait_event(slot.h2d_done)
            return
        for plo, phi, ev in slot.pieces:
            if plo < hi and lo < phi:
                self.compute.wait_event(ev)

    def put_small(self, arrays, fast=False):
        """Pack a small host update into the arena being filled (no H2D yet); returns the
        reference the batch's fold reads once ``upload_arena`` has run. ``fast``: admit it through
        the native test first (``self._admit``); None, with nothing changed, if ``arrays`` is not
        exactly this layout."""
        a = self._arena
        if a is not None and a.count >= a.cap:
            # every caller flushes a full arena right after its put; a full one here is a bug, and
            # packing into it would write past its pinned block
            raise RuntimeError(f"staging arena full ({a.count} of {a.cap} updates) before put_small")
        if a is None:
            if not self._arenas:
                # >= 2: FedAvg's first update waits in the arena outside ``pending`` (the callers'
                # full-arena flush follows the NEXT put), so one slot is never enough
                cap = max(2, min(BATCH, ARENA_BYTES // self.layout.nbytes))
                self._arenas = [_Arena(cap, self.layout.nbytes, self.device) for _ in range(2)]
            a = self._arenas[self._arena_i]
            self._arena_i = (self._arena_i + 1) % len(self._arenas)
            if a.used:
                a.done.synchronize()            # its previous H2D has read the pinned bytes
            a.count = a.uploaded = 0
            self._arena = a
        nb, j = self.layout.nbytes, a.count
        tic = time.perf_counter()
        # the copies go to the native gather thread and run while the next updates are loaded;
        # upload_arena waits for them (the source arrays stay referenced until then)
        # the arena's pinned block as allocated (not as counted): the native pack is checked against it
        window = (a.host_ptr, a.host.numel())
        if fast:
            ticket = self._admit(arrays, a.host_ptr + j * nb, window)
            if ticket < 0:
                return None
            keep = arrays
        else:
            ticket, keep = start_pack_into(self.layout, arrays, a.host_ptr + j * nb, window)
        self._pack_jobs.append(keep)
        self._pack_ticket = ticket or self._pack_ticket
        self.time_pack += time.perf_counter() - tic
        a.count += 1
        if a.count - a.uploaded >= ARENA_UPLOAD_EVERY:
            self._upload_part(a)                # this part's H2D runs while later updates load
        return _ArenaRef(a, j * nb, (j + 1) * nb)

    def _upload_part(self, a):
        """The H2D of the arena's updates packed since its last partial upload, on the compute
        stream, once their packs have landed."""
        tic = time.perf_counter()
        wait_pack_jobs(self._pack_ticket)
        self._pack_ticket, self._pack_jobs = None, []
        self.time_pack += time.perf_counter() - tic
        nb = self.layout.nbytes
        lo, n = a.uploaded * nb, (a.count - a.uploaded) * nb
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record(self.compute)
        ops.copy_ptr_async(a.dev_ptr + lo, a.host_ptr + lo, n, self.compute, self.device)
        end.record(self.compute)
        self._h2d.append((start, end))
        a.uploaded = a.count
        a.done = end
        a.used = True

    def fast_host(self, arrays):
        """Whether ``arrays`` is a list of numpy arrays with exactly this round's shapes and dtypes on
        a float-only model batched through the arena: such an update needs none of add()'s other
        checks (per-tensor path, integer n rules)."""
        if not (self.batch_host and self._plain) or len(arrays) != len(self._sig):
            return False
        for a, (sh, dt) in zip(arrays, self._sig):
            if type(a) is not np.ndarray or a.shape != sh or a.dtype != dt:
                return False
        return True

    def arena_full(self):
        return self._arena is not None and self._arena.count >= self._arena.cap

    def upload_arena(self):
        """ONE H2D of every update packed since the last upload, enqueued on the compute stream:
        after the folds that last read these device bytes, before the batch's fold."""
        a = self._arena
        if a is None or a.count == 0:
            return
        if a.count > a.uploaded:                # what the partial uploads have not sent yet
            self._upload_part(a)
        self._arena = None

    def acquire(self, arrays):
        """Device-resident source for ``arrays``: a StagedModel is used in place (the compute
        stream waits for its H2D); host arrays are packed into a ring slot."""
        if isinstance(arrays, StagedModel):
            self.layout.check_layout(arrays.layout)      # raises the numpy-like error
            return self._resident(arrays)
        self.layout.check(arrays)
        return self.stage(arrays)

    def _resident(self, arrays):
        """A StagedModel usable on this device: the compute stream waits for its H2D (one D2D
        copy first if it was staged on another GPU); held until the round ends."""
        if arrays.dev.device != self.device:         # staged on another GPU: one D2D copy
            arrays.ready.synchronize()               # (rare) order the copy after its H2D
            with torch.cuda.device(self.device):
                dev = reuse.watch(arrays.dev.to(self.device))
                ready = torch.cuda.Event()
                ready.record(torch.cuda.current_stream(self.device))
            arrays = StagedModel(arrays.layout, dev, ready, None)
        self.compute.wait_event(arrays.ready)
        self._hold.append(arrays)                    # keep HBM alive until the round ends
        return arrays

    # ---- per-tensor path (mixed.py): updates that differ from the first in dtype or shape ----
    def compatible(self, arrays):
        """Whether ``arrays`` has exactly this round's layout (the fused multi-client path)."""
        if isinstance(arrays, StagedModel):
            return arrays.layout.signature() == self.layout.signature()
        if len(arrays) != len(self.layout.shapes):
            return False
        for i, a in enumerate(arrays):
            a = np.asarray(a)
            if tuple(a.shape) != self.layout.shapes[i] or a.dtype != self.layout.dtypes[i]:
                return False
        return True

    def tensors_of(self, arrays):
        """Per-tensor device tensors of an update for the per-tensor path: views of a staged
        update (the compute stream ordered after its H2D), or host arrays copied per tensor."""
        if isinstance(arrays, StagedModel):
            arrays = self._resident(arrays)
            return mixed.tensor_views(arrays.layout, mixed.u8_flats(arrays.layout, arrays.dev))
        return mixed.upload(arrays, self.device, self.compute)

    @staticmethod
    def meta_of(arrays):
        if isinstance(arrays, StagedModel):
            return list(zip(arrays.layout.shapes, arrays.layout.dtypes))
        return mixed.host_meta(arrays)

    def group(self, slot, dt):
        """Device view (flat, torch dtype) of group ``dt`` inside a staged slot."""
        off = self.layout.group_byte_offset[dt]
        n = self.layout.group_elems[dt]
        return slot.dev[off:off + n * dt.itemsize].view(ops.torch_dtype(dt))

    def _kernel_span(self):
        a = torch.cuda.Event(enable_timing=True)
        a.record(self.compute)
        return a

    def _end_span(self, a):
        b = torch.cuda.Event(enable_timing=True)
        b.record(self.compute)
        self._kern.append((a, b))

    def _fold_then_d2h(self, src, fold_chunk, prepare=None, ready=None):
        """Copy device tensor ``src`` into a new pinned host tensor chunk by chunk: for each
        chunk [lo, hi), ``prepare(lo, hi)`` (optional: enqueue the chunk's inputs) and
        ``fold_chunk(lo, hi)`` (enqueue the launch that produces ``src[lo:hi]`` on the compute
        stream), then its D2H on the d2h stream, which overlaps the next chunk's work.
        ``ready(lo, hi)`` (optional): the events the chunk's D2H waits for instead of everything
        enqueued on the compute stream so far. The caller synchronises the d2h stream."""
        n = src.numel()
        host = torch.empty(n, dtype=src.dtype, pin_memory=True)
        if n * src.element_size() <= SMALL_UPDATE_BYTES:
            # one chunk: launch and D2H in order on the compute stream (no cross-stream hand-off);
            # the caller synchronises the compute stream too
            if prepare is not None:
                prepare(0, n)
            fold_chunk(0, n)
            ops.copy_ptr_async(host.data_ptr(), src.data_ptr(), n * src.element_size(), self.compute, self.device)
            self._d2h_on_compute = True
            return host
        self._d2h_used = True
        for lo, hi in chunks(n, src.element_size()):
            if prepare is not None:
                prepare(lo, hi)
            fold_chunk(lo, hi)
            if ready is not None:
                for ev in ready(lo, hi):
                    self.d2h.wait_event(ev)
            else:
                ev = torch.cuda.Event()
                ev.record(self.compute)
                self.d2h.wait_event(ev)
            with torch.cuda.stream(self.d2h):
                host[lo:hi].copy_(src[lo:hi], non_blocking=True)
        return host

    def _to_host(self, t):
        """D2H at the PCIe rate into a NEW pinned host tensor, which becomes the caller's
        model: it is never a staging slot, and when the caller drops the model the block goes
        back to torch's pinned-host cache, so later rounds reuse already-mapped pages instead
        of page-faulting a fresh pageable array (which cost more than the DMA itself)."""
        tic = time.perf_counter()
        pinned = torch.empty(t.numel(), dtype=t.dtype, pin_memory=True)
        pinned.copy_(t, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        self.time_d2h += time.perf_counter() - tic
        return pinned

    def timings(self):
        """GPU-side H2D and kernel time (s, HIP events) plus host pack and D2H wall time."""
        if not self._synced:                     # result() synchronised every stream its events are on
            torch.cuda.synchronize(self.device)
        h2d = sum(a.elapsed_time(b) for a, b in self._h2d) / 1e3
        kern = sum(a.elapsed_time(b) for a, b in self._kern) / 1e3 + self._kern_wall
        return {"time_h2d": h2d, "time_kernel": kern, "time_pack": self.time_pack, "time_d2h": self.time_d2h}


class FedAvgPipeline(_Pipeline):
    """Streaming FedAvg on one device: fedavg.py:47-71 with the fold on the GPU."""

    def __init__(self, device, first_arrays, nslots=3, slots=None, streams=None, cache=None, batch=True):
        staged = isinstance(first_arrays, StagedModel)
        super().__init__(device, first_arrays.layout if staged else Layout.of(first_arrays), nslots, slots, streams,
                         cache, batch)
        self.first_arrays = first_arrays         # a StagedModel materialises host arrays only if needed
        if staged:
            self.first = self.acquire(first_arrays)
        elif self.batch_host:
            # a small model: the first update rides in the arena with the round's other updates
            # (one H2D, everything on the compute stream)
            self.first = self.put_small(first_arrays, fast=True) if (
                self._admit is not None and type(first_arrays) is list) else None
            if self.first is None:
                self.layout.check(first_arrays)
                self.first = self.put_small(first_arrays)
        else:
            self.first = self.stage(first_arrays)
            self.first.reserved = True
        self.nfolds = 0
        self.agg_started = False                 # agg holds a fold of the first update
        self.agg = {}
        self.general = None                      # mixed.TensorFedAvg once an update differs in layout
        # the fold chunks of the latest large host update, (dt, lo, hi, event after the chunk) — valid
        # while nothing was folded after it: result() then D2H's each chunk of the model as soon as
        # that chunk is folded, overlapping the rest of the last update's H2D (PCIe is full duplex)
        self._last_fold = None

    def _state_meta(self):
        """(shape, dtype) per tensor of the running model: the first update's before any fold,
        numpy's fold result dtype after."""
        lay = self.layout
        if self.nfolds == 0:
            return list(zip(lay.shapes, lay.dtypes))
        return [(s, mixed.np_dtype(ops.fold_result_dtype(ops.torch_dtype(d), ops.torch_dtype(d))))
                for s, d in zip(lay.shapes, lay.dtypes)]

    def _enter_general(self):
        """Hand the running model to the per-tensor path (mixed.TensorFedAvg)."""
        self._flush()
        self._last_fold = None
        if self.agg_started:
            views = mixed.tensor_views(self.layout, {dt: self._agg(dt) for dt in self.layout.groups})
            self.general = mixed.TensorFedAvg(self.device, self.compute, views, owned=True)
        else:
            src = self.first.dev
            views = mixed.tensor_views(self.layout, mixed.u8_flats(self.layout, src))
            self.general = mixed.TensorFedAvg(self.device, self.compute, views, owned=False)

    def add(self, arrays, n, N, tag=None):
        """Fold one more update (n = its num_examples, N = running total including it).
        A device-resident update (StagedModel) joins the pending batch; host arrays are
        staged and folded on arrival (after any pending batch, keeping FIFO order). An update
        whose dtypes or shapes differ from the first's moves the round to the per-tensor path
        (numpy promotion / broadcasting, mixed.py) — checked before any state changes.
        ``tag``: reported back with the update if its batched fold fails later (``skipped``)."""
        self._check_broken()
        if self._admit is not None and self.general is None and type(arrays) is list:
            ref = self.put_small(arrays, fast=True)                 # a small float model's update
            if ref is not None:
                self.pending.append((ref, n, N, tag))
                if len(self.pending) >= BATCH or self.arena_full():
                    self._flush()
                self.nfolds += 1
                return
        elif self.general is None and type(arrays) is list and self.fast_host(arrays):
            self.pending.append((self.put_small(arrays), n, N, tag))      # a small float model's update
            if len(self.pending) >= BATCH or self.arena_full():
                self._flush()
            self.nfolds += 1
            return
        elif self.general is None and self._plain and type(arrays) is StagedModel and arrays.layout is self.layout:
            # staged on arrival in this very layout (the ingest's round end): nothing else to check
            self.pending.append((self._resident(arrays), n, N, tag))
            if len(self.pending) >= BATCH:
                self._flush()
            self.nfolds += 1
            return
        if self.general is None and (not self.compatible(arrays) or
                                     mixed.int_float_n(self.layout.dtypes, self.nfolds, n) or
                                     mixed.per_tensor_dtypes(self.layout.dtypes)):
            plan = mixed.fold_plan(self._state_meta(), self.meta_of(arrays), n, N)   # raises as numpy
            self._enter_general()
            self.general.fold(self.tensors_of(arrays), n, N, plan=plan)
            self.nfolds += 1
            return
        if self.general is not None:
            self.general.fold(self.tensors_of(arrays), n, N)
            self.nfolds += 1
            return
        if isinstance(arrays, StagedModel):
            self.layout.check_layout(arrays.layout)
        else:
            self.layout.check(arrays)
        for dt in self.layout.groups:           # refuse before touching device state
            ops.fa_dtype(ops.torch_dtype(dt))
        if isinstance(arrays, StagedModel):
            self.pending.append((self.acquire(arrays), n, N, tag))
            if len(self.pending) >= BATCH:
                self._flush()
        elif self.batch_host:
            self.pending.append((self.put_small(arrays), n, N, tag))
            if len(self.pending) >= BATCH or self.arena_full():
                self._flush()
        else:
            self._flush()
            slot = self.stage(arrays, wait=False)
            try:
                self._fold_pieces(slot, n, N)
            finally:
                slot.consumed.record(self.compute)   # the slot's next H2D waits for what was enqueued
        self.nfolds += 1

    # ---- per-update failure isolation (fedavg.py:75-78) ---------------------------------------
    def _snapshot(self, launches):
        """The running aggregate copied aside before a continuation fold of more than one launch:
        one that fails part-way leaves it half-advanced, and the recovery needs it back. None when
        not needed: not started (an init fold rewrites it) or one launch (a failed launch ran nothing)."""
        if not self.agg_started or launches <= 1:
            return None
        try:                                    # a model-sized clone for the fold's duration (the HBM
            with torch.cuda.device(self.device), torch.cuda.stream(self.compute):   # budget's headroom)
                return {dt: self._agg(dt).clone() for dt in self.layout.groups}
        except torch.cuda.OutOfMemoryError:
            return NO_SNAPSHOT                  # the fold goes ahead; only a failure part-way is fatal

    def _restore(self, snap, ran=1):
        """Put the aggregate back after a failed multi-launch fold of which ``ran`` launches had been
        enqueued (0: the aggregate is untouched, nothing to put back)."""
        if ran == 0:
            return
        if snap is NO_SNAPSHOT:
            # a launch failed after earlier ones advanced the aggregate, and HBM held no copy of it:
            # the round cannot go on with this update skipped — result() raises
            self.broken = RuntimeError("a multi-launch fold failed part-way and the aggregate could not be "
                                       "copied aside beforehand (HBM full): the round is lost")
            raise self.broken
        if snap is not None:
            with torch.cuda.device(self.device), torch.cuda.stream(self.compute):
                for dt, t in snap.items():
                    self._agg(dt).copy_(t)

    def _refold_singly(self, entries):
        """A multi-client launch over ``entries`` failed: fold them one at a time in FIFO order as
        FEDn does (fedavg.py:47-78). An update whose own fold fails is skipped and reported with its
        tag; its examples stay counted (its N is already in every later entry's running total), and
        the aggregate is as the previous update left it (each update's launches are all-or-nothing)."""
        for e in entries:
            snap, ran = None, 0
            try:
                snap = self._snapshot(len(self.layout.groups))
                for dt in self.layout.groups:
                    self._fold_group(dt, [e], not self.agg_started, 0, self.layout.group_elems[dt])
                    ran += 1
            except ops.FedAggError as ex:
                self._restore(snap, ran)
                self.skipped.append((e[3] if len(e) > 3 else None, ex))
                continue
            self._folded()

    def _fold_pieces(self, slot, n, N):
        """Fold one staged host update on arrival, one launch per H2D piece of each group, each
        waiting only for its piece (the fold of piece j overlaps the DMA of piece j + 1); the chunks'
        events are kept for result() (``_last_fold``). Same kernel, table and element ranges of one
        recurrence step: the same bits as one launch."""
        span = self._kernel_span()
        init = not self.agg_started
        plan = []
        for dt in self.layout.groups:
            off, isz, P = self.layout.group_byte_offset[dt], np.dtype(dt).itemsize, self.layout.group_elems[dt]
            if slot.pieces is None:
                bounds = [(0, P)] if P else []
            else:                               # element ranges of the group inside each piece
                bounds = [(max(0, (plo - off) // isz), min(P, (phi - off) // isz)) for plo, phi, _ in slot.pieces]
                bounds = [(lo, hi) for lo, hi in bounds if hi > lo]
                if bounds:
                    bounds[-1] = (bounds[-1][0], P)
            plan += [(dt, off, isz, lo, hi) for lo, hi in bounds]
        done = []
        snap = None
        try:
            snap = self._snapshot(len(plan))    # this update's launches are all-or-nothing
            for dt, off, isz, lo, hi in plan:
                self.wait_bytes(slot, off + lo * isz, off + hi * isz)
                self._fold_group(dt, [(slot, n, N)], init, lo, hi)
                ev = torch.cuda.Event()
                ev.record(self.compute)
                done.append((dt, lo, hi, ev))
        except ops.FedAggError:
            self._last_fold = None
            self._restore(snap, len(done))      # the update is skipped by the caller (fedavg.py:75-78)
            raise
        self._end_span(span)
        self._folded()
        self._last_fold = done

    def _fold_group(self, dt, entries, init, lo, hi):
        """Enqueue the fold of ``entries`` over elements [lo, hi) of group ``dt``. Every entry's
        bytes (a slot, an arena piece or a staged model) are a uint8 buffer on this device in this
        layout, so the client table is plain addresses (no per-update tensor views: for small models
        those cost more than the launch)."""
        off = self.layout.group_byte_offset[dt] + lo * dt.itemsize
        ptrs = [_addr(e[0]) + off for e in entries]
        ns = [e[1] for e in entries]
        Ns = [e[2] for e in entries]
        acc = self._agg(dt)[lo:hi]
        upd_dt = ops.torch_dtype(dt)
        if init:                                # agg := first update, then fold (fedavg.py:65-71)
            ops.fedavg_fold_ptrs(acc, [_addr(self.first) + off] + ptrs, upd_dt, [0.0] + ns, [1.0] + Ns,
                                 init=True, stream=self.compute)
        else:
            ops.fedavg_fold_ptrs(acc, ptrs, upd_dt, ns, Ns, init=False, stream=self.compute)

    def _agg(self, dt):
        """The running aggregate of group ``dt`` (allocated on first use, numpy's result dtype)."""
        if dt not in self.agg:
            t = ops.torch_dtype(dt)
            self.agg[dt] = torch.empty(self.layout.group_elems[dt], dtype=ops.fold_result_dtype(t, t),
                                       device=self.device)
        return self.agg[dt]

    def _folded(self):
        if not self.agg_started and isinstance(self.first, _Slot):
            self.first.consumed.record(self.compute)
            self.first.reserved = False
        self.agg_started = True

    def _fold_all(self, entries):
        self._last_fold = None
        span = self._kernel_span()
        init = not self.agg_started
        snap, ran = None, 0
        try:
            snap = self._snapshot(len(self.layout.groups))
            for dt in self.layout.groups:
                self._fold_group(dt, entries, init, 0, self.layout.group_elems[dt])
                ran += 1
        except ops.FedAggError:
            self._restore(snap, ran)
            self._refold_singly(entries)
            self._end_span(span)
            return
        self._end_span(span)
        self._folded()

    def _flush(self):
        self.upload_arena()                     # also the first update, when it waits in the arena
        if self.pending:
            entries, self.pending = self.pending, []
            try:
                self._fold_all(entries)
            except BaseException as e:          # the batch is lost: never return a model without it
                self.broken = e
                raise

    def result(self):
        """The aggregated model as a new host ``list[np.ndarray]`` (fedavg.py:83). A pending
        batch is folded here, chunk by chunk, each chunk's D2H overlapping the next fold."""
        self._check_broken()
        if self.nfolds == 0:
            return self._alias()
        if self.general is not None:
            return self.general.result()
        tic = time.perf_counter()
        out = self._zero_copy_result()
        if out is not None:
            self.time_d2h += time.perf_counter() - tic
            return out
        self.upload_arena()
        entries, self.pending = self.pending, []
        if not entries and not self.agg_started:
            return self._alias()                # every fold after the first update was skipped
        last = self._last_fold if not entries else None
        init = not self.agg_started
        span = self._kernel_span()
        hosts = {}
        # the last batch runs chunk by chunk (or per group): a failed chunk needs the aggregate back
        snap, ran = None, [0]
        try:
            snap = self._snapshot(2 if (len(self.layout.groups) > 1 or self.layout.nbytes > SMALL_UPDATE_BYTES) else 1) \
                if entries else None

            def fold_counted(dt, lo, hi):
                self._fold_group(dt, entries, init, lo, hi)
                ran[0] += 1
            for dt in self.layout.groups:
                ready = None
                if entries:
                    fold = lambda lo, hi, dt=dt: fold_counted(dt, lo, hi)  # noqa: E731
                else:
                    fold = lambda lo, hi: None  # noqa: E731
                    if last is not None:            # each D2H chunk waits only for the folds it reads
                        mine = [(lo, hi, ev) for d, lo, hi, ev in last if d == dt]
                        ready = lambda lo, hi, mine=mine: [ev for flo, fhi, ev in mine if flo < hi and lo < fhi]  # noqa: E731
                hosts[dt] = self._fold_then_d2h(self._agg(dt), fold, ready=ready)
        except ops.FedAggError:
            if not entries:
                raise
            self.compute.synchronize()          # what the failed attempt enqueued has run
            self.d2h.synchronize()
            self._restore(snap, ran[0])
            self._refold_singly(entries)
            entries = []
            if not self.agg_started:
                self.compute.synchronize()
                return self._alias()
            hosts = {dt: self._fold_then_d2h(self._agg(dt), lambda lo, hi: None) for dt in self.layout.groups}
        self._end_span(span)
        if entries:
            self._folded()
        if self._d2h_on_compute:
            self.compute.synchronize()          # a small group came back on the compute stream
        if self._d2h_used or not self._d2h_on_compute:
            self.d2h.synchronize()
        self._synced = self._d2h_on_compute and not self._d2h_used and not self._copy_used
        self.time_d2h += time.perf_counter() - tic
        out = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            self.layout.unpack_group(hosts[dt].numpy(), dt, out, copy=False)
        return out

    def _alias(self):
        """The first update itself: the model when nothing was folded into it (fedavg.py:65-66)."""
        first = self.first_arrays
        return first.host if isinstance(first, StagedModel) else first

    def _zero_copy_result(self):
        """A small round that never left the host: the first update and every pending one wait in the
        arena being filled, none uploaded yet, at most ZERO_COPY_BYTES in all. ONE launch per dtype
        group folds them reading the pinned arena and writing the new pinned result block through
        their device addresses (fa_host_device_ptr) — the same kernel and client table as the
        device path, so the same bits — and one synchronize ends the round. None if not such a round."""
        a = self._arena
        if (self.agg_started or a is None or a.uploaded or not self.pending or type(self.first) is not _ArenaRef
                or self.first._arena is not a or a.count * self.layout.nbytes > ZERO_COPY_BYTES):
            return None
        entries = self.pending
        if any(type(e[0]) is not _ArenaRef or e[0]._arena is not a for e in entries):
            return None
        try:
            if a.host_dev is None:
                a.host_dev = ops.host_device_ptr(a.host_ptr, self.device)
        except Exception:  # noqa: BLE001 — no device mapping of the arena: the copy path
            return None
        wait_pack_jobs(self._pack_ticket)
        self._pack_ticket, self._pack_jobs = None, []
        self.pending, self._arena = [], None
        ns, Ns = [0.0] + [e[1] for e in entries], [1.0] + [e[2] for e in entries]
        t0 = time.perf_counter()                # no event pair: the launch is synchronised right after
        hosts = {}
        try:
            for dt in self.layout.groups:
                t = ops.torch_dtype(dt)
                rdt = ops.fold_result_dtype(t, t)
                n = self.layout.group_elems[dt]
                host = torch.empty(n, dtype=rdt, pin_memory=True)
                hosts[dt] = host
                if n == 0:                          # a group of empty tensors: nothing to fold or map
                    continue
                off = self.layout.group_byte_offset[dt]
                ptrs = [a.host_dev + self.first._lo + off] + [a.host_dev + e[0]._lo + off for e in entries]
                ops.fedavg_fold_raw(ops.host_device_ptr(host.data_ptr(), self.device), rdt, n, ptrs, t, ns, Ns, True,
                                    self.compute, self.device)
        except ops.FedAggError:
            # the batch goes the device way instead (upload, batched launch, one-at-a-time on failure)
            self.compute.synchronize()
            self.pending, self._arena = entries, a
            return None
        self.agg_started = True
        self.compute.synchronize()              # the arena's pinned bytes are read until here: free again
        a.done, a.used = None, False
        self._kern_wall += time.perf_counter() - t0
        self._d2h_on_compute = True
        self._synced = not self._d2h_used and not self._copy_used
        out = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            self.layout.unpack_group(hosts[dt].numpy(), dt, out, copy=False)
        return out


class UnsupportedHelper(TypeError):
    """A helper plug-in whose arithmetic the aggregators do not implement."""


KNOWN_HELPERS = ("numpyhelper", "binaryhelper", "androidhelper", "fednamdhelper")


def helper_kind(helper, strict=True):
    """Which FEDn helper plug-in a round uses. package.py:24 accepts numpyhelper, binaryhelper
    and androidhelper (plus this package's fednamdhelper); the aggregators fold with the helper's
    own arithmetic (fedavg.py:68), so each is recognised by its plug-in module (androidhelper sets
    ``name`` and HelperBase resets it to the class name). None (tests, tools) means numpyhelper.
    Any other helper: UnsupportedHelper (raised inside combine_models' per-update try, so every
    update is logged and skipped and the round returns (None, data) — its arithmetic is never
    guessed), or "unknown" with ``strict=False`` (the ingest then leaves its updates host-side)."""
    if helper is None:
        return "numpyhelper"
    mod = type(helper).__module__.rsplit(".", 1)[-1]
    if mod in ("numpyhelper", "binaryhelper", "androidhelper"):
        return mod
    from .helper import Helper as OwnHelper
    if isinstance(helper, OwnHelper) or mod == "fednamdhelper":
        return "fednamdhelper"
    if not strict:
        return "unknown"
    raise UnsupportedHelper(f"helper {type(helper).__module__}.{type(helper).__name__} is not supported by the "
                            f"fedn_amd aggregators (they implement {', '.join(KNOWN_HELPERS)}); its "
                            f"increment_average is not assumed to be numpyhelper's")


class AndroidFedAvgPipeline(_Pipeline):
    """FedAvg in a session on FEDn's androidhelper, whose increment_average is
    ``(1 - w) * model + w * model_next`` with ``w = num_examples / total_examples`` on ONE flat
    array (androidhelper.py:21-39; its load gives float64, :78-92) — not numpyhelper's
    ``x + n*(y - x)/N``. Device form: one ``fa_running_mean`` launch per update,
    ``g = (g*a + m*b) / T`` with a = 1 - w, b = w, T = 1 (the division by 1 is exact), which
    rounds exactly as numpy: RN(RN(g*a) + RN(m*b)). Mobile models are small; updates are
    staged and folded on arrival."""

    def __init__(self, device, first_arrays):
        first = np.asarray(first_arrays)
        super().__init__(device, Layout.of([first]), 2)
        self.first_arrays = first_arrays
        self.nfolds = 0
        self.g = None

    def add(self, arrays, n, N, tag=None):
        arr = np.asarray(arrays)
        self.layout.check([arr])                # numpy would refuse other lengths too
        dt = self.layout.groups[0]
        if ops.torch_dtype(dt) not in (torch.float32, torch.float64):
            raise TypeError(f"androidhelper models are float arrays, got {dt}")
        w = n / N
        if self.g is None:
            s0 = self.stage([np.asarray(self.first_arrays)])
            with torch.cuda.stream(self.compute):
                self.g = self.group(s0, dt).clone()
            s0.consumed.record(self.compute)
        s = self.stage([arr])
        span = self._kernel_span()
        ops.running_mean(self.g, self.group(s, dt), 1 - w, w, 1.0, stream=self.compute)
        self._end_span(span)
        s.consumed.record(self.compute)
        self.nfolds += 1

    def result(self):
        if self.nfolds == 0:
            return self.first_arrays            # `model = model_next` alias (fedavg.py:65-66)
        return self._to_host(self.g).numpy()


class FedOptState:
    """Server-optimizer state of one fedopt Aggregator instance (fedopt.py:36-38), in HBM.

    Fused form: ``m`` / ``v`` map a layout group to a flat device tensor (m: f16, f32 or f64,
    v: f64) for ``layout``. Per-tensor form (after a round on the per-tensor path, mixed.py):
    ``m_t`` / ``v_t`` are lists of device tensors in model order. Both None until the first
    server step, exactly like the reference's ``self.m``/``self.v``.
    """

    def __init__(self, fp32=False):
        self.m = None
        self.v = None
        self.signature = None
        self.layout = None
        self.m_t = None
        self.v_t = None
        # fp32-state mode (aggregators.fedopt_f32state): groups whose global model is float32 keep
        # m, v and the new model in float32 (fa_fedopt_step_ex, state_dtype F32)
        self.fp32 = fp32

    def reset(self):
        self.__init__(self.fp32)

    def tensors(self):
        """(m, v) as per-tensor device tensors in model order, or (None, None)."""
        if self.m_t is not None:
            return self.m_t, self.v_t
        if self.m is None:
            return None, None
        return mixed.tensor_views(self.layout, self.m), mixed.tensor_views(self.layout, self.v)

    def set_tensors(self, m_t, v_t):
        self.m = self.v = self.signature = self.layout = None
        self.m_t, self.v_t = m_t, v_t

    def regroup(self, layout, sig, device):
        """Make the fused form match ``layout``: True if it does (or the state is empty), False
        if the per-tensor state cannot be grouped that way (shapes differ, or one group would
        need two m dtypes) — then the round's server step runs per tensor."""
        if self.m is None and self.m_t is None:
            return True
        if self.m is not None and self.signature == sig:
            return True
        m_t, v_t = self.tensors()
        grouped = group_tensors(layout, m_t, v_t, device)
        if grouped is None:
            return False
        self.m, self.v = grouped
        self.signature, self.layout = sig, layout
        self.m_t = self.v_t = None
        return True

    def _host(self, ts):
        if ts is None:
            return None
        return [t.to("cpu").numpy() for t in ts]

    def m_host(self):
        """``m`` as host ``list[np.ndarray]`` in tensor order (what fedopt.py keeps in self.m)."""
        return self._host(self.tensors()[0])

    def v_host(self):
        return self._host(self.tensors()[1])


def group_tensors(layout, m_t, v_t, device):
    """Per-tensor (m, v) -> fused ({group: flat m}, {group: flat v}) on ``device`` for ``layout``,
    or None when not expressible (tensor count or shapes differ; mixed m dtypes in a group)."""
    if len(m_t) != len(layout.shapes) or len(v_t) != len(layout.shapes):
        return None
    m, v = {}, {}
    for dt in layout.groups:
        idx = [i for i, _ in layout.members[dt]]
        mdts = {m_t[i].dtype for i in idx}
        if len(mdts) != 1 or any(tuple(m_t[i].shape) != layout.shapes[i] or tuple(v_t[i].shape) != layout.shapes[i]
                                 for i in idx):
            return None
        fm = torch.empty(layout.group_elems[dt], dtype=mdts.pop(), device=device)
        fv = torch.empty(layout.group_elems[dt], dtype=torch.float64, device=device)
        for i, off in layout.members[dt]:
            fm[off:off + layout.sizes[i]].copy_(m_t[i].reshape(-1))
            fv[off:off + layout.sizes[i]].copy_(v_t[i].reshape(-1))
        m[dt], v[dt] = fm, fv
    return m, v


def old_groups(layout, old_arrays):
    """The global model (fedopt.py:89-94) as one contiguous host array per update dtype group."""
    if len(old_arrays) != len(layout.shapes):
        raise ValueError("global model and update have different tensor counts")
    out = {}
    for dt in layout.groups:
        parts = []
        for i, _ in layout.members[dt]:
            o = np.asarray(old_arrays[i])
            if tuple(o.shape) != layout.shapes[i]:
                raise ValueError(f"operands could not be combined: tensor {i} has shape {o.shape}, "
                                 f"global model has {layout.shapes[i]}")
            parts.append(o)
        odt = {p.dtype for p in parts}
        if len(odt) != 1:
            raise TypeError("global-model tensors of one update dtype group must share a dtype")
        flat = np.concatenate([p.reshape(-1) for p in parts]) if parts else np.empty(0, list(odt)[0])
        out[dt] = np.ascontiguousarray(flat)
    return out


def old_members(layout, old_arrays):
    """The global model (fedopt.py:89-94) per update dtype group, WITHOUT concatenating it:
    {group: (dtype, [(flat member array, element offset in the group)])}. Same checks and
    messages as old_groups."""
    if len(old_arrays) != len(layout.shapes):
        raise ValueError("global model and update have different tensor counts")
    out = {}
    for dt in layout.groups:
        parts = []
        for i, off in layout.members[dt]:
            o = np.asarray(old_arrays[i])
            if tuple(o.shape) != layout.shapes[i]:
                raise ValueError(f"operands could not be combined: tensor {i} has shape {o.shape}, "
                                 f"global model has {layout.shapes[i]}")
            parts.append((np.ascontiguousarray(o).reshape(-1), off))
        odt = {p.dtype for p, _ in parts}
        if len(odt) != 1:
            raise TypeError("global-model tensors of one update dtype group must share a dtype")
        out[dt] = (list(odt)[0], parts)
    return out


_FUSED_OPT = {(torch.float32, torch.float32), (torch.bfloat16, torch.float32), (torch.float32, torch.float64),
              (torch.float64, torch.float64), (torch.bfloat16, torch.float64), (torch.float64, torch.float32),
              (torch.int64, torch.int64), (torch.int64, torch.float64), (torch.int64, torch.float32),
              (torch.int32, torch.int32), (torch.int32, torch.float64), (torch.int32, torch.float32),
              # float16 sessions: a half global model's pseudo-gradient is half (numpy's half loops)
              (torch.float16, torch.float16), (torch.float16, torch.float32), (torch.float16, torch.float64),
              (torch.float32, torch.float16), (torch.float64, torch.float16)}


def fused_fedopt_pair(upd, old):
    """Whether fa_fedopt_step instantiates (update dtype, global-model dtype)."""
    return (upd, old) in _FUSED_OPT


def check_fedopt_dtypes(layout):
    for dt in layout.groups:
        if ops.torch_dtype(dt) not in (torch.float16, torch.float32, torch.float64, torch.int32, torch.int64):
            raise TypeError(f"FedOpt supports float16/float32/float64/int32/int64 updates, got {dt}")


def state_dtypes(state, upd_dt, old_dt, m_in):
    """(m dtype, v / new-model dtype) of one group's server step: numpy's flow (m promoted, v and the
    model float64, fedopt.py:151-258), or in the fp32-state mode, for a float32 global model, float32
    for all three (fa_fedopt_step_ex)."""
    _, m_dt = ops.fedopt_dtypes(ops.torch_dtype(upd_dt), old_dt, None if m_in is None else m_in.dtype)
    if getattr(state, "fp32", False) and old_dt == torch.float32:
        return torch.float32, torch.float32
    return m_dt, torch.float64


class FedOptPipeline(_Pipeline):
    """Streaming FedOpt on one device: the pseudo-gradient loop of fedopt.py:74-106 on the
    GPU (pg resident in HBM), then the fused server step (fedopt.py:151-258)."""

    def __init__(self, device, old_arrays, first_arrays, nslots=2, cache=None):
        layout = first_arrays.layout if isinstance(first_arrays, StagedModel) else Layout.of(first_arrays)
        super().__init__(device, layout, nslots, cache=cache)
        self.old_arrays = old_arrays
        self.nfolds = 0
        self.pg = {}
        self.pg_started = False                  # pg holds a partial pseudo-gradient
        self.general = None                      # mixed.TensorFedOpt once an update differs in layout
        self.old_ready = set()
        # the fused path needs the global model to share the update's shapes with one dtype per
        # update-dtype group, and a (update, old) dtype pair the kernel instantiates; otherwise
        # the round runs on the per-tensor path (numpy promotion / broadcasting, mixed.py)
        self.fused_ok = True
        try:
            self.old_host = old_members(layout, old_arrays)
            check_fedopt_dtypes(layout)
            for dt, (odt, _) in self.old_host.items():
                if not fused_fedopt_pair(ops.torch_dtype(dt), ops.torch_dtype(odt)):
                    raise TypeError(f"no fused kernel for {dt} updates over a {odt} global model")
        except (ValueError, TypeError):
            self.fused_ok = False
            self.old_host = {}
        # the global model reaches HBM lazily: whole (when a host update must fold into pg) or
        # chunk by chunk inside the server step's pipeline (H2D || step || D2H)
        self.old = {dt: torch.empty(layout.group_elems[dt], dtype=ops.torch_dtype(odt), device=self.device)
                    for dt, (odt, _) in self.old_host.items()}
        if self.old:
            self.copy.wait_stream(self.compute)  # their HBM's previous owners' queued work first (stage())

    def _pg_meta(self):
        """(shape, dtype) per tensor of the pseudo-gradient folded so far (fused layout)."""
        return [(s, mixed.np_dtype(ops.fedopt_dtypes(ops.torch_dtype(d), self.old[d].dtype, None)[0]))
                for s, d in zip(self.layout.shapes, self.layout.dtypes)]

    def _enter_general(self):
        """Hand the round to the per-tensor path (mixed.TensorFedOpt): pending updates are folded
        into pg first, which then continues per tensor."""
        self._flush()
        pg = None
        if self.pg_started:
            pg = mixed.tensor_views(self.layout, {dt: self._pg(dt) for dt in self.layout.groups})
        old = mixed.upload(self.old_arrays, self.device, self.compute)
        self.general = mixed.TensorFedOpt(self.device, self.compute, old, pg)

    def add(self, arrays, n, N, tag=None):
        """One more update into the pseudo-gradient (fedopt.py:89-94). Device-resident updates
        join the pending batch, which the server step folds in its fused launch; host arrays
        are staged and folded into pg on arrival (after any pending batch). Updates that differ
        from the first in dtype or shape, or from the global model in shape, run per tensor.
        ``tag``: reported back with the update if its batched fold fails later (``skipped``)."""
        self._check_broken()
        if self._admit is not None and self.general is None and self.fused_ok and type(arrays) is list:
            ref = self.put_small(arrays, fast=True)                 # a small float model's update
            if ref is not None:
                self.pending.append((ref, n, N, tag))
                if len(self.pending) >= BATCH or self.arena_full():
                    self._flush()
                self.nfolds += 1
                return
        elif self.general is None and self.fused_ok and type(arrays) is list and self.fast_host(arrays):
            self.pending.append((self.put_small(arrays), n, N, tag))      # a small float model's update
            if len(self.pending) >= BATCH or self.arena_full():
                self._flush()
            self.nfolds += 1
            return
        elif self.general is None and self.fused_ok and type(arrays) is StagedModel and arrays.layout is self.layout:
            # staged on arrival in this very layout (the ingest's round end): nothing else to check
            self.pending.append((self._resident(arrays), n, N, tag))
            if len(self.pending) >= BATCH:
                self._flush()
            self.nfolds += 1
            return
        if self.general is None and not (self.fused_ok and self.compatible(arrays)):
            ym = self.meta_of(arrays)
            splan = mixed.sub_plan(ym, mixed.host_meta(self.old_arrays))          # raises as numpy
            if self.nfolds:
                mixed.fold_plan(self._pg_meta(), [(sh, d) for d, sh in splan], n, N)
            self._enter_general()
        if self.general is not None:
            self.general.add(self.tensors_of(arrays), n, N)
            self.nfolds += 1
            return
        if isinstance(arrays, StagedModel):
            self.pending.append((self.acquire(arrays), n, N, tag))
            if len(self.pending) >= BATCH:
                self._flush()
        elif self.batch_host:
            self.layout.check(arrays)
            self.pending.append((self.put_small(arrays), n, N, tag))
            if len(self.pending) >= BATCH or self.arena_full():
                self._flush()
        else:
            self._flush()
            slot = self.acquire(arrays)
            try:
                self._fold_pg([(slot, n, N)])   # fails as a whole: the caller skips the update
            finally:
                slot.consumed.record(self.compute)
        self.nfolds += 1

    def _pg(self, dt):
        if dt not in self.pg:
            pg_dt, _ = ops.fedopt_dtypes(ops.torch_dtype(dt), self.old[dt].dtype, None)
            self.pg[dt] = torch.empty(self.layout.group_elems[dt], dtype=pg_dt, device=self.device)
        return self.pg[dt]

    def _h2d_old(self, dt, lo, hi):
        """Enqueue the H2D of elements [lo, hi) of the global model's group ``dt`` (copy stream)."""
        odt, parts = self.old_host[dt]
        self._copy_used = True
        return self.streamer.h2d(parts, odt, lo, hi, self.old[dt][lo:hi], self.copy)

    def _h2d_old_small(self, dt):
        """A small global model's group ``dt`` to HBM: its tensors copied into one pinned block and
        one H2D enqueued on the compute stream (no ring, no copy-stream hand-off)."""
        odt, parts = self.old_host[dt]
        host = torch.empty(self.layout.group_elems[dt], dtype=ops.torch_dtype(odt), pin_memory=True)
        view = host.numpy()
        for a, off in parts:
            np.copyto(view[off:off + a.size], a, casting="no")
        with torch.cuda.device(self.device), torch.cuda.stream(self.compute):
            self.old[dt].copy_(host, non_blocking=True)
        self._hold.append(host)                 # the pinned block lives until the round's sync
        self.old_ready.add(dt)

    def _old_dev(self, dt):
        """The whole global-model group on the device (compute stream ordered after its H2D)."""
        if dt not in self.old_ready and self.layout.nbytes <= SMALL_UPDATE_BYTES:
            self._h2d_old_small(dt)
        if dt not in self.old_ready:
            self.compute.wait_event(self._h2d_old(dt, 0, self.layout.group_elems[dt]))
            self.old_ready.add(dt)
        return self.old[dt]

    def _fold_pg(self, entries):
        """Fold ``entries`` into pg (no server step): one launch per group over the entries' device
        addresses (arena pieces, slots and staged models on this device: no tensor view per update).
        All-or-nothing: on a failed launch pg is as before the call (copied aside first when the
        groups' launches continue a started pg) and the FedAggError propagates."""
        span = self._kernel_span()
        ns, Ns = [e[1] for e in entries], [e[2] for e in entries]
        addrs = [_addr(e[0]) for e in entries]
        snap = None
        if self.pg_started and len(self.layout.groups) > 1:
            with torch.cuda.device(self.device), torch.cuda.stream(self.compute):
                snap = {dt: self._pg(dt).clone() for dt in self.layout.groups}
        try:
            for dt in self.layout.groups:
                old = self._old_dev(dt)
                off = self.layout.group_byte_offset[dt]
                ops.fedopt_step_raw(old.data_ptr(), old.dtype, [p + off for p in addrs], ops.torch_dtype(dt), ns, Ns,
                                    old.numel(), first=not self.pg_started, final=False,
                                    pg_ptr=self._pg(dt).data_ptr(), stream=self.compute, device=self.device)
        except ops.FedAggError:
            if snap is not None:
                with torch.cuda.device(self.device), torch.cuda.stream(self.compute):
                    for dt, t in snap.items():
                        self._pg(dt).copy_(t)
            raise
        self._end_span(span)
        self.pg_started = True

    def _fold_pg_isolated(self, entries):
        """Fold a batch into pg; if its launch fails, fold its updates one at a time as FEDn does
        (fedopt.py:74-106): an update whose own fold fails is skipped and reported with its tag (its
        examples stay counted), the rest fold in FIFO order."""
        try:
            self._fold_pg(entries)
            return
        except ops.FedAggError:
            pass
        for e in entries:
            try:
                self._fold_pg([e])
            except ops.FedAggError as ex:
                self.skipped.append((e[3] if len(e) > 3 else None, ex))

    def _flush(self):
        if self.pending:
            self.upload_arena()
            entries, self.pending = self.pending, []
            try:
                self._fold_pg_isolated(entries)
            except BaseException as e:          # the batch is lost: never return a model without it
                self.broken = e
                raise

    def _zero_copy_step(self, state, params, opt, sig):
        """A small round that never left the host (see FedAvgPipeline._zero_copy_result): every update
        waits in the arena being filled, none uploaded, pg not started, the global model not on the
        device. ONE fused FIRST + FINAL launch per group reads the clients from the pinned arena and the
        global model from a pinned block through their device addresses and writes the new model into
        the caller's pinned block (m / v stay in HBM) — the same kernel, so the same bits — then one
        synchronize. None if not such a round."""
        a = self._arena
        entries = self.pending
        if (self.pg_started or a is None or a.uploaded or not entries or len(entries) > BATCH
                or a.count * self.layout.nbytes > ZERO_COPY_BYTES or self.old_ready
                or any(type(e[0]) is not _ArenaRef or e[0]._arena is not a for e in entries)):
            return None
        try:
            if a.host_dev is None:
                a.host_dev = ops.host_device_ptr(a.host_ptr, self.device)
        except Exception:  # noqa: BLE001 — no device mapping of the arena: the copy path
            return None
        wait_pack_jobs(self._pack_ticket)
        self._pack_ticket, self._pack_jobs = None, []
        self.pending, self._arena = [], None
        ns, Ns = [e[1] for e in entries], [e[2] for e in entries]
        new_m, new_v, hosts = {}, {}, {}
        t0 = time.perf_counter()                # no event pair: the launch is synchronised right after
        for dt in self.layout.groups:
            P = self.layout.group_elems[dt]
            odt, parts = self.old_host[dt]
            old_t = ops.torch_dtype(odt)
            m_in = state.m[dt] if state.m is not None else None
            v_in = state.v[dt] if state.v is not None else None
            m_dt, sdt = state_dtypes(state, dt, old_t, m_in)
            m_out = torch.empty(P, dtype=m_dt, device=self.device)
            v_out = torch.empty(P, dtype=sdt, device=self.device)
            out = torch.empty(P, dtype=sdt, pin_memory=True)
            new_m[dt], new_v[dt], hosts[dt] = m_out, v_out, out
            if P == 0:                          # a group of empty tensors: nothing to step or map
                continue
            old_h = torch.empty(P, dtype=old_t, pin_memory=True)
            view = old_h.numpy()
            for arr, off in parts:
                np.copyto(view[off:off + arr.size], arr, casting="no")
            self._hold.append(old_h)            # read by the launch until the round's sync
            off = self.layout.group_byte_offset[dt]
            try:
                ops.fedopt_step_raw(ops.host_device_ptr(old_h.data_ptr(), self.device), old_t,
                                    [a.host_dev + e[0]._lo + off for e in entries], ops.torch_dtype(dt), ns, Ns, P,
                                    first=True, final=True, m_in=m_in, m_out=m_out, v_in=v_in, v_out=v_out,
                                    out_ptr=ops.host_device_ptr(out.data_ptr(), self.device), state_dt=sdt,
                                    serveropt=opt, learning_rate=params["learning_rate"], beta1=params["beta1"],
                                    beta2=params["beta2"], tau=params["tau"], stream=self.compute,
                                    device=self.device)
            except ops.FedAggError:
                # nothing of the session's state was replaced: the round goes the device way (upload,
                # pseudo-gradient one update at a time if need be, then the server step alone)
                self.compute.synchronize()
                self.pending, self._arena = entries, a
                return None
        self.pg_started = True
        self.compute.synchronize()              # the arena's pinned bytes are read until here: free again
        a.done, a.used = None, False
        self._kern_wall += time.perf_counter() - t0
        self._d2h_on_compute = True
        self._synced = not self._d2h_used and not self._copy_used
        state.m, state.v, state.signature, state.layout = new_m, new_v, sig, self.layout
        model = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            self.layout.unpack_group(hosts[dt].numpy(), dt, model, copy=False)
        return model

    def server_step(self, state, params):
        """Apply adam/yogi/adagrad (fedopt.py:139-258); returns the new model (host, f64)."""
        opt = params["serveropt"]
        if opt not in ("adam", "yogi", "adagrad"):
            raise ValueError(f"Unsupported server optimizer: {opt}")
        sig = self.layout.signature()
        if self.general is None and not state.regroup(self.layout, sig, self.device):
            self._enter_general()               # the state's layout differs from this round's
        if self.general is not None:
            m, v = state.tensors()
            model, m, v = self.general.server_step(m, v, params, fp32=getattr(state, "fp32", False))
            state.set_tensors(m, v)
            return model
        self._check_broken()
        tic = time.perf_counter()
        model = self._zero_copy_step(state, params, opt, sig)
        if model is not None:
            self.time_d2h += time.perf_counter() - tic
            return model
        # one fused launch per group: the pending (device-resident) updates, if any, folded into
        # the pseudo-gradient in registers (FIRST when pg holds nothing yet) and the server
        # step; chunked so that each chunk's D2H of the new model overlaps the next chunk
        self.upload_arena()
        entries, self.pending = self.pending, []
        if not entries and not self.pg_started:
            # every update's fold was skipped: no pseudo-gradient (fedopt.py:110, 117-118)
            raise ValueError("no update was folded into the pseudo-gradient")
        old_ready = set(self.old_ready)
        try:
            return self._fused_step(state, params, opt, sig, entries, tic)
        except ops.FedAggError:
            if not entries:
                raise                           # the server step itself failed (fedopt.py:111-116)
        # the fused launch failed: the pending updates fold into pg one at a time (a failing one is
        # skipped), then the server step runs alone (K = 0); its failure is the round's (None, data)
        self.compute.synchronize()
        self.copy.synchronize()
        self.d2h.synchronize()
        self.old_ready = old_ready              # a global model streamed in part-way is streamed again
        self._fold_pg_isolated(entries)
        return self.server_step(state, params)

    def _fused_step(self, state, params, opt, sig, entries, tic):
        first = not self.pg_started
        new_m, new_v, hosts = {}, {}, {}
        span = self._kernel_span()
        for dt in self.layout.groups:
            old = self.old[dt]
            P = self.layout.group_elems[dt]
            prepare = None
            if dt not in self.old_ready and self.layout.nbytes <= SMALL_UPDATE_BYTES:
                self._h2d_old_small(dt)                 # a small model: one copy, on the compute stream
            elif dt not in self.old_ready:              # stream the global model in with the chunks
                prepare = lambda lo, hi, dt=dt: self.compute.wait_event(self._h2d_old(dt, lo, hi))  # noqa: E731
                self.old_ready.add(dt)
            m_in = state.m[dt] if state.m is not None else None
            v_in = state.v[dt] if state.v is not None else None
            m_dt, sdt = state_dtypes(state, dt, old.dtype, m_in)
            # new m / v buffers (same HBM traffic as in place): a step that fails part-way through
            # its chunks leaves the session's state exactly as the last completed round left it
            m_out = torch.empty(P, dtype=m_dt, device=self.device)
            v_out = torch.empty(P, dtype=sdt, device=self.device)
            out = torch.empty(P, dtype=sdt, device=self.device)
            # pg workspace: needed unless this launch starts AND ends the pseudo-gradient in registers
            pg = self._pg(dt) if (not first or len(entries) > BATCH) else None
            ys = [self.group(e[0], dt) for e in entries]
            ns, Ns = [e[1] for e in entries], [e[2] for e in entries]
            sl = lambda t, lo, hi: None if t is None else t[lo:hi]  # noqa: E731

            def step(lo, hi, old=old, pg=pg, m_in=m_in, m_out=m_out, v_in=v_in, v_out=v_out, out=out, ys=ys, dt=dt):
                ops.fedopt_step(old[lo:hi], [y[lo:hi] for y in ys], ns, Ns, first=first, final=True,
                                pg=sl(pg, lo, hi), m_in=sl(m_in, lo, hi), m_out=m_out[lo:hi], v_in=sl(v_in, lo, hi),
                                v_out=v_out[lo:hi], out=out[lo:hi], serveropt=opt,
                                learning_rate=params["learning_rate"], beta1=params["beta1"], beta2=params["beta2"],
                                tau=params["tau"], stream=self.compute, upd_dtype=ops.torch_dtype(dt))
            hosts[dt] = self._fold_then_d2h(out, step, prepare)
            new_m[dt], new_v[dt] = m_out, v_out
        self._end_span(span)
        self.pg_started = True
        if self._d2h_on_compute:
            self.compute.synchronize()          # a small group came back on the compute stream
        if self._d2h_used or not self._d2h_on_compute:
            self.d2h.synchronize()
        self._synced = self._d2h_on_compute and not self._d2h_used and not self._copy_used
        self.time_d2h += time.perf_counter() - tic
        state.m, state.v, state.signature, state.layout = new_m, new_v, sig, self.layout
        model = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            self.layout.unpack_group(hosts[dt].numpy(), dt, model, copy=False)
        return model


