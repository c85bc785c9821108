"""One combiner process, several GPUs: parameter-slice sharding without a collective.

FEDn runs one combiner process per node (combiner.py). With several MI355X in that node the
natural layout is the one of sharded.py, inside one process: device d owns a 4 KiB-aligned
slice of every dtype group (Layout.shard_geometry), folds that slice of every update with the
same kernel and client table, and copies its slice of the aggregate straight into the host
result buffer over its own link. The host result is the concatenation of the slices,
bit-identical to one device. No xGMI traffic: the consumer of the model is the host
(roundhandler.py:465-468).

Updates reach the devices two ways:
* host arrays: device d copies only its slice (H2D in parallel across devices), folded on
  arrival. A tensor of at least INPLACE_MIN_BYTES that lies in page-locked memory already (how
  fedn_amd.helper decodes large npz members) is DMA'd straight from the caller's array; the others
  are packed once into a pinned slot (~70-110 GB/s, native threads) — the pack of every byte bounds
  a many-GPU round on pageable host updates (tools/pack_probe.py, tools/bench_hostres.py,
  profiles/r04_hostres.log; page-locking pageable updates in place instead is INPLACE_REGISTER);
* already sliced over these devices by the streaming ingest
  (ingest.StagingUpdateHandler(devices=...) -> ShardedStagedModel): they queue and fold
  together in one multi-client launch per device (flushed at staging.BATCH), and the round's
  last launch is chunked so that each chunk's D2H — every device over its own link —
  overlaps the next chunk.

FedOpt shards the same way (ShardedFedOptPipeline): device d keeps ITS slice of the global
model, the pseudo-gradient and the server state m / v resident across rounds
(ShardedFedOptState), so a session's optimizer state is spread over the node's HBM and never
moves between devices. The global model streams in through a pinned ring (no whole-model
pinning), chunk by chunk with the server step when every update was device-resident.
"""
import time

import numpy as np
import torch

from . import mixed, ops, reuse
from .ingest import ShardedStagedModel, StagedModel, _member_spans
from .layout import Layout
from .staging import (BATCH, HostStreamer, check_fedopt_dtypes, chunks, fused_fedopt_pair, group_tensors, old_members,
                      state_dtypes)

# host tensors at least this large that are page-locked already (pinned memory: e.g. what
# fedn_amd.helper decodes large npz members into) are DMA'd slice by slice straight from where they lie
# instead of being packed into a pinned slot first (0 disables)
INPLACE_MIN_BYTES = int(__import__("os").environ.get("FEDN_AMD_INPLACE_MIN_BYTES", str(8 << 20)))
# page-lock PAGEABLE tensors in place too (hipHostRegister) — only worth it for host buffers a caller
# reuses round after round: re-registering pages costs ~0.1 ms per 400 MB, but pinning fresh pages
# ~1 ms and unpinning them (hipHostUnregister) ~13 ms per 400 MB, more than the ~4-6 ms pack
# (profiles/r04_hostres.log); FEDn decodes every round's updates into new arrays, so off by default
INPLACE_REGISTER = __import__("os").environ.get("FEDN_AMD_INPLACE_REGISTER", "0") == "1"
# caller arrays kept page-locked (and referenced) after their H2D until the round ends, at most this many
# bytes: beyond it they are unregistered in one batch (each hipHostUnregister waits for the DMA in flight)
INPLACE_HOLD_BYTES = int(__import__("os").environ.get("FEDN_AMD_INPLACE_HOLD_BYTES", str(16 << 30)))


class _DevSlot:
    __slots__ = ("dev", "h2d_done", "consumed", "used")

    def __init__(self, nbytes, device):
        self.dev = reuse.watch(torch.empty(nbytes, dtype=torch.uint8, device=device))
        self.h2d_done = torch.cuda.Event()
        self.consumed = torch.cuda.Event()
        self.used = False


def gather_group(layout, bounds, devices, per_dev, dt):
    """Concatenate the device slices ``per_dev[d]`` (bounds[d] = its [lo, hi)) of group ``dt``
    into a new host array: each device D2H's its slice over its own link."""
    rdt = per_dev[0].dtype
    flat = torch.empty(layout.group_elems[dt], dtype=rdt, pin_memory=True)
    for d, dv in enumerate(devices):
        lo, hi = bounds[d]
        if hi > lo:
            with torch.cuda.device(dv):
                flat[lo:hi].copy_(per_dev[d], non_blocking=True)
    for dv in devices:
        torch.cuda.current_stream(dv).synchronize()
    return flat.numpy()   # a new pinned block owned by the caller (see staging._Pipeline._to_host)


def allgather_devices(parts, P, engine="dma", records=None):
    """The in-process form of the sliced all-gather: ``parts`` = [(device, slice
    tensor on it, lo)] covering [0, P); returns one full P-element model per device. Device d's slice
    goes straight into every other device's model over the d -> e link (after ``fa_peer_enable``),
    all links at once: ``engine="dma"`` copies it with one ``fa_copy_async`` per (source,
    destination) pair, each on its own stream; ``engine="kernel"`` with ONE ``fa_push`` launch per
    source that reads the slice once and stores it into every destination (sharded.P2PAllGather's
    two engines). Each destination's current stream then waits for what lands in it. A device listed
    twice (tests on a one-GPU box) gets its own model buffer per entry. ``records``: a list that
    receives, per kernel push, the release record its XCD-covering release grid wrote (read with
    ``ops.read_release_record`` once the destinations have synchronised; ``misses`` must be 0)."""
    if engine not in ("dma", "kernel"):
        raise ValueError("allgather_devices: engine must be 'dma' or 'kernel'")
    parts = [(torch.device(dv), t, lo) for dv, t, lo in parts]
    fulls = []
    for d, (dv, t, lo) in enumerate(parts):
        if lo < 0 or lo + t.numel() > P:
            raise ValueError(f"allgather_devices: part {d} [{lo}, {lo + t.numel()}) outside [0, {P})")
        fulls.append(torch.empty(P, dtype=t.dtype, device=dv))
    if sum(t.numel() for _, t, _ in parts) != P:
        raise ValueError("allgather_devices: the parts do not cover the model")
    done = [[] for _ in parts]
    for i, (src_dev, t, lo) in enumerate(parts):
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(src_dev))
        es = t.element_size()
        for dst_dev, _, _ in parts:
            if src_dev.index != dst_dev.index:
                ops.peer_enable(src_dev.index, dst_dev.index)
        if engine == "kernel":
            st = torch.cuda.Stream(src_dev)
            st.wait_event(ready)
            rec = ops.release_record(src_dev) if records is not None else None
            ops.push([f.data_ptr() + lo * es for f in fulls], t, t.numel() * es, st, release_rec=rec)
            if rec is not None:
                records.append(rec)
            ev = torch.cuda.Event()
            ev.record(st)
            for j in range(len(parts)):
                done[j].append((ev, st))
            continue
        for j in range(len(parts)):
            st = torch.cuda.Stream(src_dev)
            st.wait_event(ready)
            ops.copy_async(fulls[j].data_ptr() + lo * es, t, t.numel() * es, st)
            ev = torch.cuda.Event()
            ev.record(st)
            done[j].append((ev, st))
    for j, (dst_dev, _, _) in enumerate(parts):
        cur = torch.cuda.current_stream(dst_dev)
        for ev, _ in done[j]:
            cur.wait_event(ev)
    return fulls


def _same_devices(a, b):
    return [str(torch.device(d)) for d in a] == [str(torch.device(d)) for d in b]


def _host_arrays(arrays):
    """Host arrays of an update staged for other devices (re-sharded from the host copy)."""
    return arrays.host if isinstance(arrays, (StagedModel, ShardedStagedModel)) else arrays


class _ShardedStaging:
    """Host slots packed once, each device's slice of every group copied over its own link; or
    updates already sliced over these devices (ShardedStagedModel), used in place."""

    def __init__(self, devices, layout, nslots):
        self.devices = [torch.device(d) for d in devices]
        self.layout = layout
        self.bounds, self.dev_off, self.dev_bytes = layout.shard_geometry(len(self.devices))
        self.compute = [torch.cuda.current_stream(dv) for dv in self.devices]
        self.copy = [torch.cuda.Stream(dv) for dv in self.devices]
        self.d2h = [torch.cuda.Stream(dv) for dv in self.devices]
        self.nslots = nslots
        self.host = None                               # pinned host slots: on the first host update
        self.host_done = [None] * nslots               # per host slot: the H2D events reading it
        # per host slot: the caller's arrays page-locked in place for its H2D, [(address, array)] —
        # referenced and registered until those H2D events have fired (then unregistered)
        self.inplace = [[] for _ in range(nslots)]
        self._locks = {}                               # address -> [slots using it, registered here, array, bytes]
        self._retired, self._retired_bytes = [], 0     # registered here, no longer read: [(address, array)]
        self.inplace_bytes = 0                         # bytes DMA'd from page-locked caller memory
        self.time_stage_wait = self.time_stage_host = 0.0
        self.packed_bytes = 0                          # bytes packed into the pinned slots
        self.dslots = None
        self._next = 0
        self.reserved = set()
        self.pending = []                              # resident updates not folded yet: (model, n, N, tag)
        self.skipped = []                              # (tag, exception): see staging._Pipeline.skipped
        self.broken = None
        # resident updates read by enqueued launches: kept until the pipeline (the round) ends, as
        # staging._Pipeline._hold does. Dropped when their fold is merely enqueued, their HBM went
        # back to torch's allocator and a staging worker could refill it (H2D on its own stream)
        # before the compute stream had read it — a multi-device round then folded another
        # update's bytes (GPU test test_multidevice_sharded_ingest_fedavg[3-70], round 5)
        self._hold = []

    def take_skipped(self):
        out, self.skipped = self.skipped, []
        return out

    def unsettled(self):
        return len(self.pending)

    def _check_broken(self):
        if self.broken is not None:
            raise RuntimeError(f"a batched fold failed and could not be recovered: {self.broken}") from self.broken

    def _sync_all(self):
        for st in (*self.compute, *self.copy, *self.d2h):
            st.synchronize()

    def _copy_aside(self, per_dev):
        """Device copies of ``per_dev`` ([{group: tensor}] per device) on each compute stream
        (staging.NO_SNAPSHOT when HBM cannot hold them: see staging._Pipeline._snapshot)."""
        from .staging import NO_SNAPSHOT
        out = []
        try:
            for d, dv in enumerate(self.devices):
                with torch.cuda.device(dv), torch.cuda.stream(self.compute[d]):
                    out.append({dt: t.clone() for dt, t in per_dev[d].items()})
        except torch.cuda.OutOfMemoryError:
            return NO_SNAPSHOT
        return out

    def _copy_back(self, per_dev, snap):
        from .staging import NO_SNAPSHOT
        if snap is NO_SNAPSHOT:
            self.broken = RuntimeError("a multi-launch fold failed part-way and the aggregate could not be "
                                       "copied aside beforehand (HBM full): the round is lost")
            raise self.broken
        if snap is None:
            return
        for d, dv in enumerate(self.devices):
            with torch.cuda.device(dv), torch.cuda.stream(self.compute[d]):
                for dt, t in snap[d].items():
                    per_dev[d][dt].copy_(t)

    def _ensure_slots(self):
        if self.host is None:
            self.host = [torch.empty(self.layout.nbytes, dtype=torch.uint8, pin_memory=True)
                         for _ in range(self.nslots)]
            self.dslots = [[_DevSlot(self.dev_bytes[d], self.devices[d]) for _ in range(self.nslots)]
                           for d in range(len(self.devices))]
            # fresh HBM from each compute stream's pool: its previous owners' queued work there runs
            # before the copy streams' H2D overwrite it (staging._Pipeline.stage)
            for d in range(len(self.devices)):
                self.copy[d].wait_stream(self.compute[d])

    def _dev_view(self, d, slot, dt):
        lo, hi = self.bounds[dt][d]
        off = self.dev_off[d][dt]
        return self.dslots[d][slot].dev[off:off + (hi - lo) * dt.itemsize].view(ops.torch_dtype(dt))

    def _view(self, d, src, dt):
        """Device d's slice of group dt of an update: a host-staged slot or a ShardedStagedModel."""
        return self._dev_view(d, src, dt) if isinstance(src, int) else src.view(d, dt)

    def _resident(self, arrays):
        return isinstance(arrays, ShardedStagedModel) and _same_devices(arrays.devices, self.devices)

    def _accept(self, model):
        """Order every device's compute stream after the resident update's H2D; hold its HBM until
        the round ends (see ``_hold``)."""
        for d in range(len(self.devices)):
            self.compute[d].wait_event(model.ready[d])
        self._hold.append(model)

    # ---- per-tensor path (mixed.py) on the first device: updates that differ in layout ------
    def compatible(self, arrays):
        if self._resident(arrays):
            return arrays.layout.signature() == self.layout.signature()
        arrays = _host_arrays(arrays)
        if len(arrays) != len(self.layout.shapes):
            return False
        return all(tuple(np.shape(a)) == self.layout.shapes[i] and np.asarray(a).dtype == self.layout.dtypes[i]
                   for i, a in enumerate(arrays))

    def meta_of(self, arrays):
        if self._resident(arrays):
            return list(zip(arrays.layout.shapes, arrays.layout.dtypes))
        return mixed.host_meta(_host_arrays(arrays))

    def gathered(self, layout, bounds, slices):
        """Per-tensor tensors on the first device from per-device slices ``slices[d][dt]``."""
        return mixed.tensor_views(layout, mixed.gather_flats(layout, bounds, self.devices, slices, self.devices[0]))

    def tensors_of(self, arrays):
        """An update as per-tensor tensors on the first device (the per-tensor path runs there)."""
        if self._resident(arrays):
            self._accept(arrays)
            return self.gathered(arrays.layout, arrays.bounds, [{dt: arrays.view(d, dt) for dt in arrays.layout.groups}
                                                 for d in range(len(self.devices))])
        return mixed.upload(_host_arrays(arrays), self.devices[0], self.compute[0])

    def _unlock(self, s):
        """Release the caller arrays slot ``s``'s last H2D read in place (its events have fired). One no
        other slot still uses, and that this pipeline registered, is retired: kept page-locked (and
        referenced) until the round ends — hipHostUnregister waits for every DMA in flight on the
        device (7 ms with one 400 MB H2D queued, profiles/r04_pack_inplace.log), so unregistering
        mid-round would stall the pipeline once per update. Past INPLACE_HOLD_BYTES retired bytes they
        are unregistered together (one stall per batch) so the host memory held stays bounded."""
        for ptr, _ in self.inplace[s]:
            ent = self._locks[ptr]
            ent[0] -= 1
            if ent[0] == 0:
                del self._locks[ptr]
                if ent[1]:
                    self._retired.append((ptr, ent[2]))
                    self._retired_bytes += ent[3]
        self.inplace[s] = []
        if self._retired_bytes > INPLACE_HOLD_BYTES:
            self._unregister_retired()

    def _unregister_retired(self):
        for ptr, _ in self._retired:
            ops.host_unregister_ptr(ptr)
        self._retired, self._retired_bytes = [], 0

    def quiesce(self):
        """Every host slot's H2D done and its in-place registrations undone (the round is over or
        abandoned: the caller's arrays may be freed after this; the device is idle, so each
        unregistration is cheap)."""
        for s in range(self.nslots):
            if self.host_done[s] is not None:
                for ev in self.host_done[s]:
                    ev.synchronize()
            self._unlock(s)
        self._unregister_retired()

    def __del__(self):
        try:
            self.quiesce()                             # a pipeline dropped without its round's end
        except Exception:  # noqa: BLE001 — interpreter shutdown: the process's pinnings go with it
            pass

    def _lock_in_place(self, arrays, s):
        """{tensor index: host address} of the tensors of ``arrays`` DMA'd from where they lie:
        C-contiguous ndarrays of their layout dtype of at least INPLACE_MIN_BYTES, page-locked here
        (or already page-locked, e.g. torch pinned blocks); a tensor that cannot be (pages shared
        with one already registered, ...) is packed instead."""
        out = {}
        if INPLACE_MIN_BYTES <= 0:
            return out
        for i, _, nb in self.layout.pack_plan:
            a = arrays[i]
            if nb < INPLACE_MIN_BYTES or type(a) is not np.ndarray or not a.flags.c_contiguous \
                    or a.dtype != self.layout.dtypes[i]:
                continue
            ptr = a.ctypes.data
            ent = self._locks.get(ptr)
            if ent is None:
                try:                                   # page-locked already (a torch pinned block, its owner
                    ops.host_device_ptr(ptr, self.devices[0])     # registered it, or retired here): as is
                    ent = [0, False, a, nb]
                except ops.FedAggError:
                    if not INPLACE_REGISTER:
                        continue                       # pageable: packing it is cheaper (see INPLACE_REGISTER)
                    try:
                        ops.host_register_ptr(ptr, nb)
                        ent = [0, True, a, nb]
                    except ops.FedAggError:
                        continue                       # e.g. pages shared with a registered block: pack it
                self._locks[ptr] = ent
            ent[0] += 1                                # the same array handed over twice: registered once
            self.inplace[s].append((ptr, a))
            out[i] = ptr
        return out

    def _stage(self, arrays):
        self._ensure_slots()
        for _ in range(self.nslots):
            s = self._next
            self._next = (self._next + 1) % self.nslots
            if s not in self.reserved:
                break
        t0 = time.perf_counter()
        if self.host_done[s] is not None:
            for ev in self.host_done[s]:
                ev.synchronize()                       # pinned bytes no longer read by any DMA
        t1 = time.perf_counter()
        self.time_stage_wait += t1 - t0                # backpressure of the links (slot ring full)
        self._unlock(s)
        lay = self.layout
        inplace = self._lock_in_place(arrays, s)
        if inplace:                                    # pack only the other tensors
            host = self.host[s].numpy()
            for dt in lay.groups:
                g = lay.group_view(host, dt)
                for i, off in lay.members[dt]:
                    if i not in inplace and lay.sizes[i]:
                        np.copyto(g[off:off + lay.sizes[i]], np.asarray(arrays[i]).reshape(-1), casting="no")
        else:
            lay.pack(arrays, self.host[s].numpy())
        hbase = self.host[s].data_ptr()
        evs = []
        for d, dv in enumerate(self.devices):
            ds = self.dslots[d][s]
            if ds.used:
                self.copy[d].wait_event(ds.consumed)
            with torch.cuda.device(dv), torch.cuda.stream(self.copy[d]):
                for dt in lay.groups:
                    lo, hi = self.bounds[dt][d]
                    if hi <= lo:
                        continue
                    isz, goff = dt.itemsize, lay.group_byte_offset[dt]
                    dbase = self._dev_view(d, s, dt).data_ptr()
                    if not inplace:
                        ops.copy_ptr_async(dbase, hbase + goff + lo * isz, (hi - lo) * isz, self.copy[d], dv)
                        continue
                    for i, e0, n, o in _member_spans(lay, dt, lo, hi):
                        src = inplace[i] + e0 * isz if i in inplace else hbase + goff + (lo + o) * isz
                        ops.copy_ptr_async(dbase + o * isz, src, n * isz, self.copy[d], dv)
                ds.h2d_done.record(self.copy[d])
            self.compute[d].wait_event(ds.h2d_done)
            ds.used = True
            evs.append(ds.h2d_done)
        self.host_done[s] = evs
        nin = sum(lay.sizes[i] * lay.dtypes[i].itemsize for i in inplace)
        self.inplace_bytes += nin
        self.packed_bytes += lay.nbytes - nin
        self.time_stage_host += time.perf_counter() - t1   # page-lock / pack + enqueue: the host's own work
        return s

    def _to_host_chunks(self, dt, per_dev, fold_chunk, rdtype):
        """New pinned host array of group ``dt``: device d's slice ``per_dev[d]`` is D2H'd into
        its [lo, hi) chunk by chunk on the device's d2h stream, ``fold_chunk(d, clo, chi)`` (if
        given) enqueued on its compute stream first, so each chunk's D2H overlaps the next."""
        flat = torch.empty(self.layout.group_elems[dt], dtype=rdtype, pin_memory=True)
        for d, dv in enumerate(self.devices):
            lo, hi = self.bounds[dt][d]
            src = per_dev[d]
            with torch.cuda.device(dv):
                for clo, chi in chunks(hi - lo, src.element_size()):
                    if fold_chunk is not None:
                        fold_chunk(d, clo, chi)
                    ev = torch.cuda.Event()
                    ev.record(self.compute[d])
                    self.d2h[d].wait_event(ev)
                    with torch.cuda.stream(self.d2h[d]):
                        flat[lo + clo:lo + chi].copy_(src[clo:chi], non_blocking=True)
        return flat

    def _sync_d2h(self):
        for st in self.d2h:
            st.synchronize()

    def timings(self):
        return {"bytes_h2d_in_place": self.inplace_bytes, "bytes_h2d_packed": self.packed_bytes,
                "time_stage_host": self.time_stage_host, "time_stage_wait": self.time_stage_wait}


class ShardedFedAvgPipeline(_ShardedStaging):
    """FedAvgPipeline over ``devices`` (a list; the same device may repeat, e.g. in tests)."""

    def __init__(self, devices, first_arrays, nslots=3):
        if isinstance(first_arrays, ShardedStagedModel) and _same_devices(first_arrays.devices, devices):
            super().__init__(devices, first_arrays.layout, nslots)
            self._accept(first_arrays)
            self.first = first_arrays
        else:
            first_arrays = _host_arrays(first_arrays)
            super().__init__(devices, Layout.of(first_arrays), nslots)
            self.first = self._stage(first_arrays)
            self.reserved = {self.first}
        self.first_arrays = first_arrays
        self.nfolds = 0
        self.agg_started = False
        self.agg = [dict() for _ in self.devices]
        self.general = None

    def _state_meta(self):
        lay = self.layout
        if self.nfolds == 0:
            return list(zip(lay.shapes, lay.dtypes))
        return [(sh, mixed.np_dtype(ops.fold_result_dtype(ops.torch_dtype(d), ops.torch_dtype(d))))
                for sh, d in zip(lay.shapes, lay.dtypes)]

    def _enter_general(self):
        """Continue the round per tensor on the first device (mixed.TensorFedAvg)."""
        self._flush()
        if self.agg_started:
            slices = [{dt: self._agg(d, dt) for dt in self.layout.groups} for d in range(len(self.devices))]
        else:
            slices = [{dt: self._view(d, self.first, dt) for dt in self.layout.groups} for d in range(len(self.devices))]
        self.general = mixed.TensorFedAvg(self.devices[0], self.compute[0], self.gathered(self.layout, self.bounds, slices),
                                          owned=True)

    def add(self, arrays, n, N, tag=None):
        self._check_broken()
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
        resident = self._resident(arrays)
        if not resident:
            arrays = _host_arrays(arrays)
        for dt in self.layout.groups:           # refuse before touching device state
            ops.fa_dtype(ops.torch_dtype(dt))
        if resident:
            self._accept(arrays)
            self.pending.append((arrays, n, N, tag))
            if len(self.pending) >= BATCH:
                self._flush()
        else:
            self._flush()
            s = self._stage(arrays)
            try:
                self._fold_all([(s, n, N)])     # all-or-nothing: the caller skips the update on failure
            finally:
                for d in range(len(self.devices)):
                    self.dslots[d][s].consumed.record(self.compute[d])
        self.nfolds += 1

    def _snapshot(self):
        """The aggregate slices copied aside before a continuation fold of several launches (see
        staging.FedAvgPipeline._snapshot); None when a failed fold cannot leave it half-advanced."""
        if not self.agg_started or len(self.devices) * len(self.layout.groups) <= 1:
            return None
        return self._copy_aside([{dt: self._agg(d, dt) for dt in self.layout.groups} for d in range(len(self.devices))])

    def _restore(self, snap):
        self._copy_back([{dt: self._agg(d, dt) for dt in self.layout.groups} for d in range(len(self.devices))], snap)

    def _refold_singly(self, entries):
        """A batched fold over ``entries`` failed: one update at a time (fedavg.py:47-78); an update
        whose own fold fails is skipped and reported, the aggregate left as before it."""
        for e in entries:
            try:
                self._fold_all([e])
            except ops.FedAggError as ex:
                self.skipped.append((e[3] if len(e) > 3 else None, ex))

    def _alias(self):
        return _host_arrays(self.first_arrays)   # `model = model_next` alias (fedavg.py:65-66)

    def _agg(self, d, dt):
        if dt not in self.agg[d]:
            t = ops.torch_dtype(dt)
            lo, hi = self.bounds[dt][d]
            self.agg[d][dt] = torch.empty(hi - lo, dtype=ops.fold_result_dtype(t, t), device=self.devices[d])
        return self.agg[d][dt]

    def _fold_dev(self, d, dt, entries, init, clo, chi):
        """Enqueue device d's fold of ``entries`` over elements [clo, chi) of its slice of ``dt``."""
        if chi <= clo:
            return
        ys = [self._view(d, e[0], dt)[clo:chi] for e in entries]
        ns = [e[1] for e in entries]
        Ns = [e[2] for e in entries]
        acc = self._agg(d, dt)[clo:chi]
        if init:                                # agg := first update, then fold (fedavg.py:65-71)
            x0 = self._view(d, self.first, dt)[clo:chi]
            ops.fedavg_fold(acc, [x0] + ys, [0.0] + ns, [1.0] + Ns, init=True, stream=self.compute[d])
        else:
            ops.fedavg_fold(acc, ys, ns, Ns, init=False, stream=self.compute[d])

    def _folded(self):
        if not self.agg_started and isinstance(self.first, int):
            for d in range(len(self.devices)):
                self.dslots[d][self.first].consumed.record(self.compute[d])
            self.reserved = set()
        self.agg_started = True

    def _fold_all(self, entries):
        """One fold of ``entries`` on every device and group, all-or-nothing: on a failed launch the
        aggregate is put back (or stays unstarted) and the FedAggError propagates."""
        init = not self.agg_started
        snap = None
        try:
            snap = self._snapshot()
            for d in range(len(self.devices)):
                for dt in self.layout.groups:
                    lo, hi = self.bounds[dt][d]
                    self._fold_dev(d, dt, entries, init, 0, hi - lo)
        except ops.FedAggError:
            self._restore(snap)
            raise
        self._folded()

    def _flush(self):
        if self.pending:
            entries, self.pending = self.pending, []
            try:
                try:
                    self._fold_all(entries)
                except ops.FedAggError:
                    self._refold_singly(entries)
            except BaseException as e:          # the batch is lost: never return a model without it
                self.broken = e
                raise

    def result(self):
        self._check_broken()
        if self.nfolds == 0:
            return self._alias()
        if self.general is not None:
            return self.general.result()
        entries, self.pending = self.pending, []
        if not entries and not self.agg_started:
            return self._alias()                # every fold after the first update was skipped
        init = not self.agg_started
        flats = {}
        snap = self._snapshot() if entries else None
        try:
            for dt in self.layout.groups:
                t = ops.torch_dtype(dt)
                fold = None
                if entries:
                    fold = lambda d, clo, chi, dt=dt: self._fold_dev(d, dt, entries, init, clo, chi)  # noqa: E731
                per_dev = [self._agg(d, dt) for d in range(len(self.devices))]
                flats[dt] = self._to_host_chunks(dt, per_dev, fold, ops.fold_result_dtype(t, t))
        except ops.FedAggError:
            if not entries:
                raise
            self._sync_all()
            self._restore(snap)
            self._refold_singly(entries)
            entries = []
            if not self.agg_started:
                self._sync_all()
                return self._alias()
            flats = {}
            for dt in self.layout.groups:
                t = ops.torch_dtype(dt)
                per_dev = [self._agg(d, dt) for d in range(len(self.devices))]
                flats[dt] = self._to_host_chunks(dt, per_dev, None, ops.fold_result_dtype(t, t))
        if entries:
            self._folded()
        self._sync_d2h()
        out = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            self.layout.unpack_group(flats[dt].numpy(), dt, out, copy=False)
        return out


class ShardedFedOptState:
    """FedOptState whose m / v are per-device slices: ``m[d][dt]`` is device d's slice. After a
    round on the per-tensor path the state is per tensor on the first device (``m_t``/``v_t``)
    and is re-sliced over the devices when a later round's layout allows it."""

    def __init__(self, fp32=False):
        self.m = None
        self.v = None
        self.signature = None
        self.layout = None
        self.bounds = None
        self.devices = None
        self.m_t = None
        self.v_t = None
        self.fp32 = fp32            # fp32-state mode (staging.FedOptState)

    def reset(self):
        self.__init__(self.fp32)

    def tensors(self, device=None):
        """(m, v) per tensor (model order) on ``device`` (default: the first device), or (None, None)."""
        if self.m_t is not None:
            return self.m_t, self.v_t
        if self.m is None:
            return None, None
        dev = device if device is not None else self.devices[0]
        out = []
        for per_dev in (self.m, self.v):
            flats = mixed.gather_flats(self.layout, self.bounds, self.devices, per_dev, dev)
            out.append(mixed.tensor_views(self.layout, flats))
        return out[0], out[1]

    def set_tensors(self, m_t, v_t):
        self.m = self.v = self.signature = self.layout = self.bounds = self.devices = None
        self.m_t, self.v_t = m_t, v_t

    def regroup(self, layout, sig, bounds, devices):
        """Make the sliced form match ``layout`` over ``devices`` (see staging.FedOptState.regroup)."""
        if self.m is None and self.m_t is None:
            return True
        if self.m is not None and self.signature == sig:
            return True
        m_t, v_t = self.tensors(devices[0])
        grouped = group_tensors(layout, m_t, v_t, devices[0])
        if grouped is None:
            return False
        m_flat, v_flat = grouped
        self.m = [{dt: m_flat[dt][bounds[dt][d][0]:bounds[dt][d][1]].to(dv) for dt in layout.groups}
                  for d, dv in enumerate(devices)]
        self.v = [{dt: v_flat[dt][bounds[dt][d][0]:bounds[dt][d][1]].to(dv) for dt in layout.groups}
                  for d, dv in enumerate(devices)]
        self.signature, self.layout, self.bounds, self.devices = sig, layout, bounds, list(devices)
        self.m_t = self.v_t = None
        return True

    def _host(self, ts):
        return None if ts is None else [t.to("cpu").numpy() for t in ts]

    def m_host(self):
        return self._host(self.tensors()[0])

    def v_host(self):
        return self._host(self.tensors()[1])


class ShardedFedOptPipeline(_ShardedStaging):
    """FedOptPipeline (staging.py) over ``devices``: pseudo-gradient fold and server step on
    every device's slice, each with its slice of old / pg / m / v resident in its HBM."""

    def __init__(self, devices, old_arrays, first_arrays, nslots=2):
        if isinstance(first_arrays, ShardedStagedModel) and _same_devices(first_arrays.devices, devices):
            layout = first_arrays.layout
        else:
            layout = Layout.of(_host_arrays(first_arrays))
        super().__init__(devices, layout, nslots)
        self.old_arrays = old_arrays
        self.general = None
        # see staging.FedOptPipeline: otherwise the round runs per tensor (first device)
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
        # the global model reaches each device lazily through a pinned ring: whole (when a host
        # update must fold into pg) or chunk by chunk inside the server step (H2D || step || D2H)
        self.old = []
        for d, dv in enumerate(self.devices):
            per = {}
            for dt, (odt, _) in self.old_host.items():
                lo, hi = self.bounds[dt][d]
                per[dt] = torch.empty(hi - lo, dtype=ops.torch_dtype(odt), device=dv)
            self.old.append(per)
            self.copy[d].wait_stream(self.compute[d])   # see _ensure_slots
        self.old_ready = set()
        self.streamer = HostStreamer()
        self.pg = [dict() for _ in self.devices]
        self.pg_started = False
        self.nfolds = 0

    def _pg_meta(self):
        return [(sh, mixed.np_dtype(ops.fedopt_dtypes(ops.torch_dtype(d), self.old[0][d].dtype, None)[0]))
                for sh, d in zip(self.layout.shapes, self.layout.dtypes)]

    def _enter_general(self):
        """Continue the round per tensor on the first device (mixed.TensorFedOpt)."""
        self._flush()
        pg = None
        if self.pg_started:
            pg = self.gathered(self.layout, self.bounds, [{dt: self._pg(d, dt) for dt in self.layout.groups}
                                             for d in range(len(self.devices))])
        old = mixed.upload(self.old_arrays, self.devices[0], self.compute[0])
        self.general = mixed.TensorFedOpt(self.devices[0], self.compute[0], old, pg)

    def add(self, arrays, n, N, tag=None):
        self._check_broken()
        if self.general is None and not (self.fused_ok and self.compatible(arrays)):
            splan = mixed.sub_plan(self.meta_of(arrays), mixed.host_meta(self.old_arrays))   # raises as numpy
            if self.nfolds:
                mixed.fold_plan(self._pg_meta(), [(sh, d) for d, sh in splan], n, N)
            self._enter_general()
        if self.general is not None:
            self.general.add(self.tensors_of(arrays), n, N)
            self.nfolds += 1
            return
        resident = self._resident(arrays)
        if not resident:
            arrays = _host_arrays(arrays)
        if resident:
            self._accept(arrays)
            self.pending.append((arrays, n, N, tag))
            if len(self.pending) >= BATCH:
                self._flush()
        else:
            self._flush()
            s = self._stage(arrays)
            try:
                self._fold_pg([(s, n, N)])      # all-or-nothing: the caller skips the update on failure
            finally:
                for d in range(len(self.devices)):
                    self.dslots[d][s].consumed.record(self.compute[d])
        self.nfolds += 1

    def _pg(self, d, dt):
        if dt not in self.pg[d]:
            lo, hi = self.bounds[dt][d]
            pg_dt, _ = ops.fedopt_dtypes(ops.torch_dtype(dt), self.old[d][dt].dtype, None)
            self.pg[d][dt] = torch.empty(hi - lo, dtype=pg_dt, device=self.devices[d])
        return self.pg[d][dt]

    def _h2d_old(self, d, dt, clo, chi):
        """Enqueue the H2D of elements [clo, chi) of device d's slice of the global model."""
        odt, parts = self.old_host[dt]
        lo = self.bounds[dt][d][0]
        return self.streamer.h2d(parts, odt, lo + clo, lo + chi, self.old[d][dt][clo:chi], self.copy[d])

    def _old_all(self, dt):
        if dt not in self.old_ready:
            for d in range(len(self.devices)):
                lo, hi = self.bounds[dt][d]
                self.compute[d].wait_event(self._h2d_old(d, dt, 0, hi - lo))
            self.old_ready.add(dt)

    def _fold_pg(self, entries):
        """``entries`` into every device's pg slices, all-or-nothing (pg copied aside first when a
        started pg is continued by several launches); a failed launch's FedAggError propagates."""
        snap = None
        if self.pg_started and len(self.devices) * len(self.layout.groups) > 1:
            snap = self._copy_aside([{dt: self._pg(d, dt) for dt in self.layout.groups} for d in range(len(self.devices))])
        try:
            for dt in self.layout.groups:
                self._old_all(dt)
                for d in range(len(self.devices)):
                    lo, hi = self.bounds[dt][d]
                    pg = self._pg(d, dt)
                    if hi > lo:
                        ys = [self._view(d, e[0], dt) for e in entries]
                        ops.fedopt_step(self.old[d][dt], ys, [e[1] for e in entries], [e[2] for e in entries],
                                        first=not self.pg_started, final=False, pg=pg, stream=self.compute[d])
        except ops.FedAggError:
            self._copy_back([{dt: self._pg(d, dt) for dt in self.layout.groups} for d in range(len(self.devices))], snap)
            raise
        self.pg_started = True

    def _fold_pg_isolated(self, entries):
        """A batch into pg; on a failed launch one update at a time (fedopt.py:74-106), skipping and
        reporting each update whose own fold fails."""
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
            entries, self.pending = self.pending, []
            try:
                self._fold_pg_isolated(entries)
            except BaseException as e:          # the batch is lost: never return a model without it
                self.broken = e
                raise

    def server_step(self, state, params):
        opt = params["serveropt"]
        if opt not in ("adam", "yogi", "adagrad"):
            raise ValueError(f"Unsupported server optimizer: {opt}")
        sig = (self.layout.signature(), tuple(str(d) for d in self.devices))
        if self.general is None and not state.regroup(self.layout, sig, self.bounds, self.devices):
            self._enter_general()               # the state's layout differs from this round's
        if self.general is not None:
            m, v = state.tensors(self.devices[0])
            model, m, v = self.general.server_step(m, v, params, fp32=getattr(state, "fp32", False))
            state.set_tensors(m, v)
            return model
        self._check_broken()
        # per device and group, one fused launch: pending (resident) updates folded into the
        # pseudo-gradient in registers (FIRST when pg holds nothing yet) and the server step,
        # chunked so that the global model's H2D, the step and the result's D2H overlap
        entries, self.pending = self.pending, []
        if not entries and not self.pg_started:
            raise ValueError("no update was folded into the pseudo-gradient")   # fedopt.py:110, 117-118
        old_ready = set(self.old_ready)
        try:
            return self._fused_step(state, params, opt, sig, entries)
        except ops.FedAggError:
            if not entries:
                raise                           # the server step itself failed (fedopt.py:111-116)
        # see staging.FedOptPipeline.server_step: the batch one update at a time, then K = 0
        self._sync_all()
        self.old_ready = old_ready
        self._fold_pg_isolated(entries)
        return self.server_step(state, params)

    def _fused_step(self, state, params, opt, sig, entries):
        first = not self.pg_started
        ns, Ns = [e[1] for e in entries], [e[2] for e in entries]
        new_m = [dict() for _ in self.devices]
        new_v = [dict() for _ in self.devices]
        flats = {}
        sl = lambda t, lo, hi: None if t is None else t[lo:hi]  # noqa: E731
        for dt in self.layout.groups:
            stream_old = dt not in self.old_ready
            ctx = []
            for d, dv in enumerate(self.devices):
                lo, hi = self.bounds[dt][d]
                P = hi - lo
                old = self.old[d][dt]
                m_in = state.m[d][dt] if state.m is not None else None
                v_in = state.v[d][dt] if state.v is not None else None
                m_dt, sdt = state_dtypes(state, dt, old.dtype, m_in)
                # new m / v buffers: a failed step leaves the session's state untouched (staging.py)
                m_out = torch.empty(P, dtype=m_dt, device=dv)
                v_out = torch.empty(P, dtype=sdt, device=dv)
                out = torch.empty(P, dtype=sdt, device=dv)
                pg = self._pg(d, dt) if (not first or len(entries) > BATCH) else None
                new_m[d][dt], new_v[d][dt] = m_out, v_out
                ctx.append((old, pg, m_in, m_out, v_in, v_out, out))

            def step(d, clo, chi, dt=dt, ctx=ctx, stream_old=stream_old):
                old, pg, m_in, m_out, v_in, v_out, out = ctx[d]
                if stream_old:
                    self.compute[d].wait_event(self._h2d_old(d, dt, clo, chi))
                ys = [self._view(d, e[0], dt)[clo:chi] for e in entries]
                ops.fedopt_step(old[clo:chi], ys, ns, Ns, first=first, final=True, pg=sl(pg, clo, chi),
                                m_in=sl(m_in, clo, chi), m_out=m_out[clo:chi], v_in=sl(v_in, clo, chi),
                                v_out=v_out[clo:chi], out=out[clo:chi], serveropt=opt,
                                learning_rate=params["learning_rate"], beta1=params["beta1"],
                                beta2=params["beta2"], tau=params["tau"], stream=self.compute[d],
                                upd_dtype=ops.torch_dtype(dt))
            flats[dt] = self._to_host_chunks(dt, [c[6] for c in ctx], step, ctx[0][6].dtype)
            self.old_ready.add(dt)
        self.pg_started = True
        self._sync_d2h()
        state.m, state.v, state.signature = new_m, new_v, sig
        state.layout, state.bounds, state.devices = self.layout, self.bounds, self.devices
        model = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            self.layout.unpack_group(flats[dt].numpy(), dt, model, copy=False)
        return model
