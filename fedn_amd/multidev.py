"""One combiner process, several GPUs: parameter-slice sharding without a collective.

FEDn runs one combiner process per node (combiner.py). With several MI355X in that node the
natural layout is the one of sharded.py, inside one process: every update is packed ONCE
into pinned host memory, device d copies only its 4 KiB-aligned slice of every dtype group
over its own PCIe link (H2D in parallel across devices), folds that slice with the same
kernel and client table, and at the end copies its slice of the aggregate straight into
the host result buffer. The host result is the concatenation of the slices, bit-identical
to one device. No xGMI traffic: the consumer of the model is the host
(roundhandler.py:465-468).
"""
import numpy as np
import torch

from . import ops
from .ingest import StagedModel
from .layout import ALIGN, Layout
from .sharded import shard_bounds


class _DevSlot:
    __slots__ = ("dev", "h2d_done", "consumed", "used")

    def __init__(self, nbytes, device):
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.h2d_done = torch.cuda.Event()
        self.consumed = torch.cuda.Event()
        self.used = False


class ShardedFedAvgPipeline:
    """FedAvgPipeline over ``devices`` (a list; the same device may repeat, e.g. in tests)."""

    def __init__(self, devices, first_arrays, nslots=3):
        if isinstance(first_arrays, StagedModel):
            first_arrays = first_arrays.host     # staged on one device: re-shard from the host copy
        self.devices = [torch.device(d) for d in devices]
        self.layout = Layout.of(first_arrays)
        D = len(self.devices)
        # per device: its [lo, hi) of every group and the byte offset of that slice in its slot
        self.bounds = {dt: shard_bounds(self.layout.group_elems[dt], D) for dt in self.layout.groups}
        self.dev_off, self.dev_bytes = [], []
        for d in range(D):
            off, offs = 0, {}
            for dt in self.layout.groups:
                lo, hi = self.bounds[dt][d]
                offs[dt] = off
                off += -(-((hi - lo) * dt.itemsize) // ALIGN) * ALIGN
            self.dev_off.append(offs)
            self.dev_bytes.append(max(off, ALIGN))
        self.compute = [torch.cuda.current_stream(dv) for dv in self.devices]
        self.copy = [torch.cuda.Stream(dv) for dv in self.devices]
        self.nslots = nslots
        self.host = [torch.empty(self.layout.nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(nslots)]
        self.host_done = [None] * nslots               # per host slot: the H2D events reading it
        self.dslots = [[_DevSlot(self.dev_bytes[d], self.devices[d]) for _ in range(nslots)] for d in range(D)]
        self._next = 0
        self.first_arrays = first_arrays
        self.first = self._stage(first_arrays)
        self.reserved = {self.first}
        self.nfolds = 0
        self.agg = [dict() for _ in range(D)]

    def _dev_view(self, d, slot, dt):
        lo, hi = self.bounds[dt][d]
        off = self.dev_off[d][dt]
        return self.dslots[d][slot].dev[off:off + (hi - lo) * dt.itemsize].view(ops.torch_dtype(dt))

    def _stage(self, arrays):
        for _ in range(self.nslots):
            s = self._next
            self._next = (self._next + 1) % self.nslots
            if s not in getattr(self, "reserved", ()):
                break
        if self.host_done[s] is not None:
            for ev in self.host_done[s]:
                ev.synchronize()                       # pinned bytes no longer read by any DMA
        self.layout.pack(arrays, self.host[s].numpy())
        evs = []
        for d, dv in enumerate(self.devices):
            ds = self.dslots[d][s]
            if ds.used:
                self.copy[d].wait_event(ds.consumed)
            with torch.cuda.device(dv), torch.cuda.stream(self.copy[d]):
                for dt in self.layout.groups:
                    lo, hi = self.bounds[dt][d]
                    if hi > lo:
                        off = self.layout.group_byte_offset[dt]
                        src = self.host[s][off + lo * dt.itemsize: off + hi * dt.itemsize]
                        self._dev_view(d, s, dt).view(torch.uint8).copy_(src, non_blocking=True)
                ds.h2d_done.record(self.copy[d])
            self.compute[d].wait_event(ds.h2d_done)
            ds.used = True
            evs.append(ds.h2d_done)
        self.host_done[s] = evs
        return s

    def add(self, arrays, n, N):
        if isinstance(arrays, StagedModel):
            arrays = arrays.host
        self.layout.check(arrays)
        for dt in self.layout.groups:
            ops.fa_dtype(ops.torch_dtype(dt))
        s = self._stage(arrays)
        for d, dv in enumerate(self.devices):
            for dt in self.layout.groups:
                y = self._dev_view(d, s, dt)
                if self.nfolds == 0:
                    x0 = self._dev_view(d, self.first, dt)
                    acc = torch.empty(y.numel(), dtype=ops.fold_result_dtype(y.dtype, y.dtype), device=dv)
                    if y.numel():
                        ops.fedavg_fold(acc, [x0, y], [0.0, n], [1.0, N], init=True, stream=self.compute[d])
                    self.agg[d][dt] = acc
                elif y.numel():
                    ops.fedavg_fold(self.agg[d][dt], [y], [n], [N], init=False, stream=self.compute[d])
            self.dslots[d][s].consumed.record(self.compute[d])
            if self.nfolds == 0:
                self.dslots[d][self.first].consumed.record(self.compute[d])
        if self.nfolds == 0:
            self.reserved = set()
        self.nfolds += 1

    def result(self):
        if self.nfolds == 0:
            return self.first_arrays
        out = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            rdt = self.agg[0][dt].dtype
            flat = torch.empty(self.layout.group_elems[dt], dtype=rdt, pin_memory=True)
            for d, dv in enumerate(self.devices):
                lo, hi = self.bounds[dt][d]
                if hi > lo:
                    with torch.cuda.device(dv):
                        flat[lo:hi].copy_(self.agg[d][dt], non_blocking=True)
            for d, dv in enumerate(self.devices):
                self.compute[d].synchronize()
            owned = np.empty(flat.numel(), dtype=ops.numpy_dtype(rdt))
            owned[:] = flat.numpy()
            self.layout.unpack_group(owned, dt, out, copy=False)
        return out

    def timings(self):
        return {}
