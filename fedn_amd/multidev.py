"""One combiner process, several GPUs: parameter-slice sharding without a collective.

FEDn runs one combiner process per node (combiner.py). With several MI355X in that node the
natural layout is the one of sharded.py, inside one process: every update is packed ONCE
into pinned host memory, device d copies only its 4 KiB-aligned slice of every dtype group
over its own PCIe link (H2D in parallel across devices), folds that slice with the same
kernel and client table, and at the end copies its slice of the aggregate straight into
the host result buffer. The host result is the concatenation of the slices, bit-identical
to one device. No xGMI traffic: the consumer of the model is the host
(roundhandler.py:465-468).

FedOpt shards the same way (ShardedFedOptPipeline): device d keeps ITS slice of the global
model, the pseudo-gradient and the server state m / v resident across rounds
(ShardedFedOptState), so a session's optimizer state is spread over the node's HBM and never
moves between devices.
"""
import torch

from . import ops
from .ingest import StagedModel
from .layout import ALIGN, Layout
from .staging import check_fedopt_dtypes, old_groups
from .sharded import shard_bounds


class _DevSlot:
    __slots__ = ("dev", "h2d_done", "consumed", "used")

    def __init__(self, nbytes, device):
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
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


class _ShardedStaging:
    """Host slots packed once, each device's slice of every group copied over its own link."""

    def __init__(self, devices, layout, nslots):
        self.devices = [torch.device(d) for d in devices]
        self.layout = layout
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
        self.reserved = set()

    def _dev_view(self, d, slot, dt):
        lo, hi = self.bounds[dt][d]
        off = self.dev_off[d][dt]
        return self.dslots[d][slot].dev[off:off + (hi - lo) * dt.itemsize].view(ops.torch_dtype(dt))

    def _stage(self, arrays):
        for _ in range(self.nslots):
            s = self._next
            self._next = (self._next + 1) % self.nslots
            if s not in self.reserved:
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

    def _gather_group(self, per_dev, dt):
        return gather_group(self.layout, self.bounds[dt], self.devices, per_dev, dt)

    def timings(self):
        return {}


class ShardedFedAvgPipeline(_ShardedStaging):
    """FedAvgPipeline over ``devices`` (a list; the same device may repeat, e.g. in tests)."""

    def __init__(self, devices, first_arrays, nslots=3):
        if isinstance(first_arrays, StagedModel):
            first_arrays = first_arrays.host     # staged on one device: re-shard from the host copy
        super().__init__(devices, Layout.of(first_arrays), nslots)
        self.first_arrays = first_arrays
        self.first = self._stage(first_arrays)
        self.reserved = {self.first}
        self.nfolds = 0
        self.agg = [dict() for _ in self.devices]

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
            owned = self._gather_group([a[dt] for a in self.agg], dt)
            self.layout.unpack_group(owned, dt, out, copy=False)
        return out


class ShardedFedOptState:
    """FedOptState whose m / v are per-device slices: ``m[d][dt]`` is device d's slice."""

    def __init__(self):
        self.m = None
        self.v = None
        self.signature = None
        self.layout = None
        self.bounds = None
        self.devices = None

    def reset(self):
        self.__init__()

    def _host(self, per_dev):
        if per_dev is None:
            return None
        out = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            owned = gather_group(self.layout, self.bounds[dt], self.devices, [x[dt] for x in per_dev], dt)
            self.layout.unpack_group(owned, dt, out, copy=False)
        return out

    def m_host(self):
        return self._host(self.m)

    def v_host(self):
        return self._host(self.v)


class ShardedFedOptPipeline(_ShardedStaging):
    """FedOptPipeline (staging.py) over ``devices``: pseudo-gradient fold and server step on
    every device's slice, each with its slice of old / pg / m / v resident in its HBM."""

    def __init__(self, devices, old_arrays, first_arrays, nslots=2):
        if isinstance(first_arrays, StagedModel):
            first_arrays = first_arrays.host
        super().__init__(devices, Layout.of(first_arrays), nslots)
        self.old = [dict() for _ in self.devices]
        for dt, flat in old_groups(self.layout, old_arrays).items():
            for d, dv in enumerate(self.devices):
                lo, hi = self.bounds[dt][d]
                src = torch.from_numpy(flat[lo:hi]).pin_memory()
                with torch.cuda.device(dv):
                    self.old[d][dt] = src.to(dv, non_blocking=True)
        self.pg = [dict() for _ in self.devices]
        self.nfolds = 0

    def add(self, arrays, n, N):
        if isinstance(arrays, StagedModel):
            arrays = arrays.host
        self.layout.check(arrays)
        check_fedopt_dtypes(self.layout)
        s = self._stage(arrays)
        first = self.nfolds == 0
        for d, dv in enumerate(self.devices):
            for dt in self.layout.groups:
                y = self._dev_view(d, s, dt)
                old = self.old[d][dt]
                if first:
                    pg_dt, _ = ops.fedopt_dtypes(y.dtype, old.dtype, None)
                    self.pg[d][dt] = torch.empty(y.numel(), dtype=pg_dt, device=dv)
                if y.numel():
                    ops.fedopt_step(old, [y], [n], [N], first=first, final=False, pg=self.pg[d][dt],
                                    stream=self.compute[d])
            self.dslots[d][s].consumed.record(self.compute[d])
        self.nfolds += 1

    def server_step(self, state, params):
        opt = params["serveropt"]
        if opt not in ("adam", "yogi", "adagrad"):
            raise ValueError(f"Unsupported server optimizer: {opt}")
        sig = (self.layout.signature(), tuple(str(d) for d in self.devices))
        if state.signature is not None and state.signature != sig:
            raise ValueError("model layout or devices changed between rounds; FedOpt state (m, v) does not match")
        new_m = [dict() for _ in self.devices]
        new_v = [dict() for _ in self.devices]
        outs = [dict() for _ in self.devices]
        for d, dv in enumerate(self.devices):
            for dt in self.layout.groups:
                old, pg = self.old[d][dt], self.pg[d][dt]
                m_in = state.m[d][dt] if state.m is not None else None
                v_in = state.v[d][dt] if state.v is not None else None
                _, m_dt = ops.fedopt_dtypes(ops.torch_dtype(dt), old.dtype, None if m_in is None else m_in.dtype)
                P = pg.numel()
                m_out = m_in if (m_in is not None and m_in.dtype == m_dt) else torch.empty(P, dtype=m_dt, device=dv)
                v_out = v_in if v_in is not None else torch.empty(P, dtype=torch.float64, device=dv)
                out = torch.empty(P, dtype=torch.float64, device=dv)
                if P:
                    ops.fedopt_step(old, [], [], [], first=False, final=True, pg=pg, m_in=m_in, m_out=m_out,
                                    v_in=v_in, v_out=v_out, out=out, serveropt=opt,
                                    learning_rate=params["learning_rate"], beta1=params["beta1"],
                                    beta2=params["beta2"], tau=params["tau"], stream=self.compute[d],
                                    upd_dtype=ops.torch_dtype(dt))
                new_m[d][dt], new_v[d][dt], outs[d][dt] = m_out, v_out, out
        state.m, state.v, state.signature = new_m, new_v, sig
        state.layout, state.bounds, state.devices = self.layout, self.bounds, self.devices
        model = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            owned = self._gather_group([o[dt] for o in outs], dt)
            self.layout.unpack_group(owned, dt, model, copy=False)
        return model
