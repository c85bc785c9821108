"""Device pipelines behind the aggregator plug-ins: pinned H2D staging overlapped with the fold.

FEDn hands the aggregator one client update at a time, in FIFO order, as host
``list[np.ndarray]`` (UpdateHandler.load_model_update, updatehandler.py:90-117). That
order IS the fold order, so each update is folded on arrival:

    host: pack update k+1 into pinned slot  |  copy stream: H2D slot k+1  |  compute stream: fold k

A ring of pinned-host/device slot pairs decouples the three: the host waits only for
the H2D that last read a pinned slot; the copy stream waits (GPU-side event) only for
the fold that last read a device slot. The running aggregate (and FedOpt's pseudo-
gradient, m and v) never leaves HBM until the round's result is copied back.
"""
import time

import numpy as np
import torch

from . import ops
from .ingest import StagedModel
from .layout import Layout


class _Slot:
    __slots__ = ("host", "host_np", "dev", "h2d_start", "h2d_done", "consumed", "used", "reserved")

    def __init__(self, nbytes, device):
        self.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.host_np = self.host.numpy()
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.h2d_start = torch.cuda.Event(enable_timing=True)
        self.h2d_done = torch.cuda.Event(enable_timing=True)
        self.consumed = torch.cuda.Event()
        self.used = False
        self.reserved = False


class _Pipeline:
    def __init__(self, device, layout, nslots):
        self.device = torch.device(device)
        self.layout = layout
        self.compute = torch.cuda.current_stream(self.device)
        self.copy = torch.cuda.Stream(self.device)
        self.nslots = nslots
        self.slots = []                          # created on first use (staged inputs need none)
        self._next = 0
        self._h2d = []
        self._kern = []
        self.time_pack = 0.0
        self.time_d2h = 0.0
        self._hold = []

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

    def stage(self, arrays):
        """Pack host ``arrays`` into a pinned slot and start its H2D copy; returns the slot."""
        s = self._take_slot()
        if s.used:
            s.h2d_done.synchronize()            # pinned bytes no longer read by the DMA
            self.copy.wait_event(s.consumed)    # device bytes no longer read by a fold
        tic = time.perf_counter()
        self.layout.pack(arrays, s.host_np)
        self.time_pack += time.perf_counter() - tic
        with torch.cuda.stream(self.copy):
            s.h2d_start.record(self.copy)
            s.dev.copy_(s.host, non_blocking=True)
            s.h2d_done.record(self.copy)
        self._h2d.append((s.h2d_start, s.h2d_done))
        self.compute.wait_event(s.h2d_done)
        s.used = True
        return s

    def acquire(self, arrays):
        """Device-resident source for ``arrays``: a StagedModel is used in place (the compute
        stream waits for its H2D); host arrays are packed into a ring slot."""
        if isinstance(arrays, StagedModel):
            self.layout.check_layout(arrays.layout)      # raises the numpy-like error
            if arrays.dev.device != self.device:         # staged on another GPU: one D2D copy
                arrays.ready.synchronize()               # (rare) order the copy after its H2D
                with torch.cuda.device(self.device):
                    dev = arrays.dev.to(self.device)
                    ready = torch.cuda.Event()
                    ready.record(torch.cuda.current_stream(self.device))
                arrays = StagedModel(arrays.layout, dev, ready, None)
            self.compute.wait_event(arrays.ready)
            self._hold.append(arrays)                    # keep HBM alive until the round ends
            return arrays
        self.layout.check(arrays)
        return self.stage(arrays)

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
        torch.cuda.synchronize(self.device)
        h2d = sum(a.elapsed_time(b) for a, b in self._h2d) / 1e3
        kern = sum(a.elapsed_time(b) for a, b in self._kern) / 1e3
        return {"time_h2d": h2d, "time_kernel": kern, "time_pack": self.time_pack, "time_d2h": self.time_d2h}


class FedAvgPipeline(_Pipeline):
    """Streaming FedAvg on one device: fedavg.py:109-133 with the fold on the GPU."""

    def __init__(self, device, first_arrays, nslots=3):
        staged = isinstance(first_arrays, StagedModel)
        super().__init__(device, first_arrays.layout if staged else Layout.of(first_arrays), nslots)
        self.first_arrays = first_arrays         # a StagedModel materialises host arrays only if needed
        self.first = self.acquire(first_arrays) if staged else self.stage(first_arrays)
        if not staged:
            self.first.reserved = True
        self.n0 = None
        self.nfolds = 0
        self.agg = {}

    def add(self, arrays, n, N):
        """Fold one more update (n = its num_examples, N = running total including it)."""
        if isinstance(arrays, StagedModel):
            self.layout.check_layout(arrays.layout)
        else:
            self.layout.check(arrays)
        for dt in self.layout.groups:           # refuse before touching device state
            ops.fa_dtype(ops.torch_dtype(dt))
        slot = self.acquire(arrays)
        span = self._kernel_span()
        for dt in self.layout.groups:
            y = self.group(slot, dt)
            if self.nfolds == 0:
                x0 = self.group(self.first, dt)
                acc = torch.empty(y.numel(), dtype=ops.fold_result_dtype(y.dtype, y.dtype), device=self.device)
                ops.fedavg_fold(acc, [x0, y], [0.0, n], [1.0, N], init=True, stream=self.compute)
                self.agg[dt] = acc
            else:
                ops.fedavg_fold(self.agg[dt], [y], [n], [N], init=False, stream=self.compute)
        self._end_span(span)
        if isinstance(slot, _Slot):
            slot.consumed.record(self.compute)
        if self.nfolds == 0 and isinstance(self.first, _Slot):
            self.first.consumed.record(self.compute)
            self.first.reserved = False
        self.nfolds += 1

    def result(self):
        """The aggregated model as a new host ``list[np.ndarray]`` (fedavg.py:145)."""
        if self.nfolds == 0:
            first = self.first_arrays           # `model = model_next` alias (fedavg.py:127-128)
            return first.host if isinstance(first, StagedModel) else first
        out = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            h = self._to_host(self.agg[dt])
            self.layout.unpack_group(h.numpy(), dt, out, copy=False)
        return out


class FedOptState:
    """Server-optimizer state of one fedopt Aggregator instance (fedopt.py:36-38), in HBM.

    ``m`` / ``v`` map a layout group to a flat device tensor (m: f32 or f64, v: f64);
    None until the first server step, exactly like the reference's ``self.m``/``self.v``.
    """

    def __init__(self):
        self.m = None
        self.v = None
        self.signature = None
        self.layout = None

    def reset(self):
        self.__init__()

    def _host(self, d):
        if d is None:
            return None
        out = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            h = d[dt].to("cpu").numpy()
            for i, off in self.layout.members[dt]:
                out[i] = np.array(h[off:off + self.layout.sizes[i]]).reshape(self.layout.shapes[i])
        return out

    def m_host(self):
        """``m`` as host ``list[np.ndarray]`` in tensor order (what fedopt.py keeps in self.m)."""
        return self._host(self.m)

    def v_host(self):
        return self._host(self.v)


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


def check_fedopt_dtypes(layout):
    for dt in layout.groups:
        if ops.torch_dtype(dt) not in (torch.float32, torch.float64, torch.int32, torch.int64):
            raise TypeError(f"FedOpt supports float32/float64/int32/int64 updates, got {dt}")


class FedOptPipeline(_Pipeline):
    """Streaming FedOpt on one device: the pseudo-gradient loop of fedopt.py:74-106 on the
    GPU (pg resident in HBM), then the fused server step (fedopt.py:151-258)."""

    def __init__(self, device, old_arrays, first_arrays, nslots=2):
        layout = first_arrays.layout if isinstance(first_arrays, StagedModel) else Layout.of(first_arrays)
        super().__init__(device, layout, nslots)
        self.old = {dt: torch.from_numpy(flat).pin_memory().to(self.device, non_blocking=True)
                    for dt, flat in old_groups(layout, old_arrays).items()}
        self.pg = {}
        self.old_arrays = old_arrays
        self.nfolds = 0

    def add(self, arrays, n, N):
        if isinstance(arrays, StagedModel):
            self.layout.check_layout(arrays.layout)
        else:
            self.layout.check(arrays)
        check_fedopt_dtypes(self.layout)
        slot = self.acquire(arrays)
        span = self._kernel_span()
        first = self.nfolds == 0
        for dt in self.layout.groups:
            y = self.group(slot, dt)
            old = self.old[dt]
            if first:
                pg_dt, _ = ops.fedopt_dtypes(y.dtype, old.dtype, None)
                self.pg[dt] = torch.empty(y.numel(), dtype=pg_dt, device=self.device)
            ops.fedopt_step(old, [y], [n], [N], first=first, final=False, pg=self.pg[dt], stream=self.compute)
        self._end_span(span)
        if isinstance(slot, _Slot):
            slot.consumed.record(self.compute)
        self.nfolds += 1

    def server_step(self, state, params):
        """Apply adam/yogi/adagrad (fedopt.py:139-258); returns the new model (host, f64)."""
        opt = params["serveropt"]
        if opt not in ("adam", "yogi", "adagrad"):
            raise ValueError(f"Unsupported server optimizer: {opt}")
        sig = self.layout.signature()
        if state.signature is not None and state.signature != sig:
            raise ValueError("model layout changed between rounds; FedOpt state (m, v) does not match")
        new_m, new_v, outs = {}, {}, {}
        span = self._kernel_span()
        for dt in self.layout.groups:
            old, pg = self.old[dt], self.pg[dt]
            m_in = state.m[dt] if state.m is not None else None
            v_in = state.v[dt] if state.v is not None else None
            _, m_dt = ops.fedopt_dtypes(ops.torch_dtype(dt), old.dtype, None if m_in is None else m_in.dtype)
            m_out = m_in if (m_in is not None and m_in.dtype == m_dt) else torch.empty(pg.numel(), dtype=m_dt,
                                                                                        device=self.device)
            v_out = v_in if v_in is not None else torch.empty(pg.numel(), dtype=torch.float64, device=self.device)
            out = torch.empty(pg.numel(), dtype=torch.float64, device=self.device)
            ops.fedopt_step(old, [], [], [], first=False, final=True, pg=pg, m_in=m_in, m_out=m_out, v_in=v_in,
                            v_out=v_out, out=out, serveropt=opt, learning_rate=params["learning_rate"],
                            beta1=params["beta1"], beta2=params["beta2"], tau=params["tau"], stream=self.compute,
                            upd_dtype=ops.torch_dtype(dt))
            new_m[dt], new_v[dt], outs[dt] = m_out, v_out, out
        self._end_span(span)
        state.m, state.v, state.signature, state.layout = new_m, new_v, sig, self.layout
        model = [None] * len(self.layout.shapes)
        for dt in self.layout.groups:
            h = self._to_host(outs[dt])
            self.layout.unpack_group(h.numpy(), dt, model, copy=False)
        return model


