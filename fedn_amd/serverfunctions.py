"""GPU helpers for FEDn server functions.

FEDn runs user aggregation code in its hooks server (fedn/network/combiner/hooks/hooks.py):
``aggregate(previous_global, client_updates)`` once per round (:127-141), or
``incremental_aggregate(client_id, model, metadata, previous_global)`` as each client's
model and metadata arrive (:107-117) followed by ``get_incremental_aggregate_model()``.
The reference ships one example of each (examples/server-functions/server_functions.py,
sf_incremental_aggregation.py). These classes run those two rules on the GPU with numpy's
rounding, so they return bit-identical models:

* :class:`WeightedAverage` — ``aggregate`` of server_functions.py:53-68: running
  ``weighted_sum += params * num_examples`` in previous_global's dtypes, then
  ``/ total_weight``; each client is packed into pinned memory, copied to HBM and folded on
  arrival (``fa_weighted_sum``) — small models in arena batches of up to 64 clients, one copy
  and one launch each (staging.SMALL_UPDATE_BYTES) — and the division is one elementwise pass.
* :class:`IncrementalAverage` — sf_incremental_aggregation.py:24-48: the running model stays
  in HBM between calls; each arriving model is one ``fa_running_mean`` launch
  ``g = (g*(T-n) + m*n)/T``. Like the example, ``total_examples`` is not reset between
  rounds (:12, :30), and an empty round returns the ``previous_global`` last seen (:26, :45-47).

The hooks server decides which functions a user implemented by looking for their ``def`` in
the submitted source (hooks.py:166-182), so user code delegates to these objects rather than
inheriting them (INTEGRATION.md §3 shows the ServerFunctions class).
"""
import torch

from . import ops
from .layout import Layout
from .staging import BATCH, _Pipeline


def _device(device):
    if device is not None:
        return torch.device(device)
    from .aggregators.fedavg import default_device
    return default_device()


def _acc_dtypes(layout, previous_global):
    """np.zeros_like(previous_global[i]) dtype per update-dtype group (must be uniform)."""
    if len(previous_global) != len(layout.shapes):
        raise ValueError("previous global model and client model have different tensor counts")
    out = {}
    for dt in layout.groups:
        dts = set()
        for i, _ in layout.members[dt]:
            p = previous_global[i]
            if tuple(p.shape) != layout.shapes[i]:
                raise ValueError(f"operands could not be broadcast: tensor {i} has shape {layout.shapes[i]}, "
                                 f"previous global has {tuple(p.shape)}")
            dts.add(p.dtype)
        if len(dts) != 1:
            raise TypeError("previous-global tensors of one client dtype group must share a dtype")
        out[dt] = ops.torch_dtype(dts.pop())
    return out


class WeightedAverage:
    """GPU ``aggregate`` rule of examples/server-functions/server_functions.py:53-68."""

    def __init__(self, device=None):
        self.device = device
        self.timings = {}

    def aggregate(self, previous_global, client_updates):
        if len(client_updates) == 0:
            return previous_global                                   # :55-57
        dev = _device(self.device)
        first = next(iter(client_updates.values()))[0]
        layout = Layout.of(first)
        acc_dt = _acc_dtypes(layout, previous_global)
        for dt in layout.groups:
            if acc_dt[dt] not in (torch.float32, torch.float64) or ops.torch_dtype(dt) not in (torch.float32,
                                                                                               torch.float64):
                raise TypeError(f"weighted average on the GPU supports float32/float64, got {dt} into {acc_dt[dt]}")
        pipe = _Pipeline(dev, layout, nslots=2)
        with torch.cuda.device(dev):
            acc = {dt: torch.zeros(layout.group_elems[dt], dtype=acc_dt[dt], device=dev) for dt in layout.groups}
        total_weight = 0
        pending = []                      # small models: arena-batched clients, one launch per batch

        def flush():
            pipe.upload_arena()
            for dt in layout.groups:
                ops.weighted_sum(acc[dt], [pipe.group(e, dt) for e, _ in pending], [w for _, w in pending],
                                 stream=pipe.compute)
            pending.clear()

        for _cid, (client_parameters, metadata) in client_updates.items():   # :60-64, arrival order
            num_examples = metadata.get("num_examples", 1)
            total_weight += num_examples
            layout.check(client_parameters)
            if pipe.batch_host:
                pending.append((pipe.put_small(client_parameters), num_examples))
                if len(pending) >= BATCH or pipe.arena_full():
                    flush()
                continue
            slot = pipe.stage(client_parameters)
            for dt in layout.groups:
                ops.weighted_sum(acc[dt], [pipe.group(slot, dt)], [num_examples], stream=pipe.compute)
            slot.consumed.record(pipe.compute)
        if pending:
            flush()
        out = [None] * len(layout.shapes)
        for dt in layout.groups:                                     # :67 weighted / total_weight
            ops.elementwise("div", acc[dt], x=acc[dt], a=total_weight, stream=pipe.compute)
            layout.unpack_group(pipe._to_host(acc[dt]).numpy(), dt, out, copy=False)
        self.timings = pipe.timings()
        return out


class IncrementalAverage:
    """GPU ``incremental_aggregate`` / ``get_incremental_aggregate_model`` rule of
    examples/server-functions/sf_incremental_aggregation.py:24-48 (running model in HBM)."""

    def __init__(self, device=None):
        self.device = device
        self.total_examples = 0          # :12, never reset (as in the example)
        self.previous_global = None
        self._pipe = None
        self._g = None                   # running model: {group dtype: device tensor}

    def incremental_aggregate(self, client_id, model, client_metadata, previous_global):
        self.previous_global = previous_global                       # :26
        num_examples = client_metadata.get("num_examples", 1)        # :29-30
        self.total_examples += num_examples
        if self._g is None:                                          # :32-33 global_model = model
            layout = Layout.of(model)
            for dt in layout.groups:
                if ops.torch_dtype(dt) not in (torch.float32, torch.float64):
                    raise TypeError(f"incremental average on the GPU supports float32/float64, got {dt}")
            if self._pipe is None or self._pipe.layout.signature() != layout.signature():
                self._pipe = _Pipeline(_device(self.device), layout, nslots=2)
            pipe = self._pipe
            slot = pipe.stage(model)
            with torch.cuda.device(pipe.device), torch.cuda.stream(pipe.compute):
                self._g = {dt: pipe.group(slot, dt).clone() for dt in layout.groups}
            slot.consumed.record(pipe.compute)
            return
        pipe = self._pipe                                            # :36-37
        pipe.layout.check(model)
        slot = pipe.stage(model)
        T = self.total_examples
        for dt in pipe.layout.groups:
            ops.running_mean(self._g[dt], pipe.group(slot, dt), T - num_examples, num_examples, T,
                             stream=pipe.compute)
        slot.consumed.record(pipe.compute)

    def get_incremental_aggregate_model(self):
        g, self._g = self._g, None                                   # :43-44
        if g is None:
            return self.previous_global                              # :45-47
        pipe = self._pipe
        out = [None] * len(pipe.layout.shapes)
        for dt in pipe.layout.groups:
            pipe.layout.unpack_group(pipe._to_host(g[dt]).numpy(), dt, out, copy=False)
        return out
