"""Parameter-slice sharding of the aggregation across the GPUs of one node.

Every output element depends only on the same element of the K client buffers (and of
old / m / v for FedOpt), so the flat parameter vector splits into contiguous slices with
no exchange during the reduce: rank r folds slice r of every update with the same kernel
and the same (n_k, N_k) table, which is bit-identical to the single-GPU result.

Slices are aligned to 4 KiB (1024 fp32) so every shard starts on the kernels' 16-B vector
boundary and on its own DRAM pages. One process per GPU (torch.distributed, backend
"nccl" = RCCL on ROCm). The only collective is optional and outside the reduce: an
all-gather that reassembles the model on every rank (``allgather``), or a gather of the
slices to the host of one rank (``gather_to_host``), which is what FEDn needs because
the combiner serialises the model on the host (roundhandler.py:465-468).
"""
import torch
import torch.distributed as dist

ALIGN_ELEMS = 1024


def shard_bounds(P, nshards, align=ALIGN_ELEMS):
    """Contiguous [lo, hi) slices of P elements, each a multiple of ``align`` except the last."""
    if nshards < 1:
        raise ValueError("nshards must be >= 1")
    per = -(-P // nshards)
    per = -(-per // align) * align
    out = []
    for r in range(nshards):
        lo = min(r * per, P)
        out.append((lo, min(lo + per, P)))
    return out


class ShardedFedAvg:
    """One rank's share of a FedAvg over a P-element flat model.

    ``fold_fn(agg, updates, n, N, init)`` defaults to the libfedagg kernel
    (:func:`fedn_amd.ops.fedavg_fold`); it is a parameter so the sharding and exchange
    logic can be exercised on CPU-only ranks (gloo) by tests with a reference fold.
    """

    def __init__(self, P, group=None, fold_fn=None, align=ALIGN_ELEMS, collective_at_world1=False):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.P = P
        # issue the collectives even at world size 1 (a one-GPU rehearsal of the RCCL calls)
        self.collective = self.world > 1 or (collective_at_world1 and dist.is_initialized())
        self.bounds = shard_bounds(P, self.world, align)
        self.lo, self.hi = self.bounds[self.rank]
        self.shard = self.bounds[0][1] - self.bounds[0][0]   # padded per-rank length
        if fold_fn is None:
            from .ops import fedavg_fold as fold_fn
        self.fold_fn = fold_fn

    def local(self, flat):
        """This rank's slice of a full flat buffer (a view)."""
        return flat[self.lo:self.hi]

    def fold(self, agg_local, updates_local, n, N, init):
        return self.fold_fn(agg_local, updates_local, n, N, init)

    def allgather(self, agg_local):
        """Reassemble the full P-element model on every rank (RCCL all-gather over xGMI)."""
        if not self.collective:
            return agg_local
        buf = agg_local
        if agg_local.numel() != self.shard:
            buf = torch.zeros(self.shard, dtype=agg_local.dtype, device=agg_local.device)
            buf[:agg_local.numel()].copy_(agg_local)
        full = torch.empty(self.shard * self.world, dtype=agg_local.dtype, device=agg_local.device)
        if dist.get_backend(self.group) == "gloo":
            dist.all_gather(list(full.chunk(self.world)), buf, group=self.group)
        else:
            dist.all_gather_into_tensor(full, buf, group=self.group)
        return full[:self.P]

    def gather_to_host(self, agg_local, dst=0):
        """Collect every slice into one host tensor on rank ``dst`` (None elsewhere)."""
        host = agg_local.to("cpu")
        if self.world == 1:
            return host
        buf = torch.zeros(self.shard, dtype=host.dtype)
        buf[:host.numel()] = host
        parts = [torch.empty_like(buf) for _ in range(self.world)] if self.rank == dst else None
        if dist.get_backend(self.group) == "gloo":
            dist.gather(buf, parts, dst=dst, group=self.group)
        else:
            # RCCL gathers device tensors; stage through the device and bring the result back
            dbuf = buf.to(agg_local.device)
            dparts = [torch.empty_like(dbuf) for _ in range(self.world)] if self.rank == dst else None
            dist.gather(dbuf, dparts, dst=dst, group=self.group)
            parts = [p.cpu() for p in dparts] if self.rank == dst else None
        if self.rank != dst:
            return None
        return torch.cat(parts)[:self.P]


class ShardedFedOpt:
    """One rank's share of FedOpt (fedopt.py:74-258) over a P-element flat model: the
    pseudo-gradient fold and the server step are elementwise, so rank r keeps ITS slice of
    ``old``, ``m`` and ``v`` resident and never exchanges state; only the new model slice is
    gathered (``allgather`` / ``gather_to_host`` as in :class:`ShardedFedAvg`).

    ``step_fn(old, updates, n, N, m_in, v_in, params) -> (out, m_out, v_out)`` defaults to the
    libfedagg kernel (:func:`fedn_amd.ops.fedopt_step`); tests inject a reference step.
    """

    def __init__(self, P, group=None, step_fn=None, align=ALIGN_ELEMS):
        self._avg = ShardedFedAvg(P, group=group, fold_fn=lambda *a: None, align=align)
        self.rank, self.world, self.lo, self.hi = self._avg.rank, self._avg.world, self._avg.lo, self._avg.hi
        self.step_fn = step_fn or _kernel_fedopt_step
        self.m = None
        self.v = None

    def local(self, flat):
        return flat[self.lo:self.hi]

    def step(self, old_local, updates_local, n, N, params):
        out, self.m, self.v = self.step_fn(old_local, updates_local, n, N, self.m, self.v, params)
        return out

    def allgather(self, out_local):
        return self._avg.allgather(out_local)

    def gather_to_host(self, out_local, dst=0):
        return self._avg.gather_to_host(out_local, dst)


def _kernel_fedopt_step(old, updates, n, N, m_in, v_in, params):
    from .ops import fedopt_dtypes, fedopt_step
    pg_dt, m_dt = fedopt_dtypes(updates[0].dtype, old.dtype, None if m_in is None else m_in.dtype)
    dev, P = old.device, old.numel()
    m_out = m_in if (m_in is not None and m_in.dtype == m_dt) else torch.empty(P, dtype=m_dt, device=dev)
    v_out = v_in if v_in is not None else torch.empty(P, dtype=torch.float64, device=dev)
    out = torch.empty(P, dtype=torch.float64, device=dev)
    pg = torch.empty(P, dtype=pg_dt, device=dev) if len(updates) > 64 else None
    fedopt_step(old, updates, n, N, first=True, final=True, pg=pg, m_in=m_in, m_out=m_out, v_in=v_in, v_out=v_out,
                out=out, **params)
    return out, m_out, v_out


class CyclicShardedFedAvg:
    """FedAvg sharded block-cyclically, with the all-gather chunked and overlapped with the
    fold ("chunk it and overlap it with the reduce of the next chunk").

    The flat model is cut into chunks of C elements; chunk j belongs to rank j mod world, so
    round i of the reduce covers the W consecutive chunks [i·W·C, (i+1)·W·C) — one per rank.
    Rank r's local buffers hold its chunks back to back (round i at [i·C, (i+1)·C)). Then
    ``all_gather_into_tensor(full[i·W·C : (i+1)·W·C], agg_local[i·C : (i+1)·C])`` writes
    round i straight into natural model order — no reassembly pass — and it runs on a
    communication stream while round i+1 is folded on the compute stream. Every element is
    folded by the same kernel and client table: bit-identical to one GPU.
    """

    def __init__(self, P, chunk=1 << 22, group=None, fold_fn=None, align=ALIGN_ELEMS, collective_at_world1=False):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.P = P
        # issue the all-gathers even at world size 1 (a one-GPU rehearsal of the RCCL calls)
        self.collective = self.world > 1 or (collective_at_world1 and dist.is_initialized())
        self.C = max(align, -(-chunk // align) * align)
        nchunks = max(1, -(-P // self.C))
        self.rounds = -(-nchunks // self.world)
        self.local_len = self.rounds * self.C
        self.full_len = self.rounds * self.world * self.C
        if fold_fn is None:
            from .ops import fedavg_fold as fold_fn
        self.fold_fn = fold_fn
        self._comm = None

    def owned(self):
        """This rank's chunks as (global_lo, global_hi, local_lo), clipped to [0, P)."""
        out = []
        for i in range(self.rounds):
            g = (i * self.world + self.rank) * self.C
            if g < self.P:
                out.append((g, min(g + self.C, self.P), i * self.C))
        return out

    def local(self, flat):
        """This rank's chunks of a full flat buffer, as a new padded local buffer."""
        loc = torch.zeros(self.local_len, dtype=flat.dtype, device=flat.device)
        for lo, hi, l0 in self.owned():
            loc[l0:l0 + hi - lo].copy_(flat[lo:hi])
        return loc

    def fold_allgather(self, agg_local, updates_local, n, N, init, out=None):
        """Fold every round and gather it as soon as it is folded; returns the full model
        (``full[:P]``; on the host for gloo). ``agg_local`` / ``updates_local``: local_len each."""
        C, W = self.C, self.world
        coll = self.collective
        gloo = coll and dist.get_backend(self.group) == "gloo"
        dev = agg_local.device
        on_gpu = dev.type == "cuda" and not gloo
        if out is None:
            out = torch.empty(self.full_len, dtype=agg_local.dtype, device=dev if not gloo else "cpu")
        if on_gpu and coll and self._comm is None:
            self._comm = torch.cuda.Stream(dev)
        cur = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        for i in range(self.rounds):
            sl = slice(i * C, (i + 1) * C)
            self.fold_fn(agg_local[sl], [u[sl] for u in updates_local], n, N, init)
            dst = out[i * W * C:(i + 1) * W * C]
            if not coll:
                dst.copy_(agg_local[sl], non_blocking=True)
            elif on_gpu:
                ev = torch.cuda.Event()
                ev.record(cur)
                self._comm.wait_event(ev)
                with torch.cuda.stream(self._comm):
                    dist.all_gather_into_tensor(dst, agg_local[sl], group=self.group)
            else:
                src = agg_local[sl].to("cpu")
                dist.all_gather(list(dst.chunk(W)), src, group=self.group)
        if on_gpu and coll:
            cur.wait_stream(self._comm)
        return out[:self.P]
