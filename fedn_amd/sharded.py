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

    def gather_to_host(self, agg_local, dst=0, gather=None):
        """The whole model as ONE host tensor on rank ``dst`` (None elsewhere): every rank D2H's its
        slice over its own PCIe link straight into the node's shared host model (:class:`HostGather`,
        made on first use and kept for later rounds; pass ``gather`` to share one). FEDn serialises
        the model on the host (roundhandler.py:465-468), so no device collective is needed."""
        if self.world == 1:
            return agg_local.to("cpu")
        if gather is None:
            gather = self._host_gather = _cached_gather(self, agg_local.dtype, dst, self.bounds)
        return gather.gather(agg_local)


def _agree(failed, group=None, device=None):
    """Whether ANY rank of ``group`` failed (``failed`` is this rank's verdict): a one-element MAX
    all-reduce every rank takes part in — where a barrier would stand — so a step that fails on one
    rank only fails on every rank at the same point, and no rank is left waiting in a collective the
    failed one never reaches. On device ``device`` under RCCL, on the CPU under gloo."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return bool(failed)
    dev = device if (device is not None and dist.get_backend(group) == "nccl") else "cpu"
    flag = torch.tensor([1 if failed else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    return bool(int(flag[0]))


def _cached_gather(owner, dtype, dst, bounds):
    """``owner``'s HostGather for (dst, dtype) — made on first use, replaced (and the old one closed)
    when a later gather asks for another destination rank or dtype. Every rank of the group makes the
    same calls, so they replace it together."""
    hg = getattr(owner, "_host_gather", None)
    if hg is not None and hg.dst == dst and hg.dtype == dtype and hg.P == owner.P:
        return hg
    if hg is not None:
        hg.close()
    return HostGather(owner.P, dtype, bounds, group=owner.group, dst=dst)


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

    def gather_to_host(self, out_local, dst=0, gather=None):
        return self._avg.gather_to_host(out_local, dst, gather)


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
        # the libfedagg fold by default: then each round's launch takes its client table as device
        # addresses (``fold_round``), not as 64 tensor slices per round — at N = 8 a round's fold is
        # ~0.15 ms of GPU time, less than the ~0.2 ms of Python the slices and checks cost
        self._kernel = fold_fn is None
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

    def gather_to_host(self, agg_local, dst=0, gather=None):
        """The folded model as ONE host tensor on rank ``dst`` (None elsewhere), without a device
        collective: every rank D2H's its chunks straight into the node's shared host model
        (:class:`HostGather`, kept for later rounds) — FEDn's consumer (roundhandler.py:465-468)."""
        if gather is None:
            gather = self._host_gather = _cached_gather(self, agg_local.dtype, dst, None)
        return gather.gather(agg_local, self.owned())

    def round_folder(self, agg_local, updates_local, n, N, init, stream=None):
        """``fold(i)`` folding round i (the local chunk [i·C, (i+1)·C)) of every update into
        ``agg_local``: one launch over the updates' device addresses with the default kernel on device
        buffers of one dtype (the addresses and scalars prepared once per call), else ``fold_fn`` on
        slices."""
        C = self.C
        if (self._kernel and agg_local.is_cuda and updates_local
                and all(u.is_cuda and u.device == agg_local.device and u.dtype == updates_local[0].dtype
                        and u.is_contiguous() and u.numel() >= self.local_len for u in updates_local)
                and agg_local.is_contiguous() and agg_local.numel() >= self.local_len):
            from . import ops
            bases = [u.data_ptr() for u in updates_local]
            es = updates_local[0].element_size()
            udt = updates_local[0].dtype
            if stream is None:
                stream = torch.cuda.current_stream(agg_local.device)

            def fold(i):
                off = i * C * es
                ops.fedavg_fold_ptrs(agg_local[i * C:(i + 1) * C], [b + off for b in bases], udt, n, N, init=init,
                                     stream=stream)
            return fold

        def fold(i):
            sl = slice(i * C, (i + 1) * C)
            self.fold_fn(agg_local[sl], [u[sl] for u in updates_local], n, N, init)
        return fold

    def _fusable(self, agg_local, updates_local, out):
        """The fused fold + push applies: the default kernel, fp32 updates, aggregate and model on
        one device, contiguous buffers of the geometry's sizes."""
        return bool(self._kernel and out.dtype == torch.float32 and out.is_cuda and updates_local
                    and all(t.dtype == torch.float32 and t.device == out.device and t.is_contiguous()
                            and t.numel() >= self.local_len for t in [agg_local, *updates_local])
                    and out.numel() >= self.full_len)

    def fold_allgather(self, agg_local, updates_local, n, N, init, out=None, p2p=None):
        """Fold every round and gather it as soon as it is folded; returns the full model
        (``full[:P]``; on the host for gloo). ``agg_local`` / ``updates_local``: local_len each.

        ``p2p``: a :class:`P2PAllGather` over this geometry's ``full_len`` buffer — round i is then
        pushed by direct copies into every peer's buffer (one copy stream per peer) instead of an RCCL
        all-gather, and the result is a view of ``p2p``'s buffer: overwritten by the NEXT call (the
        call fences on entry — every rank done with the previous result — and on exit — every
        rank's pushes landed), or by the call after next with a double-buffered ``p2p`` (one fence
        per call)."""
        C, W = self.C, self.world
        if p2p is not None:
            if p2p.full.numel() < self.full_len:
                raise ValueError(f"p2p buffer has {p2p.full.numel()} elements, this geometry needs {self.full_len}")
            dev = agg_local.device
            cur = torch.cuda.current_stream(dev)
            p2p.begin()
            out = p2p.full
            if p2p.engine == "fused" and self._fusable(agg_local, updates_local, out):
                from . import ops
                bases = [u.data_ptr() for u in updates_local]
                for i in range(self.rounds):
                    at = (i * W + self.rank) * C
                    # the running aggregate is agg_local (read back when init is False, and what a later
                    # gather_to_host(agg_local) copies); this rank's copy in ``out`` is one more store
                    # destination beside the peers'
                    p2p.count_release(cur, ops.fedavg_fold_push(
                        agg_local.data_ptr() + i * C * 4, [b + i * C * 4 for b in bases], n, N, C, init,
                        p2p.peer_ptrs(at) + [out.data_ptr() + at * 4], cur, dev, release_rec=p2p.release_rec(cur)))
                p2p.fence()
                return out[:self.P]
            fold = self.round_folder(agg_local, updates_local, n, N, init, cur)
            for i in range(self.rounds):
                sl = slice(i * C, (i + 1) * C)
                fold(i)
                at = (i * W + self.rank) * C
                ev = torch.cuda.Event()
                ev.record(cur)
                if not p2p.push(at, agg_local[sl], ev, local=True):
                    out[at:at + C].copy_(agg_local[sl], non_blocking=True)
            p2p.fence()
            return out[:self.P]
        coll = self.collective
        gloo = coll and dist.get_backend(self.group) == "gloo"
        dev = agg_local.device
        on_gpu = dev.type == "cuda" and not gloo
        if out is None:
            out = torch.empty(self.full_len, dtype=agg_local.dtype, device=dev if not gloo else "cpu")
        if on_gpu and coll and self._comm is None:
            self._comm = torch.cuda.Stream(dev)
        cur = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        fold = self.round_folder(agg_local, updates_local, n, N, init, cur)
        for i in range(self.rounds):
            sl = slice(i * C, (i + 1) * C)
            fold(i)
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


class P2PAllGather:
    """Direct peer-to-peer all-gather over xGMI ("prefer ... direct (all 7
    links)"), the alternative to RCCL's ring / multi-channel all-gather for
    :meth:`CyclicShardedFedAvg.fold_allgather`.

    Every rank owns a model buffer ``full`` of the same length for the session. The ranks exchange
    IPC handles of those buffers ONCE (``fa_ipc_get_handle`` / ``fa_ipc_open``, handles passed with
    ``all_gather_object``), so each rank holds a device pointer into every peer's buffer. A rank then
    pushes each piece it folds into all peers with one DMA copy per peer (``fa_copy_async``), each
    peer on its own stream, i.e. over its own link, all links busy at once and no rank forwarding
    another's data (a ring moves every byte W - 1 hops over one link per rank).

    ``fence()`` orders the ranks: every rank's earlier pushes have completed before any rank's
    stream runs past it. Under RCCL it is a one-element all-reduce issued after the copy streams
    (device-side, the host does not block); under gloo (CPU tests, one-GPU rehearsals) a device
    synchronize and a barrier.

    ``engine``: how a piece reaches the peers — ``"dma"``, one ``hipMemcpyAsync`` per peer on that
    peer's stream (the DMA engines; each copy reads the piece from local HBM again), or
    ``"kernel"``, ONE ``fa_push`` launch on a push stream that reads the piece once and stores it
    into every peer's buffer (the CUs drive all links at once; it shares the chip with the next
    round's fold). Which one moves a node's links faster is measured there (``bench.py`` chooses in
    its warm-up); the attribute may be switched between steps. ``"fused"``: no separate push at all —
    ``CyclicShardedFedAvg.fold_allgather`` folds each round with ``fa_fedavg_fold_push``, whose kernel
    stores every result element into this rank's buffer and every peer's as it is produced (fp32;
    other dtypes push with the kernel engine).

    ``spare``: a second buffer of the same size makes the gather double-buffered: the steps
    alternate between the two, so the exit fence of step t (every rank has entered step t, i.e. is
    done with step t − 2's result in the same buffer) also clears that buffer for step t + 1's
    pushes — one fence per step instead of two; a result then stays valid until the step after next.
    """

    ENGINES = ("dma", "kernel", "fused")

    def __init__(self, full, group=None, spare=None, engine="dma", verify="round"):
        from . import ops
        if engine not in self.ENGINES:
            raise ValueError(f"P2PAllGather: engine must be one of {self.ENGINES}")
        if verify not in ("round", "close"):
            raise ValueError("P2PAllGather: verify must be 'round' or 'close'")
        self.engine = engine
        # "round": every fence() reads the release records (one small D2H after the fence; under RCCL
        # the host waits for the round there) and fails that round's exchange on a missed XCD or a
        # release grid that never ran; "close": only close() / check_release() do (bench.py, whose
        # timed steps must not block the host; it reads and reports the records itself)
        self.verify = verify
        self.bufs = [full] if spare is None else [full, spare]
        self.cur = 0
        self.steps = 0
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.device = full.device
        self.esize = full.element_size()
        if spare is not None and (spare.numel() != full.numel() or spare.dtype != full.dtype or
                                  spare.device != full.device):
            raise ValueError("P2PAllGather: the spare buffer must match the first")
        # every rank reaches the handle exchange, and every rank sees every rank's export failure
        # (the same exception everywhere: a caller falls back together, bench.py to the collective)
        try:
            mine = [ops.ipc_handle(b) + (b.numel(), str(b.dtype)) for b in self.bufs]
        except Exception as e:  # noqa: BLE001 — exchanged, then raised on every rank
            mine = f"{type(e).__name__}: {e}"
        objs = [None] * self.world
        if self.world > 1:
            dist.all_gather_object(objs, mine, group=group)
        else:
            objs = [mine]
        bad = [(r, o) for r, o in enumerate(objs) if isinstance(o, str)]
        if bad:
            raise RuntimeError(f"P2PAllGather: rank {bad[0][0]} could not export its buffers ({bad[0][1]})")
        for r, lst in enumerate(objs):
            if len(lst) != len(self.bufs) or any(n != full.numel() or dt != str(full.dtype) for _, _, n, dt in lst):
                raise ValueError(f"P2PAllGather: rank {r} buffers {[(n, dt) for _, _, n, dt in lst]}, this rank's "
                                 f"{len(self.bufs)} x {full.numel()} x {full.dtype}")
        self.peers = {}                            # rank -> [(base, pointer) per buffer]
        err = None
        try:
            for r, lst in enumerate(objs):
                if r != self.rank:
                    self.peers[r] = []
                    for h, o, _, _ in lst:
                        self.peers[r].append(ops.ipc_open(h, o, self.device))
        except Exception as e:  # noqa: BLE001 — agreed on below
            err = e
        # one rank that cannot map a peer fails the transport on every rank
        if _agree(err is not None, group, self.device):
            self.close(fence=False)
            if err is not None:
                raise err
            raise RuntimeError("P2PAllGather: another rank could not map its peers' buffers")
        self.streams = {r: torch.cuda.Stream(self.device) for r in self.peers}
        self.push_stream = torch.cuda.Stream(self.device)       # the "kernel" engine's launches
        self.nccl = dist.is_initialized() and dist.get_backend(group) == "nccl"
        self._flag = torch.zeros(1, dtype=torch.float32, device=self.device) if self.nccl else None
        self._release = {}                          # stream handle -> its release record (kernel engines)
        self._issued = {}                           # stream handle -> release grids launched with it

    def release_rec(self, stream):
        """The release record of ``stream`` (one per stream: a record's reset is ordered by the stream)
        that the kernel engines' release grids fill with the XCDs they ran on (fa_push /
        fa_fedavg_fold_push, include/fedagg.h); :meth:`check_release` reads them."""
        key = stream.cuda_stream
        rec = self._release.get(key)
        if rec is None:
            from . import ops
            with torch.cuda.stream(stream):      # zeroed in the order of the stream that fills it
                rec = self._release[key] = ops.release_record(self.device)
        return rec

    def count_release(self, stream, launched):
        """One release grid was launched on ``stream`` (``launched``: what ops.push /
        ops.fedavg_fold_push returned — counted only after the call succeeded and only when it did
        launch one, so a call that stored nothing or failed its checks leaves the count right)."""
        if launched:
            key = stream.cuda_stream
            self._issued[key] = self._issued.get(key, 0) + 1

    def check_release(self):
        """Synchronise and verify that every release grid of the peer-storing kernels so far covered
        every XCD of the device (each XCD's L2 written back at system scope before the fence).
        Returns the summed record; raises FedAggError on any launch that missed an XCD — the peers
        may then have read stale bytes, so the exchange is not trusted."""
        from . import _abi, ops
        tot = {"launches": 0, "misses": 0, "seen_mask": 0, "expect_mask": 0}
        for rec in self._release.values():
            r = ops.read_release_record(rec)
            tot["launches"] += r["launches"]
            tot["misses"] += r["misses"]
            tot["seen_mask"] |= r["seen_mask"]
            tot["expect_mask"] |= r["expect_mask"]
        tot["xcds_seen"] = bin(tot["seen_mask"]).count("1")
        tot["xcds"] = ops.device_xccs(self.device)
        issued = sum(self._issued.values())
        if tot["launches"] != issued:
            raise _abi.FedAggError(_abi.FA_EHIP, f"P2PAllGather: {tot['launches']} release grids recorded, {issued} "
                                                 f"launched: a release did not run (or its record was reset)")
        if tot["misses"]:
            raise _abi.FedAggError(_abi.FA_EHIP, f"P2PAllGather: {tot['misses']} of {tot['launches']} release grids "
                                                 f"did not cover every XCD (seen {tot['seen_mask']:#x}, device "
                                                 f"{tot['expect_mask']:#x}): peer stores may not have been visible")
        return tot

    @property
    def full(self):
        """The buffer the current step gathers into."""
        return self.bufs[self.cur]

    def begin(self):
        """Start a step: double-buffered, switch buffers (the last exit fence cleared this one);
        single-buffered, fence (every rank is done with the previous result)."""
        if len(self.bufs) == 2:
            self.cur = self.steps % 2
        elif self.steps:
            self.fence()
        self.steps += 1

    def push(self, at, src, after, local=False):
        """Copy device tensor ``src`` to elements [at, at + len(src)) of every peer's current buffer
        once ``after`` (an event on the folding stream) has fired. ``local``: this rank's own buffer
        too, if the engine can do it in the same pass (the kernel engine stores it as one more
        destination); returns whether it did — else the caller copies it (ordered by ``fence``)."""
        from . import ops
        if at < 0 or at + src.numel() > self.full.numel():
            raise ValueError("P2PAllGather.push: piece outside the buffer")
        nbytes = src.numel() * self.esize
        if self.engine in ("kernel", "fused"):
            dsts = [maps[self.cur][1] + at * self.esize for maps in self.peers.values()]
            if local:
                dsts.append(self.full.data_ptr() + at * self.esize)
            if dsts:
                self.push_stream.wait_event(after)
                self.count_release(self.push_stream, ops.push(dsts, src, nbytes, self.push_stream,
                                                              release_rec=self.release_rec(self.push_stream)))
            return local
        for r, st in self.streams.items():
            st.wait_event(after)
            ops.copy_async(self.peers[r][self.cur][1] + at * self.esize, src, nbytes, st)
        return False

    def peer_ptrs(self, at):
        """Device addresses of element ``at`` of every peer's current buffer (the fused engine's
        destinations)."""
        return [maps[self.cur][1] + at * self.esize for maps in self.peers.values()]

    def fence(self, check=None):
        """Order the ranks (see the class doc); ``check`` (default: ``verify == "round"``) then reads
        the release records and raises on a missed XCD or a release grid that did not run."""
        if check is None:
            check = self.verify == "round"
        cur = torch.cuda.current_stream(self.device)
        for st in self.streams.values():
            cur.wait_stream(st)
        cur.wait_stream(self.push_stream)
        if self.world > 1 and dist.is_initialized():
            if self.nccl:
                dist.all_reduce(self._flag, group=self.group)
            else:
                torch.cuda.synchronize(self.device)
                dist.barrier(group=self.group)
        if check and self._release:
            # this round's release records, read after the fence (check_release's D2H is ordered after
            # it on the current stream): a miss fails the round's exchange here, not at close()
            self.check_release()

    def close(self, fence=True, check=True):
        """Unmap the peers' buffers (after a fence: no copy into them is in flight). ``check``: the
        release records are checked first (:meth:`check_release`; raised after the unmapping) — a
        caller that already read them (bench.py reports them in its line) passes False."""
        from . import ops
        err = None
        if fence and (self.peers or self._release):
            self.fence(check=False)             # checked below, raised once the peers are unmapped
            torch.cuda.synchronize(self.device)
            if check:
                try:
                    self.check_release()
                except Exception as e:  # noqa: BLE001 — raised once the peers are unmapped
                    err = e
        for r, maps in list(self.peers.items()):
            for base, _ in maps:
                ops.ipc_close(base, self.device)
        self.peers = {}
        if fence and self.world > 1 and dist.is_initialized():
            dist.barrier(group=self.group)       # no peer unmaps while another still copies
        if err is not None:
            raise err


class HostGather:
    """The node's ONE host copy of a sliced model: every rank D2H's its slice over its own PCIe link
    straight into it (FEDn's consumer of the aggregate is host serialisation, roundhandler.py:465-468;
    SURVEY.md §8(e): "each GPU could also D2H its own slice into one pinned host buffer").

    Rank ``dst`` creates a shared-memory file of the model's size (space reserved up front with
    ``posix_fallocate``: a full /dev/shm raises here, not as a fault later), every rank of the node
    maps it and page-locks its mapping (``fa_host_register``) once, and the file's name is removed as
    soon as all ranks hold it, so nothing outlives the processes. :meth:`gather` then costs one
    D2H per rank plus a barrier, all links at once.
    """

    def __init__(self, P, dtype, bounds, group=None, dst=0, shm_dir="/dev/shm"):
        import os
        import uuid
        self.P, self.dtype, self.bounds, self.group, self.dst = P, dtype, bounds, group, dst
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        esize = torch.empty((), dtype=dtype).element_size()
        nbytes = max(1, P) * esize
        name = [None]
        if self.rank == dst:
            path = os.path.join(shm_dir, f"fedn_amd_model_{os.getpid()}_{uuid.uuid4().hex[:12]}")
            try:
                fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
                try:
                    os.posix_fallocate(fd, 0, nbytes)
                finally:
                    os.close(fd)
                name = [path]
            except OSError as e:
                try:
                    os.unlink(path)
                except OSError:
                    pass
                name = [f"error: {e}"]
        if self.world > 1:
            dist.broadcast_object_list(name, src=dst, group=self.group)
        if name[0].startswith("error: "):
            raise OSError(f"HostGather: shared host model not created ({name[0][7:]})")
        self.host = torch.from_file(name[0], shared=True, size=max(1, P), dtype=dtype)
        if self.world > 1:
            dist.barrier(group=self.group)
        if self.rank == dst:
            os.unlink(name[0])
        self.pinned = False
        self._stream = None

    def _pin(self, device):
        from . import ops
        if not self.pinned:
            with torch.cuda.device(device):
                ops.host_register(self.host)
            self.pinned = True
            self._stream = torch.cuda.Stream(device)

    def gather(self, local, pieces=None):
        """``local``: this rank's part of the model (device or CPU tensor). ``pieces``: where it goes,
        as (global_lo, global_hi, local_lo) triples; default: this rank's contiguous slice of
        ``bounds`` from local[0]. Returns the host model (a shared-memory tensor, valid until rank
        ``dst``'s next gather: every gather starts with a barrier) on rank ``dst``, None elsewhere.
        ``local`` must have the host model's dtype."""
        from . import ops
        if local.dtype != self.dtype:
            raise TypeError(f"HostGather.gather: a {local.dtype} slice into a {self.dtype} host model")
        if pieces is None:
            lo, hi = self.bounds[self.rank]
            pieces = [(lo, hi, 0)] if hi > lo else []
        if self.world > 1:
            # the previous result stays valid until rank dst enters the next gather: no rank writes
            # into the shared model before then
            dist.barrier(group=self.group)
        es = self.host.element_size()
        err = None
        try:
            for lo, hi, l0 in pieces:
                if l0 + hi - lo > local.numel() or hi > self.P:
                    raise ValueError("HostGather.gather: piece outside the local buffer or the model")
            if local.device.type == "cuda" and pieces:
                self._pin(local.device)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(local.device))
                self._stream.wait_event(ev)
                for lo, hi, l0 in pieces:
                    ops.copy_async(self.host.data_ptr() + lo * es, local[l0:], (hi - lo) * es, self._stream)
                self._stream.synchronize()
            else:
                for lo, hi, l0 in pieces:
                    self.host[lo:hi].copy_(local[l0:l0 + hi - lo])
        except Exception as e:  # noqa: BLE001 — agreed on below
            err = e
        # the exit barrier, as an agreement: a rank whose copy failed fails the gather on every rank
        # (the host model is incomplete) instead of leaving the others waiting
        if self.world > 1:
            failed = _agree(err is not None, self.group, local.device if local.device.type == "cuda" else None)
        else:
            failed = err is not None
        if failed:
            if err is not None:
                raise err
            raise RuntimeError("HostGather.gather: another rank's copy into the host model failed")
        return self.host[:self.P] if self.rank == self.dst else None

    def close(self):
        from . import ops
        if self.pinned:
            ops.host_unregister(self.host)
            self.pinned = False
