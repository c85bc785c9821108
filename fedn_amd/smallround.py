"""configs[0]'s rounds: a small model's FedAvg round in as few host steps as the GPU allows.

FEDn's own example (examples/mnist-pytorch: 52,650 fp32 parameters, two clients) folds each round
with ``helper.increment_average`` in ~27 µs of numpy inside a ~47 µs loop (fedavg.py:45-83,
numpyhelper.py:32). Through the general pipeline (staging.FedAvgPipeline) the same round built a
pipeline object, packed the updates, mapped a fresh pinned result block, built ctypes argument
arrays and unpacked the result — ~38 µs of Python above the GPU's own floor.

Here an aggregator keeps, per (device, layout), a ``SmallSession``: one pinned arena the updates are
packed into, the native admission plan, the fold plan, a dedicated stream and a pool of pinned
result blocks. A round then costs, per update, one native admission call (exact layout test + the
pack queued to the gather thread: ``_fastpack.admit``) and, at its end, ONE native call
(``_fastpack.fold_host``: wait for the packs, ``fa_fedavg_fold_host`` — the fold reading the arena
and writing the result block in pinned host memory through their device mappings — and the stream
wait) plus one native call building the model's arrays as views of the result block.

Same observable behaviour as the general path (fedavg.py:47-83): FIFO order, ``total_examples``
before the fold, the first update aliased when it is the only one, and the fold is
``fa_fedavg_fold``'s kernel and client table, so the same bits. An update that is not exactly the
first one's layout (dtype, shape, contiguity), one too many for the arena, or a fold that fails
hands the round to the general pipeline, which replays the admitted updates in order and goes on
(``SmallRound.general``): nothing has been launched or deleted before the round's end.
"""
import ctypes
import sys
import time

import numpy as np
import torch

from . import _abi, ops
from .layout import PACK_THREADS, Layout

# a round's updates, packed, at most staging.ZERO_COPY_BYTES (read at each round: one knob for both
# zero-copy forms, FEDN_AMD_ZERO_COPY_BYTES; 0 turns them off) and 64 of them (one launch) go the
# one-call way


def _zero_copy_bytes():
    from . import staging
    return staging.ZERO_COPY_BYTES
_FOLDABLE = {np.dtype(np.float32): _abi.FA_F32, np.dtype(np.float64): _abi.FA_F64,
             np.dtype(np.float16): _abi.FA_F16}   # dtypes whose fold result is their own dtype (numpy)
_POOL = 4                     # pinned result blocks kept per session (a block a caller still holds is skipped)

_native = None


def _entry_points():
    """(_fastpack module, fa_fedavg_fold_host address, fnpz_gather_start address, fnpz_gather_wait
    address), or False if an extension is not built (the general path is then taken)."""
    global _native
    if _native is None:
        try:
            from . import _fastpack, codec
            lib, npz = _abi.load(), codec.load_lib()
            if not hasattr(_fastpack, "fold_host"):
                raise ImportError("stale _fastpack")
            addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
            _native = (_fastpack, addr(lib.fa_fedavg_fold_host), addr(npz.fnpz_gather_start),
                       addr(npz.fnpz_gather_wait), addr(lib.fa_fedopt_step_host))
        except (ImportError, AttributeError):
            _native = False
    return _native


def eligible(layout, K_hint=2):
    """Whether a round over ``layout`` can take the one-call path: float16/32/64 tensors only (numpy's
    fold keeps their dtype, so the result block has the arena's layout), and at least two updates
    (the first and one more) fit the arena (a layout is never 0 bytes: groups are 256-B aligned)."""
    zc = _zero_copy_bytes()
    return (all(dt in _FOLDABLE for dt in layout.groups) and max(2, K_hint) * layout.nbytes <= zc
            and bool(_entry_points()))


class SmallSession:
    """The per-(device, layout) resources a session's small rounds reuse (module docstring)."""

    def __init__(self, device, layout):
        fp, self._fold, gstart, self._wait, _ = _entry_points()
        self._fp = fp
        self.device = torch.device(device)
        self.layout = layout
        nb = layout.nbytes
        self.stride = nb
        self.cap = max(2, min(64, _zero_copy_bytes() // nb))
        self.arena = torch.empty(self.cap * nb, dtype=torch.uint8, pin_memory=True)
        self.arena_ptr = self.arena.data_ptr()
        self.window = (self.arena_ptr, self.cap * nb)
        offs = {i: off for i, off, _ in layout.pack_plan}
        self.plan = fp.plan([(tuple(sh), np.dtype(dt), offs.get(i, 0))
                             for i, (sh, dt) in enumerate(zip(layout.shapes, layout.dtypes))])
        self.fold_plan = fp.fold_plan([(_FOLDABLE[dt], _FOLDABLE[dt], layout.group_byte_offset[dt],
                                        layout.group_elems[dt]) for dt in layout.groups])
        self._gstart = gstart
        with torch.cuda.device(self.device):
            self.stream = torch.cuda.Stream(self.device)   # the fold touches host memory only: no ordering
        self.stream_ptr = self.stream.cuda_stream          # with torch's streams is needed
        self.blocks = []                                   # [(uint8 numpy block, torch tensor)]

    def admit(self, arrays, slot):
        """Queue the pack of ``arrays`` into arena slot ``slot``: ticket (> 0), 0 (nothing to copy) or
        -1 (not exactly this layout: nothing done)."""
        t = self._fp.admit(self.plan, arrays, self.arena_ptr + slot * self.stride, self._gstart, PACK_THREADS,
                           self.window[0], self.window[1])
        if t == -2:
            from . import codec
            why = codec.load_lib().fnpz_last_error().decode(errors="replace")
            raise codec.CodecError(f"fnpz_gather_start: {why}")
        return t

    def wait(self, ticket):
        if ticket and ticket > 0:
            from . import codec
            codec.gather_wait(ticket)

    def result_block(self):
        """A pinned block for the round's model: a pooled one no caller holds any more (the arrays a
        round returned are views of their block and keep it referenced), else a new one."""
        for ent in self.blocks:
            if sys.getrefcount(ent[0]) == 2:   # the pool's entry and this call's argument only
                return ent[0]
        t = torch.empty(self.layout.nbytes, dtype=torch.uint8, pin_memory=True)
        ent = (t.numpy(), t)
        if len(self.blocks) < _POOL:
            self.blocks.append(ent)
        return ent[0]

    def fold(self, block, K, ns, Ns, ticket):
        """Wait for the packs, fold arena slots 0..K-1 into ``block`` (pinned) and wait: one call."""
        fp, plan, fold, wait, arena, stride, stream = (self._fp, self.fold_plan, self._fold, self._wait,
                                                       self.arena_ptr, self.stride, self.stream_ptr)
        ops.fedavg_fold_host(lambda n, N: fp.fold_host(plan, fold, wait, ticket or 0, arena, stride, K,
                                                       block.ctypes.data, n, N, stream), ns, Ns)

    def views(self, block):
        return self._fp.views(self.plan, block)


class SmallRound:
    """One FedAvg round on a SmallSession: the pipeline interface the aggregator uses (add, result,
    timings, quiesce, release), with nothing launched before ``result``."""

    def __init__(self, session, first):
        self.s = session
        self.first = first
        self.held = []             # (arrays, n, N, tag) of the updates after the first, in FIFO order
        self.ns, self.Ns = [0.0], [1.0]
        self.ticket = None
        self.time_pack = 0.0
        self.time_kernel = 0.0

    @classmethod
    def start(cls, session, first):
        """The round if ``first`` is exactly the session's layout (its pack queued), else None."""
        tic = time.perf_counter()
        t = session.admit(first, 0)
        if t < 0:
            return None
        r = cls(session, first)
        r.ticket = t or None
        r.time_pack = time.perf_counter() - tic
        return r

    def add(self, arrays, n, N, tag=None):
        """Admit one more update; False (nothing done) if it is not exactly the layout or the arena is
        full — the caller then hands the round to the general pipeline (``general``)."""
        k = len(self.held) + 1
        if k >= self.s.cap or type(arrays) is not list:
            return False
        tic = time.perf_counter()
        t = self.s.admit(arrays, k)
        if t < 0:
            return False
        if t:
            self.ticket = t
        self.held.append((arrays, n, N, tag))
        self.ns.append(n)
        self.Ns.append(N)
        self.time_pack += time.perf_counter() - tic
        return True

    def quiesce(self):
        """The packs still queued to the gather thread have finished (they read the updates and write
        the arena, which the next round reuses)."""
        if self.ticket is not None:
            self.s.wait(self.ticket)
            self.ticket = None

    def general(self, make_pipeline):
        """The round handed to the general pipeline: ``make_pipeline(first)`` and the admitted updates
        added in order (same n, N and tags), as if they had gone that way from the start."""
        self.quiesce()
        pipe = make_pipeline(self.first)
        try:
            for arrays, n, N, tag in self.held:
                pipe.add(arrays, n, N, tag=tag)
        except BaseException:
            if hasattr(pipe, "quiesce"):        # its packs in flight end before the arrays can go
                pipe.quiesce()
            raise
        return pipe

    def result(self):
        """The model: the first update itself when nothing was folded into it (fedavg.py:65-66), else
        the fold of every admitted update in one native call, as views of a pinned block. Raises
        FedAggError (nothing changed, the arena intact) if the launch fails: the caller goes general."""
        if not self.held:
            self.quiesce()
            return self.first
        block = self.s.result_block()
        tic = time.perf_counter()
        ticket, self.ticket = self.ticket, None
        try:
            self.s.fold(block, len(self.ns), self.ns, self.Ns, ticket)
        except BaseException:
            self.s.wait(ticket)
            raise
        self.time_kernel = time.perf_counter() - tic
        return self.s.views(block)

    def take_skipped(self):
        return []

    def unsettled(self):
        return 0

    def timings(self):
        """``data`` keys as the general pipeline reports them: no H2D / D2H copies here; the kernel
        time is the one call's wall time (launch, fold over PCIe, wait)."""
        return {"time_h2d": 0.0, "time_kernel": self.time_kernel, "time_pack": self.time_pack, "time_d2h": 0.0}

    def release(self):
        self.quiesce()


class SmallSessions:
    """An aggregator's SmallSession per (device, layout): the last one used is tried first, so a
    session's rounds find theirs with one admission call and no layout lookup."""

    def __init__(self, keep=2):
        self.keep = keep
        self._by_key = {}
        self._last = None

    def round(self, first, device, k_hint=1):
        """A SmallRound for ``first`` on ``device``, or None (not a list of arrays, not eligible, or
        ``k_hint`` — the round's update count as far as the queue shows it — more than the arena holds:
        those rounds go the general way from the start instead of replaying into it part-way)."""
        if type(first) is not list or not first:
            return None
        last = self._last
        if (last is not None and last.device == device and last.cap * last.stride <= _zero_copy_bytes()
                and k_hint <= last.cap):
            r = SmallRound.start(last, first)
            if r is not None:
                return r
        try:
            layout = Layout.of(first)
        except Exception:  # noqa: BLE001 — not an array list: the general path raises numpy's error
            return None
        key = (str(device), id(layout))
        s = self._by_key.get(key)
        if s is not None and s.layout is not layout:   # a recycled id (Layout.of's cache was cleared)
            s = None
        if not eligible(layout, k_hint) or k_hint > 64:
            return None
        if s is None or s.cap * s.stride > _zero_copy_bytes():
            s = SmallSession(device, layout)
            self._by_key[key] = s
            while len(self._by_key) > self.keep:
                self._by_key.pop(next(iter(self._by_key)))
        self._last = s
        return SmallRound.start(s, first)


# ---- FedOpt (fedopt.py:74-121 + 151-258): the same one-call round ---------------------------------

class SmallFedOptSession:
    """The per-(device, update layout, global-model layout) resources of a FedOpt session's small rounds:
    a pinned block for the global model (packed on the round's first update, fedopt.py:89-90), the
    updates' arena, admission plans for both, pinned result blocks per state dtype, and two pairs of HBM
    buffers per (m, v) dtype the server step writes in turn — the pair the session's state does not
    hold, so a step that fails leaves the state as the last round left it (fedopt.py:36-38).

    Unlike FedAvg's one-call fold (host memory only), the step reads and writes HBM that torch's
    streams also use — m / v from a general round or a regroup copy, and the pair buffers, which the
    caching allocator hands out in the order of the device's current stream (a block freed there may
    still have queued writes from its previous owner) — so it runs on that current stream, ordered
    after them, never on a private one."""

    def __init__(self, device, layout, old_layout):
        fp, _, gstart, self._wait, self._fn = _entry_points()
        self._fp, self._gstart = fp, gstart
        self.device = torch.device(device)
        self.dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.layout, self.old_layout = layout, old_layout
        (self.dt,) = layout.groups
        (self.odt,) = old_layout.groups
        self.P = layout.group_elems[self.dt]
        nb = layout.nbytes
        self.stride = nb
        self.cap = max(1, min(64, _zero_copy_bytes() // nb))
        self.arena = torch.empty(self.cap * nb, dtype=torch.uint8, pin_memory=True)
        self.arena_ptr = self.arena.data_ptr()
        self.old = torch.empty(old_layout.nbytes, dtype=torch.uint8, pin_memory=True)
        self.old_ptr = self.old.data_ptr()
        self.plan = self._plan(layout, self.dt)
        self.old_plan = self._plan(old_layout, self.odt)
        self.out_plans = {}                  # state dtype -> views plan of the new model
        self.blocks = {}                     # state dtype -> [(uint8 numpy block, torch tensor)]
        self.pairs = {}                      # (m dtype, state dtype) -> [(m, v) HBM buffers]

    def _plan(self, layout, dt, out_dt=None):
        """Admission / views plan: each tensor at its element offset in the (single) group."""
        out_dt = np.dtype(out_dt if out_dt is not None else dt)
        offs = dict(layout.members[dt])
        return self._fp.plan([(tuple(sh), out_dt, offs[i] * out_dt.itemsize) for i, sh in enumerate(layout.shapes)])

    def admit(self, arrays, dst_ptr, window, plan):
        t = self._fp.admit(plan, arrays, dst_ptr, self._gstart, PACK_THREADS, window[0], window[1])
        if t == -2:
            from . import codec
            raise codec.CodecError(f"fnpz_gather_start: {codec.load_lib().fnpz_last_error().decode(errors='replace')}")
        return t

    def admit_old(self, arrays):
        return self.admit(arrays, self.old_ptr, (self.old_ptr, self.old_layout.nbytes), self.old_plan)

    def admit_update(self, arrays, slot):
        return self.admit(arrays, self.arena_ptr + slot * self.stride, (self.arena_ptr, self.cap * self.stride), self.plan)

    def wait(self, ticket):
        if ticket and ticket > 0:
            from . import codec
            codec.gather_wait(ticket)

    def result_block(self, sdt):
        pool = self.blocks.setdefault(sdt, [])
        for ent in pool:
            if sys.getrefcount(ent[0]) == 2:     # no array of an earlier round views it any more
                return ent[0]
        t = torch.empty(self.P * ops.numpy_dtype(sdt).itemsize, dtype=torch.uint8, pin_memory=True)
        ent = (t.numpy(), t)
        if len(pool) < _POOL:
            pool.append(ent)
        return ent[0]

    def views(self, block, sdt):
        plan = self.out_plans.get(sdt)
        if plan is None:
            plan = self.out_plans[sdt] = self._plan(self.layout, self.dt, ops.numpy_dtype(sdt))
        return self._fp.views(plan, block)

    def state_pair(self, m_dt, sdt, m_in, v_in):
        """HBM buffers for the new m / v: a pair whose memory the state does not hold (compared by
        address: the state may hold a view of a pair buffer rather than the buffer object)."""
        pairs = self.pairs.setdefault((m_dt, sdt), [])
        held = {t.data_ptr() for t in (m_in, v_in) if t is not None and t.numel()}
        for m, v in pairs:
            if m.data_ptr() not in held and v.data_ptr() not in held:
                return m, v
        with torch.cuda.device(self.device):
            pair = (torch.empty(self.P, dtype=m_dt, device=self.device), torch.empty(self.P, dtype=sdt, device=self.device))
        pairs.append(pair)
        return pair


class SmallFedOptRound:
    """One FedOpt round on a SmallFedOptSession: add() admits each update, server_step() is one native
    call (pack wait + fa_fedopt_step_host, FIRST | FINAL: the pseudo-gradient in registers, then Adam /
    Yogi / AdaGrad). Anything else — another layout, a full arena, a failed launch, a state in another
    form — hands the round to the general pipeline (``make_pipeline(old, first)``), replaying the
    admitted updates in FIFO order: nothing was launched or deleted before."""

    def __init__(self, session, old_arrays, first_arrays, make_pipeline):
        self.s = session
        self.old_arrays, self.first_arrays = old_arrays, first_arrays
        self.make_pipeline = make_pipeline
        self.held = []
        self.ns, self.Ns = [], []
        self.ticket = None
        self.time_pack = 0.0
        self.time_kernel = 0.0
        self.fallback = None       # the general pipeline the step was handed to (it reports from then on)

    @classmethod
    def start(cls, session, old_arrays, first_arrays, make_pipeline):
        """The round if the global model packs into the session's layout (queued), else None."""
        tic = time.perf_counter()
        t = session.admit_old(old_arrays)
        if t < 0:
            return None
        r = cls(session, old_arrays, first_arrays, make_pipeline)
        r.ticket = t or None
        r.time_pack = time.perf_counter() - tic
        return r

    def add(self, arrays, n, N, tag=None):
        k = len(self.held)
        if k >= self.s.cap or type(arrays) is not list:
            return False
        tic = time.perf_counter()
        t = self.s.admit_update(arrays, k)
        if t < 0:
            return False
        if t:
            self.ticket = t
        self.held.append((arrays, n, N, tag))
        self.ns.append(n)
        self.Ns.append(N)
        self.time_pack += time.perf_counter() - tic
        return True

    def quiesce(self):
        if self.ticket is not None:
            self.s.wait(self.ticket)
            self.ticket = None
        if self.fallback is not None and hasattr(self.fallback, "quiesce"):
            self.fallback.quiesce()

    def general(self):
        """The round handed to the general pipeline, the admitted updates added in order."""
        self.quiesce()
        pipe = self.make_pipeline(self.old_arrays, self.first_arrays)
        try:
            for arrays, n, N, tag in self.held:
                pipe.add(arrays, n, N, tag=tag)
        except BaseException:
            if hasattr(pipe, "quiesce"):
                pipe.quiesce()
            raise
        return pipe

    def server_step(self, state, params):
        """The new model (fedopt.py:108-118): one native call; a state that is not in this layout's
        fused form, or a failed launch (state untouched), goes the general way."""
        opt = params["serveropt"]
        if opt not in ops._OPTS:
            raise ValueError(f"Unsupported server optimizer: {opt}")
        s = self.s
        sig = s.layout.signature()
        if not state.regroup(s.layout, sig, s.device):
            self.fallback = self.general()
            return self.fallback.server_step(state, params)
        dt = s.dt
        old_t = ops.torch_dtype(s.odt)
        m_in = state.m[dt] if state.m is not None else None
        v_in = state.v[dt] if state.v is not None else None
        from .staging import state_dtypes
        m_dt, sdt = state_dtypes(state, dt, old_t, m_in)
        m_out, v_out = s.state_pair(m_dt, sdt, m_in, v_in)
        block = s.result_block(sdt)
        ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        fa = ops.fa_dtype
        st = (ptr(m_in), _abi.FA_NONE if m_in is None else fa(m_in), ptr(m_out), fa(m_out), ptr(v_in),
              _abi.FA_F64 if v_in is None else fa(v_in), ptr(v_out), fa(sdt))
        ticket, self.ticket = self.ticket, None
        fp, fn, wait, old, arena, stride, K, P = s._fp, s._fn, s._wait, s.old_ptr, s.arena_ptr, s.stride, len(self.ns), s.P
        stream = torch._C._cuda_getCurrentRawStream(s.dev_index)      # the current stream: see SmallFedOptSession
        upd_fa, old_fa, out = fa(ops.torch_dtype(dt)), fa(old_t), block.ctypes.data
        args = (ops._OPTS[opt], float(params["learning_rate"]), float(params["beta1"]), float(params["beta2"]),
                float(params["tau"]))
        tic = time.perf_counter()
        try:
            ops.fedopt_step_host(lambda n, N: fp.fedopt_host(fn, wait, ticket or 0, old, arena, stride, K, upd_fa,
                                                              old_fa, P, out, n, N, stream, st, *args),
                                 self.ns, self.Ns, first=True, final=True)
        except ops.FedAggError:
            s.wait(ticket)                        # nothing of the state was replaced: the general way
            self.fallback = self.general()
            return self.fallback.server_step(state, params)
        except BaseException:
            s.wait(ticket)
            raise
        self.time_kernel = time.perf_counter() - tic
        state.m, state.v, state.signature, state.layout = {dt: m_out}, {dt: v_out}, sig, s.layout
        return s.views(block, sdt)

    def take_skipped(self):
        return self.fallback.take_skipped() if self.fallback is not None else []

    def unsettled(self):
        return self.fallback.unsettled() if self.fallback is not None else 0

    def timings(self):
        if self.fallback is not None:
            return self.fallback.timings()
        return {"time_h2d": 0.0, "time_kernel": self.time_kernel, "time_pack": self.time_pack, "time_d2h": 0.0}

    def release(self):
        self.quiesce()
        if self.fallback is not None and hasattr(self.fallback, "release"):
            self.fallback.release()


def fedopt_eligible(layout, old_layout):
    """One float16/32/64 group in both the updates and the global model, with the same shapes, a pair the
    fused kernel instantiates, and at least one update fitting the arena."""
    from .staging import fused_fedopt_pair
    if len(layout.groups) != 1 or len(old_layout.groups) != 1 or layout.shapes != old_layout.shapes:
        return False
    dt, odt = layout.groups[0], old_layout.groups[0]
    return (dt in _FOLDABLE and odt in _FOLDABLE and fused_fedopt_pair(ops.torch_dtype(dt), ops.torch_dtype(odt))
            and layout.nbytes <= _zero_copy_bytes() and bool(_entry_points()))


class SmallFedOptSessions:
    """A FedOpt aggregator's SmallFedOptSession per (device, update layout, global-model layout)."""

    def __init__(self, keep=2):
        self.keep = keep
        self._by_key = {}
        self._last = None

    def round(self, old_arrays, first, device, make_pipeline, k_hint=1):
        """A SmallFedOptRound, or None (see SmallSessions.round; ``k_hint``: the round's update count as
        far as the queue shows it)."""
        if type(first) is not list or not first or type(old_arrays) is not list:
            return None
        last = self._last
        if (last is not None and last.device == device and last.cap * last.stride <= _zero_copy_bytes()
                and k_hint <= last.cap and last.layout is _layout_of(first)):
            r = SmallFedOptRound.start(last, old_arrays, first, make_pipeline)
            if r is not None:
                return r
        try:
            layout, old_layout = Layout.of(first), Layout.of(old_arrays)
        except Exception:  # noqa: BLE001
            return None
        if not fedopt_eligible(layout, old_layout) or k_hint > 64 or k_hint * layout.nbytes > _zero_copy_bytes():
            return None
        key = (str(device), id(layout), id(old_layout))
        s = self._by_key.get(key)
        if s is not None and (s.layout is not layout or s.old_layout is not old_layout
                              or s.cap * s.stride > _zero_copy_bytes()):
            s = None
        if s is None:
            s = SmallFedOptSession(device, layout, old_layout)
            self._by_key[key] = s
            while len(self._by_key) > self.keep:
                self._by_key.pop(next(iter(self._by_key)))
        self._last = s
        return SmallFedOptRound.start(s, old_arrays, first, make_pipeline)


def _layout_of(arrays):
    try:
        return Layout.of(arrays)
    except Exception:  # noqa: BLE001
        return None
