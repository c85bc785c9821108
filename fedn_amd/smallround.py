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
                       addr(npz.fnpz_gather_wait))
        except (ImportError, AttributeError):
            _native = False
    return _native


def eligible(layout, K_hint=2):
    """Whether a round over ``layout`` can take the one-call path: float16/32/64 tensors only (numpy's
    fold keeps their dtype, so the result block has the arena's layout), and at least two updates
    (the first and one more) fit the arena."""
    zc = _zero_copy_bytes()
    return (all(dt in _FOLDABLE for dt in layout.groups) and max(2, K_hint) * layout.nbytes <= zc
            and bool(_entry_points()))


class SmallSession:
    """The per-(device, layout) resources a session's small rounds reuse (module docstring)."""

    def __init__(self, device, layout):
        fp, self._fold, gstart, self._wait = _entry_points()
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

    def round(self, first, device):
        """A SmallRound for ``first`` on ``device``, or None (not a list of arrays, not eligible)."""
        if type(first) is not list or not first:
            return None
        last = self._last
        if last is not None and last.device == device and last.cap * last.stride <= _zero_copy_bytes():
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
        if not eligible(layout):
            return None
        if s is None or s.cap * s.stride > _zero_copy_bytes():
            s = SmallSession(device, layout)
            self._by_key[key] = s
            while len(self._by_key) > self.keep:
                self._by_key.pop(next(iter(self._by_key)))
        self._last = s
        return SmallRound.start(s, first)
