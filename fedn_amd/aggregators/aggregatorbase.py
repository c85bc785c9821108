"""Aggregator plug-in base and loader — mirror of
fedn/network/combiner/aggregators/aggregatorbase.py:6-62.

``get_aggregator(name, update_handler)`` imports ``fedn_amd.aggregators.<name>`` and
returns ``module.Aggregator(update_handler)``, the same contract FEDn's RoundHandler
uses (roundhandler.py:110-111). To serve an unmodified FEDn combiner, a one-line shim
module at ``fedn/network/combiner/aggregators/<name>.py`` re-exports our Aggregator
(see INTEGRATION.md).
"""
import importlib
import io
import os
import threading
import time
import zipfile
from abc import ABC, abstractmethod
from collections import deque
from concurrent.futures import ThreadPoolExecutor
from concurrent.futures import wait as wait_futures

import numpy as np

AGGREGATOR_PLUGIN_PATH = "fedn_amd.aggregators.{}"
LOAD_AHEAD = int(os.environ.get("FEDN_AMD_LOAD_AHEAD", "8"))
# host bytes of decoded-but-not-yet-folded updates the read-ahead may hold (FEDn holds one)
LOAD_AHEAD_BYTES = int(os.environ.get("FEDN_AMD_LOAD_AHEAD_BYTES", str(4 << 30)))
# loads faster than this (mean over the last round: in-memory handlers, tiny models) are not worth a
# thread hand-off each; the next round then drains its queue on the calling thread
CHEAP_LOAD_S = float(os.environ.get("FEDN_AMD_CHEAP_LOAD_S", "100e-6"))


_pools = {}
_pools_lock = threading.Lock()


def _load_pool(workers):
    """The read-ahead workers: one process-wide pool per size, created once (a pool per round cost
    ~0.2 ms of thread start-up, as much as a whole small-model round's GPU work)."""
    key = (os.getpid(), workers)          # a forked child starts its own (its parent's threads are gone)
    with _pools_lock:
        pool = _pools.get(key)
        if pool is None:
            pool = _pools[key] = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="fedn_amd_load")
        return pool


def _raiser(e):
    def load():
        raise e
    return load


def model_nbytes(model):
    """Host bytes of a decoded update (list of arrays; a staged update counts its packed layout);
    0 if unknown."""
    lay = getattr(model, "layout", None)
    if lay is not None and hasattr(lay, "nbytes"):
        return int(lay.nbytes)
    try:
        return int(sum(np.asarray(a).nbytes for a in model))
    except Exception:  # noqa: BLE001
        return 0


def npz_decoded_bytes(data):
    """Decoded size of an npz payload from its zip central directory (no inflate), else None."""
    try:
        with zipfile.ZipFile(io.BytesIO(data)) as z:
            return sum(i.file_size for i in z.infolist())
    except Exception:  # noqa: BLE001 — not an npz: the size is learned from the first decoded update
        return None


def requeue_front(q, items):
    """Put dequeued ``items`` back at the HEAD of queue ``q`` in their FIFO order, as if they
    had never been taken (``get`` does not count towards ``task_done``, so neither does this)."""
    if not items:
        return
    with q.mutex:
        q.queue.extendleft(reversed(items))
        q.not_empty.notify(len(items))


def queued_updates(update_handler, helper, ahead=None, ahead_bytes=None, size_box=None):
    """The aggregators' drain of ``update_handler.model_updates`` (fedavg.py:47-50,
    fedopt.py:76-80): yields ``(model_update, load)`` in FIFO order until the queue is empty,
    where ``load()`` returns ``update_handler.load_model_update(model_update, helper)`` or
    raises its error (``model_update`` is None if dequeuing itself raised). The caller folds
    in that order, under its per-update error handling, exactly as the sequential loop.

    FEDn decodes each update inside the loop, one after the other; an npz update is one
    deflate stream per tensor (one core per update). Here queued updates are dequeued and
    decoded concurrently while earlier ones fold, so the fold waits for at most one decode:
    up to ``ahead`` updates, and — once the first decoded update shows the model's size — no
    more than ``ahead_bytes`` of decoded updates (one at least), counting the one being folded. A handler that stages updates
    on arrival (ingest.StagingUpdateHandler) is drained one by one: its loads are already done.

    ``size_box``: a list the caller keeps across rounds (the aggregator instance does): [0] holds
    the decoded size of the last update seen, so a later round admits its read-ahead at once
    instead of decoding its first update alone; [1] the mean time of one load last round — when it
    is below CHEAP_LOAD_S (an in-memory handler, a tiny model) the round is drained on the calling
    thread, as the thread hand-off would cost more than the load.

    Lossless: if the caller stops early (an exception that escapes its per-update handling,
    e.g. a BaseException, or ``close()``), the updates dequeued ahead but not yet handed out go
    back to the head of the queue in FIFO order — what FEDn's sequential loop leaves queued.
    Use it under ``contextlib.closing`` so that happens deterministically."""
    ahead = LOAD_AHEAD if ahead is None else ahead
    ahead_bytes = LOAD_AHEAD_BYTES if ahead_bytes is None else ahead_bytes
    q = update_handler.model_updates
    size = size_box if size_box is not None else [None]   # bytes of one decoded update, once known
    if len(size) < 2:
        size.append(None)
    load_times = []                       # this round's loads (s): [1] of the box for the next round

    def timed_load(mu):
        t0 = time.perf_counter()
        try:
            return update_handler.load_model_update(mu, helper)
        finally:
            load_times.append(time.perf_counter() - t0)

    cheap = size[1] is not None and size[1] < CHEAP_LOAD_S
    if ahead <= 1 or cheap or getattr(update_handler, "stages_on_arrival", False):
        try:
            while not q.empty():
                try:
                    mu = update_handler.next_model_update()
                except Exception as e:  # noqa: BLE001 — raised inside the caller's try, as FEDn's loop
                    yield None, _raiser(e)
                    continue
                yield mu, (lambda mu=mu: timed_load(mu))
        finally:
            if load_times:
                size[1] = sum(load_times) / len(load_times)
        return
    pool = _load_pool(ahead)
    window = deque()
    issued = []                           # loads submitted this round and not finished
    # with no size yet, the first update's raw bytes (UpdateHandler.load_model_update_byte,
    # updatehandler.py:119-144) show it from the npz directory before its decode ends
    known = threading.Event()
    peek = [size[0] is None and hasattr(update_handler, "load_model_update_byte")]
    peeking = [False]                     # a peek was issued: ``known`` will be set

    def peek_then_load(mu):
        try:
            est = npz_decoded_bytes(update_handler.load_model_update_byte(mu)[0])
            if est and size[0] is None:
                size[0] = est
        except Exception:  # noqa: BLE001 — no raw bytes: the first decode shows the size
            pass
        known.set()
        return timed_load(mu)

    def allowed():
        if size[0] is None:
            return 1
        return max(1, min(ahead, ahead_bytes // max(1, size[0])))

    def fill(held=0):
        # ``held``: an update handed out and still being folded keeps its decoded arrays
        while len(window) + held < allowed() and not q.empty():
            try:
                mu = update_handler.next_model_update()
            except Exception as e:  # noqa: BLE001
                window.append((None, None, e))
                continue
            if peek[0]:
                peek[0] = False
                peeking[0] = True
                fut = pool.submit(peek_then_load, mu)
            else:
                fut = pool.submit(timed_load, mu)
            issued[:] = [f for f in issued if not f.done()]   # done loads: their arrays are the caller's
            issued.append(fut)
            window.append((mu, fut, None))

    first = [True]

    def sized(fut):
        def load():
            res = fut.result()
            if first[0]:                  # this round's size (a hint from an earlier round is replaced)
                first[0] = False
                size[0] = model_nbytes(res[0]) or size[0]
            return res
        return load

    try:
        fill()
        while window:
            mu, fut, err = window.popleft()
            if fut is not None and size[0] is None and peeking[0]:
                while not fut.done() and not known.wait(0.002):
                    pass                  # the first update's npz directory admits the others early
            fill(held=1)
            yield mu, (_raiser(err) if err is not None else sized(fut))
            fill()
    finally:
        back = [mu for mu, _, _ in window if mu is not None]
        for _, fut, _ in window:
            if fut is not None:
                fut.cancel()
        window.clear()
        wait_futures([f for f in issued if not f.cancelled()])   # no load of this round outlives it
        requeue_front(q, back)
        if load_times:
            size[1] = sum(load_times) / len(load_times)


class AggregatorBase(ABC):
    """Abstract aggregator (aggregatorbase.py:9-41)."""

    @abstractmethod
    def __init__(self, update_handler):
        self.name = self.__class__.__name__
        self.update_handler = update_handler
        self._ahead_size = [None, None]  # last round's decoded update size and mean load time (queued_updates)

    @abstractmethod
    def combine_models(self, helper=None, delete_models=True, parameters=None):
        """Drain the update queue and return ``(model, data)``."""

    def _settle(self, pipe, waiting, delete_models):
        """Bookkeeping of updates whose fold is deferred to a batched launch. ``waiting``: the admitted
        updates (``ModelUpdate`` tags, FIFO) not yet deleted from storage. An update the pipeline
        skipped — its batch's launch failed and its own one-at-a-time fold failed too — is logged as
        FEDn logs a fold that raises (fedavg.py:75-78, fedopt.py:103-106), is not counted, and stays in
        storage (FEDn deletes only after a successful fold, fedavg.py:71-74); the others are deleted
        once folded (the pipeline's ``unsettled()`` newest ones still wait). Returns how many were
        skipped."""
        import traceback
        skipped = pipe.take_skipped() if hasattr(pipe, "take_skipped") else []
        for tag, exc in skipped:
            self._log_skip(exc, "".join(traceback.format_exception(type(exc), exc, exc.__traceback__)))
            for i, mu in enumerate(waiting):
                if mu is tag:
                    del waiting[i]
                    break
        keep = pipe.unsettled() if hasattr(pipe, "unsettled") else 0
        while len(waiting) > keep:
            mu = waiting.popleft()
            if delete_models:
                try:
                    self.update_handler.delete_model(mu)
                except Exception as e:  # noqa: BLE001 — inside the per-update try in the reference
                    self._log_skip(e, traceback.format_exc())   # (fedavg.py:73-78): logged, still counted
        return len(skipped)

    def _queued(self):
        """Updates still in the queue (0 if the handler's queue cannot say): with the one being folded,
        the round's size as the small-round paths see it (smallround.py)."""
        try:
            return self.update_handler.model_updates.qsize()
        except Exception:  # noqa: BLE001
            return 0

    def _begin_deletes(self):
        """The round's store deletes may run side by side (ingest.StagingUpdateHandler.begin_deletes)
        until :meth:`_finish_deletes`."""
        begin = getattr(self.update_handler, "begin_deletes", None)
        if begin is not None:
            begin()

    def _end_round(self, pipe):
        """However a round ends: the native gather thread is done with the round's update arrays and
        arenas before they can be freed or reused (staging._Pipeline.quiesce), and — even when that
        wait raises — the round's store deletes are all done, their failures logged."""
        try:
            if pipe is not None and hasattr(pipe, "quiesce"):
                pipe.quiesce()
        finally:
            try:
                self._finish_deletes()
            except Exception as e:  # noqa: BLE001 — logged; never masks the round's own exception
                import traceback
                self._log_skip(e, traceback.format_exc())

    def _finish_deletes(self):
        """Wait for the store deletes an update handler runs side by side
        (ingest.StagingUpdateHandler.finish_deletes): every folded update is deleted when
        combine_models returns, as in the reference; one that raised is logged as fedavg.py:75-78
        logs it."""
        fin = getattr(self.update_handler, "finish_deletes", None)
        if fin is None:
            return
        import traceback
        for _mu, exc in fin():
            self._log_skip(exc, "".join(traceback.format_exception(type(exc), exc, exc.__traceback__)))

    def _log_skip(self, exc, tb):
        import logging
        log = logging.getLogger("fedn")
        log.error(f"AGGREGATOR({self.name}): Error encoutered while processing model update: {exc}")
        log.error(tb)


def get_aggregator(aggregator_module_name, update_handler):
    """aggregatorbase.py:44-62."""
    module = importlib.import_module(AGGREGATOR_PLUGIN_PATH.format(aggregator_module_name))
    return module.Aggregator(update_handler)
