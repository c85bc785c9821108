"""Controller-level reduce of combiner models on the GPU — mirror of
``Control.reduce`` (fedn/network/controller/control.py:648-693).

FEDn's controller combines the models produced by its combiners with the same helper
arithmetic as FedAvg, unweighted: ``model = helper.increment_average(model, model_next,
1.0, i)`` (control.py:682) with i counting the models fetched so far. Quirks kept:
the first model becomes the running model because ``increment_average(None, ...)``
raises (control.py:683-686); a later model whose fold raises REPLACES the running model
(same except branch); ``i`` advances for every fetched model; every combiner's model is
deleted from the repository whether or not it could be fetched (control.py:690).

Use it from FEDn by mixing :class:`GpuReduceMixin` into ``Control``.
"""
import threading
import time
from concurrent.futures import ThreadPoolExecutor

from .aggregators.aggregatorbase import LOAD_AHEAD_BYTES, model_nbytes, npz_decoded_bytes
from .aggregators.fedavg import default_device
from .staging import FedAvgPipeline


def _fetch_load(fetch, load, model_id, on_size=None):
    """(data, model or None, load exception or None, t_fetch, t_load) for one combiner;
    ``on_size(bytes)`` hears the decoded size as soon as the fetched payload shows it."""
    tic = time.time()
    try:
        data = fetch(model_id)
    except Exception:  # noqa: BLE001 — control.py:671-673
        data = None
    t_fetch = time.time() - tic
    if data is None:
        return None, None, None, t_fetch, 0.0
    if on_size is not None and isinstance(data, (bytes, bytearray, memoryview)):
        est = npz_decoded_bytes(data)
        if est:
            on_size(est)
    tic = time.time()
    try:
        model = load(data)
    except Exception as e:  # noqa: BLE001 — re-raised in order by reduce_models
        return data, None, e, t_fetch, time.time() - tic
    return data, model, None, t_fetch, time.time() - tic


def reduce_models(combiners, fetch, load, delete=None, device=None, workers=8):
    """Combine ``combiners`` = [{"name", "model_id"}, ...] in order; returns (model, meta).

    fetch(model_id) -> bytes (may raise: treated as missing, control.py:671-673)
    load(bytes)     -> list[np.ndarray]  (FEDn: load_model_from_bytes(data, helper))
    delete(model_id) optional repository cleanup.
    workers         combiners fetched + decoded ahead of the fold, concurrently (decoding an
                    npz is one deflate stream per tensor, i.e. one core per model; FEDn does
                    them one after the other), within LOAD_AHEAD_BYTES of decoded models. The
                    fold order, the replace-on-error rule and the deletions stay those of the
                    sequential loop.
    """
    meta = {"time_fetch_model": 0.0, "time_load_model": 0.0, "time_aggregate_model": 0.0}
    i = 1
    pipe = None
    ids = [c["model_id"] for c in combiners]
    pool = ThreadPoolExecutor(max_workers=max(1, workers), thread_name_prefix="fedn_amd_reduce") if workers > 1 else None
    pending = {}
    nxt = [0]                              # next combiner index to submit
    size = [None]                          # host bytes of one decoded model, once known

    known = threading.Event()

    def on_size(nbytes):
        if size[0] is None:
            size[0] = nbytes
        known.set()

    def top_up(held=0):
        """Keep up to ``workers`` decodes in flight, and no more decoded-but-unfolded bytes than
        LOAD_AHEAD_BYTES (``held``: a model being waited for or folded counts too) once a model's
        size is known — from the first payload's zip directory, or the first decoded model —
        and one at a time until then."""
        cap = 1 if size[0] is None else max(1, min(workers, LOAD_AHEAD_BYTES // max(1, size[0])))
        while pool is not None and nxt[0] < len(ids) and len(pending) + held < cap:
            pending[nxt[0]] = pool.submit(_fetch_load, fetch, load, ids[nxt[0]], on_size)
            nxt[0] += 1

    try:
        for j, model_id in enumerate(ids):
            top_up()
            fut = pending.pop(j, None)
            if fut is not None:
                while size[0] is None and not fut.done() and not known.wait(0.002):
                    pass                         # the first payload's size admits the others early
                top_up(held=1)
            data, model_next, err, t_fetch, t_load = fut.result() if fut is not None else \
                _fetch_load(fetch, load, model_id)
            if size[0] is None and model_next is not None:
                size[0] = model_nbytes(model_next)
            top_up(held=1)
            meta["time_fetch_model"] += t_fetch
            if data is not None:
                meta["time_load_model"] += t_load if err is None else 0.0
                try:
                    if err is not None:
                        raise err
                    tic = time.time()
                    if pipe is None:
                        raise TypeError("no running model yet")   # increment_average(None, ...) raises
                    pipe.add(model_next, 1.0, i)
                    meta["time_aggregate_model"] += time.time() - tic
                except Exception:  # noqa: BLE001 — control.py:683-686
                    tic = time.time()
                    if model_next is None:       # the load itself raised: FEDn loads again (and raises)
                        model_next = load(data)
                    # else the fold raised: FEDn re-decodes the same bytes; the decoded arrays are reused
                    # no deferred batches: a fold that fails must raise here, where FEDn replaces the
                    # running model with this one (control.py:683-686)
                    pipe = FedAvgPipeline(device or default_device(), model_next, batch=False)
                    meta["time_aggregate_model"] += time.time() - tic
                i = i + 1
            if delete is not None:
                delete(model_id)
    finally:
        if pool is not None:
            for f in pending.values():
                f.cancel()
            pool.shutdown(wait=True)
    model = None
    if pipe is not None:
        tic = time.time()
        model = pipe.result()
        meta["time_aggregate_model"] += time.time() - tic
    return model, meta


class GpuReduceMixin:
    """``class Control(GpuReduceMixin, fedn.network.controller.control.Control)`` replaces
    ``Control.reduce`` with :func:`reduce_models` on the controller's repository/helper."""

    def reduce(self, combiners):
        from fedn.network.combiner.modelservice import load_model_from_bytes  # FEDn install

        helper = self.get_helper()
        return reduce_models(combiners, fetch=self.repository.get_model,
                             load=lambda data: load_model_from_bytes(data, helper),
                             delete=self.repository.delete_model)
