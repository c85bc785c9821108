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
import time

from .aggregators.fedavg import default_device
from .staging import FedAvgPipeline


def reduce_models(combiners, fetch, load, delete=None, device=None):
    """Combine ``combiners`` = [{"name", "model_id"}, ...] in order; returns (model, meta).

    fetch(model_id) -> bytes (may raise: treated as missing, control.py:671-673)
    load(bytes)     -> list[np.ndarray]  (FEDn: load_model_from_bytes(data, helper))
    delete(model_id) optional repository cleanup.
    """
    meta = {"time_fetch_model": 0.0, "time_load_model": 0.0, "time_aggregate_model": 0.0}
    i = 1
    pipe = None
    for combiner in combiners:
        model_id = combiner["model_id"]
        try:
            tic = time.time()
            data = fetch(model_id)
            meta["time_fetch_model"] += time.time() - tic
        except Exception:  # noqa: BLE001 — control.py:671-673
            data = None
        if data is not None:
            try:
                tic = time.time()
                model_next = load(data)
                meta["time_load_model"] += time.time() - tic
                tic = time.time()
                if pipe is None:
                    raise TypeError("no running model yet")   # increment_average(None, ...) raises
                pipe.add(model_next, 1.0, i)
                meta["time_aggregate_model"] += time.time() - tic
            except Exception:  # noqa: BLE001 — control.py:683-686
                tic = time.time()
                model_next = load(data)
                pipe = FedAvgPipeline(device or default_device(), model_next)
                meta["time_aggregate_model"] += time.time() - tic
            i = i + 1
        if delete is not None:
            delete(model_id)
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
