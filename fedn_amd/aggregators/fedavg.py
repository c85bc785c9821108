"""FedAvg aggregator plug-in — drop-in for fedn/network/combiner/aggregators/fedavg.py.

Same contract and observable behaviour as fedavg.py:8-83:
  * drains ``update_handler.model_updates`` in FIFO order (fedavg.py:47-50);
  * ``total_examples`` grows BEFORE the fold (fedavg.py:62), so an update whose fold
    fails is skipped but still counted; a load failure is skipped uncounted;
  * the first update is the model (fedavg.py:65-66): K = 1 returns it unchanged;
  * returns ``(model, data)`` with ``time_model_load``, ``time_model_aggregation``,
    ``nr_aggregated_models`` (fedavg.py:37-39, 80), ``(None, data)`` if nothing folded.
The fold ``x + (n*(y-x))/N`` (numpyhelper.py:32; binaryhelper inherits it) runs in libfedagg
on the GPU, bit-exact; a session on androidhelper folds with ITS rule instead,
``(1 - w)*x + w*y`` on one flat array (androidhelper.py:21-39, staging.AndroidFedAvgPipeline);
updates are staged through pinned memory and folded on arrival (fedn_amd/staging.py).
Extra ``data`` keys: ``time_h2d`` / ``time_kernel`` (HIP events), ``time_pack``, ``time_d2h``.
"""
import contextlib
import logging
import os
import time
import traceback
from collections import deque

import torch

from .. import ops
from ..ingest import ShardedStagedModel
from ..layout import Layout, spread
from ..smallround import SmallSessions
from ..staging import AndroidFedAvgPipeline, FedAvgPipeline, StagingCache, helper_kind
from .aggregatorbase import AggregatorBase, queued_updates

logger = logging.getLogger("fedn")


def env_devices():
    """FEDN_AMD_DEVICES="cuda:0,cuda:1,..." selects the single-process multi-GPU pipeline."""
    v = os.environ.get("FEDN_AMD_DEVICES")
    return [d.strip() for d in v.split(",") if d.strip()] if v else None


def _packed_bytes(model):
    """Packed size of an update (host arrays or a staged model): what layout.spread decides on."""
    lay = getattr(model, "layout", None)
    return (lay if lay is not None else Layout.of(model)).nbytes


def make_fedavg_pipeline(first, device=None, devices=None, helper=None, cache=None):
    devices = devices or env_devices()
    if helper_kind(helper) == "androidhelper":   # its own fold rule and model format
        return AndroidFedAvgPipeline(device or (devices[0] if devices else None) or default_device(), first)
    # several devices: slice the model over them when it is large (or already staged that way)
    if devices and len(devices) > 1 and (isinstance(first, ShardedStagedModel) or
                                         len(spread(devices, _packed_bytes(first))) > 1):
        from ..multidev import ShardedFedAvgPipeline
        return ShardedFedAvgPipeline(devices, first)
    return FedAvgPipeline(device or (devices[0] if devices else None) or default_device(), first, cache=cache)


_HIP_SEEN = False      # torch.cuda.is_available() was True once in this process (it stays so)


_DEVICES = {}          # torch.device per (FEDN_AMD_DEVICE, current device): built once, not per round


def default_device():
    global _HIP_SEEN
    env = os.environ.get("FEDN_AMD_DEVICE")
    if not env and not _HIP_SEEN:
        if not torch.cuda.is_available():
            raise RuntimeError("fedn_amd aggregators need a HIP device (torch.cuda.is_available() is False)")
        _HIP_SEEN = True
    key = env or torch.cuda.current_device()
    dev = _DEVICES.get(key)
    if dev is None:
        dev = _DEVICES[key] = torch.device(env) if env else torch.device("cuda", key)
    return dev


class Aggregator(AggregatorBase):
    """Federated Averaging on MI355X (weighted incremental mean of client updates)."""

    def __init__(self, update_handler, device=None, devices=None):
        super().__init__(update_handler)
        self.name = "fedavg"
        self.device = torch.device(device) if device is not None else None
        self.devices = devices   # several devices: parameter-slice sharding in this process (multidev.py)
        self._staging = StagingCache()   # pinned slots, arenas and streams reused by the next round
        self._small = SmallSessions()    # configs[0]-sized rounds: arena, plans, result blocks (smallround.py)

    def combine_models(self, helper=None, delete_models=True, parameters=None):
        self._begin_deletes()
        try:
            return self._combine(helper, delete_models, parameters)
        finally:
            pipe, self._live = getattr(self, "_live", None), None
            self._end_round(pipe)

    def _small_round(self, first, helper):
        """configs[0]'s one-call round (smallround.py) when ``first`` is a small float model's update
        on one device with numpyhelper's arithmetic; None: the general pipeline."""
        if self.devices or os.environ.get("FEDN_AMD_DEVICES") or helper_kind(helper) == "androidhelper":
            return None
        return self._small.round(first, self.device or default_device(), 1 + self._queued())

    def _general(self, helper):
        return lambda first: make_fedavg_pipeline(first, self.device, self.devices, helper, self._staging)

    def _combine(self, helper, delete_models, parameters):
        data = {"time_model_load": 0.0, "time_model_aggregation": 0.0}
        model = None
        nr_aggregated_models = 0
        total_examples = 0
        pipe = None
        small = False           # pipe is a SmallRound: nothing launched or deleted before its result
        waiting = deque()       # admitted updates not deleted yet: a batched fold may still skip them

        logger.info("AGGREGATOR({}): Aggregating model updates... ".format(self.name))
        with contextlib.closing(queued_updates(self.update_handler, helper, size_box=self._ahead_size)) as updates:
            for model_update, load in updates:
                try:
                    tic = time.time()
                    model_next, metadata = load()
                    data["time_model_load"] += time.time() - tic

                    total_examples += metadata["num_examples"]

                    tic = time.time()
                    if nr_aggregated_models == 0:
                        pipe = self._small_round(model_next, helper)
                        small = pipe is not None
                        if not small:
                            pipe = self._general(helper)(model_next)
                        self._live = pipe
                    elif not (small and pipe.add(model_next, metadata["num_examples"], total_examples, model_update)):
                        if small:       # not this layout, or the arena is full: the general path from here
                            pipe, small = pipe.general(self._general(helper)), False
                            self._live = pipe
                        pipe.add(model_next, metadata["num_examples"], total_examples, tag=model_update)
                    data["time_model_aggregation"] += time.time() - tic

                    nr_aggregated_models += 1
                    waiting.append(model_update)
                    # updates of a batch whose launch failed were refolded one at a time: the ones
                    # whose own fold failed are skipped (fedavg.py:75-78); the folded ones deleted
                    if not small:
                        nr_aggregated_models -= self._settle(pipe, waiting, delete_models)
                except Exception as e:  # noqa: BLE001 — fedavg.py:75-78: log and continue
                    logger.error(f"AGGREGATOR({self.name}): Error encoutered while processing model update: {e}")
                    logger.error(traceback.format_exc())

        if pipe is not None:
            tic = time.time()
            if small:
                try:
                    model = pipe.result()
                except ops.FedAggError:      # the launch failed: the general path's per-update recovery
                    pipe, small = pipe.general(self._general(helper)), False
                    self._live = pipe
            if not small:
                model = pipe.result()
            data["time_model_aggregation"] += time.time() - tic
            nr_aggregated_models -= self._settle(pipe, waiting, delete_models)
            data.update(pipe.timings())
            if hasattr(pipe, "release"):
                pipe.release()
        data["nr_aggregated_models"] = nr_aggregated_models
        logger.info("AGGREGATOR({}): Aggregation completed, aggregated {} models.".format(self.name, nr_aggregated_models))
        return model, data
