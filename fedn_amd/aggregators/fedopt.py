"""FedOpt aggregator plug-in (FedAdam / FedYogi / FedAdaGrad) — drop-in for
fedn/network/combiner/aggregators/fedopt.py.

Same contract and observable behaviour as fedopt.py:13-258:
  * hyper-parameters: defaults {serveropt: adam, learning_rate: 1e-3, beta1: 0.9,
    beta2: 0.99, tau: 1e-4} merged with validated user kwargs; invalid ones return
    ``(None, data)`` without touching the queue (fedopt.py:52-66, 123-137);
  * the pseudo-gradient is the running weighted mean of ``update - model_old``, where
    ``model_old`` is the model the first folded update names (fedopt.py:89-94);
  * server step without bias correction; ``m``, ``v`` persist on the instance across the
    rounds of a session (fedopt.py:36-38) — here they stay resident in HBM;
  * an unknown ``serveropt`` drains the queue and returns ``(None, data)`` (fedopt.py:110-116);
  * output dtype float64 (``v`` starts as ``np.ones(...) * tau**2``, numpyhelper.py:141).
The whole reduction runs in libfedagg (bit-exact to the numpy reference).
"""
import contextlib
import logging
import time
import traceback
from collections import deque

from ..exceptions import InvalidParameterError
from ..parameters import Parameters
from ..ingest import ShardedStagedModel
from ..layout import spread
from ..smallround import SmallFedOptSessions
from ..staging import FedOptPipeline, FedOptState, StagingCache, helper_kind
from .aggregatorbase import AggregatorBase, queued_updates
from .fedavg import _packed_bytes, default_device, env_devices

logger = logging.getLogger("fedn")

import torch  # noqa: E402

DEFAULT_PARAMETERS = {"serveropt": "adam", "learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
PARAMETER_SCHEMA = {"serveropt": str, "learning_rate": float, "beta1": float, "beta2": float, "tau": float}


class Aggregator(AggregatorBase):
    """Federated Optimization (FedOpt) on MI355X."""

    #: server state storage: False = the reference's dtype flow (m promoted, v and the model
    #: float64); True = fp32-state mode (fedopt_f32state.py)
    fp32_state = False

    def __init__(self, update_handler, device=None, devices=None):
        super().__init__(update_handler)
        self.name = "fedopt"
        self.device = torch.device(device) if device is not None else None
        # several devices (argument or FEDN_AMD_DEVICES): old / pg / m / v sharded by parameter
        # slice over them inside this process (multidev.py); fixed for the instance's lifetime
        self.devices = devices or env_devices()
        # with several devices the model is sliced over them only when it is large enough
        # (layout.spread, decided by the session's first round; the state follows that choice)
        self.state = None
        self.sharded = None
        self._staging = StagingCache()   # pinned slots, arenas, streams and ring reused by the next round
        self._small = SmallFedOptSessions()   # configs[0]-sized rounds in one native call (smallround.py)

    def _pipeline(self, model_old, model_next):
        if self.sharded is None:
            self.sharded = bool(self.devices and len(self.devices) > 1 and
                                (isinstance(model_next, ShardedStagedModel) or
                                 len(spread(self.devices, _packed_bytes(model_next))) > 1))
            if self.sharded:
                from ..multidev import ShardedFedOptState
                self.state = ShardedFedOptState(self.fp32_state)
            else:
                self.state = FedOptState(self.fp32_state)
        if self.sharded:
            from ..multidev import ShardedFedOptPipeline
            return ShardedFedOptPipeline(self.devices, model_old, model_next)
        dev = self.device or (self.devices[0] if self.devices else None) or default_device()
        return FedOptPipeline(dev, model_old, model_next, cache=self._staging)

    def _small_round(self, model_old, model_next):
        """The one-call round (smallround.SmallFedOptRound) for a small single-dtype model on one
        device; None: the general pipeline."""
        if self.devices or self.sharded:
            return None
        dev = self.device or default_device()
        r = self._small.round(model_old, model_next, dev, self._pipeline, 1 + self._queued())
        if r is not None and self.sharded is None:
            self.sharded = False                 # what _pipeline decides for a one-device session
            self.state = FedOptState(self.fp32_state)
        return r

    # reference attribute names (fedopt.py:37-38): host copies of the HBM-resident state
    @property
    def m(self):
        return None if self.state is None else self.state.m_host()

    @property
    def v(self):
        return None if self.state is None else self.state.v_host()

    def combine_models(self, helper=None, delete_models=True, parameters=None):
        self._begin_deletes()
        try:
            return self._combine(helper, delete_models, parameters)
        finally:
            pipe, self._live = getattr(self, "_live", None), None
            self._end_round(pipe)

    def _combine(self, helper, delete_models, parameters):
        data = {"time_model_load": 0.0, "time_model_aggregation": 0.0}
        try:
            parameters = self._validate_and_merge_parameters(parameters, DEFAULT_PARAMETERS)
        except InvalidParameterError as e:
            logger.error(f"Aggregator {self.name} received invalid parameters: {e}")
            return None, data

        pipe = None
        small = False           # pipe is a SmallFedOptRound: nothing launched or deleted before its step
        nr_aggregated_models, total_examples = 0, 0
        waiting = deque()       # admitted updates not deleted yet: a batched fold may still skip them
        with contextlib.closing(queued_updates(self.update_handler, helper, size_box=self._ahead_size)) as updates:
            for model_update, load in updates:
                try:
                    tic = time.time()
                    model_next, metadata = load()
                    data["time_model_load"] += time.time() - tic

                    total_examples += metadata["num_examples"]
                    tic = time.time()
                    helper_kind(helper)            # UnsupportedHelper for a helper this does not implement
                    if helper is not None and not hasattr(helper, "subtract"):
                        # androidhelper has no numpyhelper primitives: fedopt.py:91 raises here for every
                        # update, each is logged and skipped, and the round returns (None, data)
                        raise AttributeError(f"'{type(helper).__name__}' object has no attribute 'subtract'")
                    if nr_aggregated_models == 0:
                        model_old = self.update_handler.load_model(helper, model_update.model_id)
                        pipe = self._small_round(model_old, model_next)
                        small = pipe is not None
                        if not small:
                            pipe = self._pipeline(model_old, model_next)
                        self._live = pipe
                    if not (small and pipe.add(model_next, metadata["num_examples"], total_examples, model_update)):
                        if small:       # not this layout, or the arena is full: the general path from here
                            pipe, small = pipe.general(), False
                            self._live = pipe
                        pipe.add(model_next, metadata["num_examples"], total_examples, tag=model_update)
                    data["time_model_aggregation"] += time.time() - tic

                    nr_aggregated_models += 1
                    waiting.append(model_update)
                    # a batch whose launch failed was folded one update at a time: skipped ones are
                    # logged and uncounted (fedopt.py:103-106), folded ones deleted
                    if not small:
                        nr_aggregated_models -= self._settle(pipe, waiting, delete_models)
                except Exception as e:  # noqa: BLE001 — fedopt.py:103-106
                    logger.error(f"Error processing model update: {e}. Skipping this update.")
                    logger.error(traceback.format_exc())
                    if nr_aggregated_models == 0:
                        if pipe is not None and hasattr(pipe, "quiesce"):
                            pipe.quiesce()          # its pack of the global model reads model_old
                        pipe, small = None, False
                    continue

        data["nr_aggregated_models"] = nr_aggregated_models
        if pipe is None or nr_aggregated_models == 0:
            return None, data
        try:
            tic = time.time()
            # (a one-call round whose launch fails hands its step to the general pipeline, which it then
            # reports through: skipped updates, timings)
            model = pipe.server_step(self.state, parameters)
            data["time_model_aggregation"] += time.time() - tic
            data.update(pipe.timings())
            if hasattr(pipe, "release"):
                pipe.release()
        except Exception as e:  # noqa: BLE001 — fedopt.py:111-116
            data["nr_aggregated_models"] = nr_aggregated_models - self._settle(pipe, waiting, delete_models)
            logger.error(f"Error during model aggregation: {e}")
            logger.error(traceback.format_exc())
            return None, data
        nr_aggregated_models -= self._settle(pipe, waiting, delete_models)
        data["nr_aggregated_models"] = nr_aggregated_models
        logger.info(f"Aggregator {self.name} completed. Aggregated {nr_aggregated_models} models.")
        return model, data

    def _validate_and_merge_parameters(self, parameters, default_parameters):
        """fedopt.py:123-137."""
        if parameters:
            Parameters(parameters).validate(PARAMETER_SCHEMA)
            parameters = dict(parameters)
        else:
            parameters = {}
        return {**default_parameters, **parameters}
