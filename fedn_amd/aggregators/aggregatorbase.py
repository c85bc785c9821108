"""Aggregator plug-in base and loader — mirror of
fedn/network/combiner/aggregators/aggregatorbase.py:6-62.

``get_aggregator(name, update_handler)`` imports ``fedn_amd.aggregators.<name>`` and
returns ``module.Aggregator(update_handler)``, the same contract FEDn's RoundHandler
uses (roundhandler.py:110-111). To serve an unmodified FEDn combiner, a one-line shim
module at ``fedn/network/combiner/aggregators/<name>.py`` re-exports our Aggregator
(see INTEGRATION.md).
"""
import importlib
from abc import ABC, abstractmethod

AGGREGATOR_PLUGIN_PATH = "fedn_amd.aggregators.{}"


class AggregatorBase(ABC):
    """Abstract aggregator (aggregatorbase.py:9-41)."""

    @abstractmethod
    def __init__(self, update_handler):
        self.name = self.__class__.__name__
        self.update_handler = update_handler

    @abstractmethod
    def combine_models(self, helper=None, delete_models=True, parameters=None):
        """Drain the update queue and return ``(model, data)``."""


def get_aggregator(aggregator_module_name, update_handler):
    """aggregatorbase.py:44-62."""
    module = importlib.import_module(AGGREGATOR_PLUGIN_PATH.format(aggregator_module_name))
    return module.Aggregator(update_handler)
