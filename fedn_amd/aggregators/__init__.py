"""FEDn aggregator plug-ins (fedavg, fedopt) running their reduction on MI355X."""
from .aggregatorbase import AGGREGATOR_PLUGIN_PATH, AggregatorBase, get_aggregator  # noqa: F401
