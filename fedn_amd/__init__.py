"""fedn_amd — MI355X-native (gfx950) implementation of FEDn's combiner-side aggregation.

The hot path (FedAvg / FedAdam / FedYogi / FedAdaGrad over client parameter buffers)
runs in hand-written HIP kernels behind the C ABI in ``include/fedagg.h``
(``fedn_amd/libfedagg.so``). Python here only mirrors FEDn's plug-in interfaces:

  fedn_amd.aggregators.get_aggregator(name, update_handler)   (aggregatorbase.py:44-62)
  fedn_amd.aggregators.fedavg.Aggregator / fedopt.Aggregator  (fedavg.py, fedopt.py)
  fedn_amd.ops.fedavg_fold / fedopt_step                      (device-tensor level)
  fedn_amd.sharded                                            (parameter-slice sharding, N GPUs)
"""
__version__ = "0.1.0"
