"""fedscale_amd — MI355X-native (gfx950 HIP) aggregator update-reduction path for FedScale.

Drop-in replacements for the reference's aggregation plugin surface:
  fedscale_amd.cloud.aggregation.aggregator   DeviceAggregatorMixin / DeviceAsyncAggregatorMixin
  fedscale_amd.cloud.aggregation.optimizers   TorchServerOptimizer
  fedscale_amd.cloud.internal.torch_model_adapter  TorchModelAdapter
  fedscale_amd.utils.optimizer.yogi           YoGi
The arithmetic runs in libfedagg.so (fedscale_amd/csrc/fedagg.hip, C ABI in include/fedagg.h).
"""
__version__ = "0.1.0"
