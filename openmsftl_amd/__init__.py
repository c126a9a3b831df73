"""openmsftl_amd — MI355X-native gradient codec + FedAVG reduce for OpenMSFTL's hot path.

Drop-in surfaces (same names/arguments as the reference):
  openmsftl_amd.compression.Compression   <- ftl/compression/compression.py:8-77
  openmsftl_amd.gar.FedAvg / GAR          <- ftl/gradient_aggregation/gar.py:11-56
Device-resident API: openmsftl_amd.codec (encode_top, encode_mask, decode, decode_accumulate).
Multi-GPU sharding: openmsftl_amd.distributed.
"""
from .compression import Compression  # noqa: F401
from .gar import GAR, FedAvg  # noqa: F401

__all__ = ["Compression", "FedAvg", "GAR"]
