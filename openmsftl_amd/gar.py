"""Drop-in FedAVG reduce (ftl/gradient_aggregation/gar.py:11-56) on MI355X.

``FedAvg(aggregation_config).aggregate(G, client_ids)`` keeps the reference's contract —
weights default to ``full(M, 1/M, dtype=G.dtype)``, persist across rounds and are asserted
on M (gar.py:37-42) — and computes ``np.sum(G * w[:, None], axis=0)`` (gar.py:44) in the
HIP kernel ``k_wsum`` with the reference's exact fp32 operation order (bit-exact).

``aggregate_packets`` is the compressed fast path: it consumes device packets directly
(``k_decode<ACC>``) so the dense M x N matrix G of aggregation.py:61 is never built.
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np
import torch

from . import codec


class GAR:
    def __init__(self, aggregation_config: Dict):
        self.aggregation_config = aggregation_config
        self.gradient_weights = None
        self.Sigma_tracked = []
        self.alpha_tracked = []
        self.num_updates = 0

    def aggregate(self, G, client_ids=None):
        self.num_updates += 1

    def _weights(self, m: int, dtype) -> np.ndarray:
        if self.gradient_weights is None:                                  # gar.py:37-40
            self.gradient_weights = np.full(m, fill_value=1.0 / m, dtype=dtype)
        else:                                                              # gar.py:41-42
            assert len(self.gradient_weights) == m
        return self.gradient_weights

    def weighted_average(self, stacked_grad):
        """gar.py:32-46 for an (M, N) float32 G (NumPy array or CUDA tensor)."""
        on_device = isinstance(stacked_grad, torch.Tensor)
        m = int(stacked_grad.shape[0])
        dtype = np.float32 if on_device else stacked_grad.dtype
        w = self._weights(m, dtype)
        if on_device:
            G = stacked_grad
        else:
            if stacked_grad.dtype != np.float32:
                raise TypeError("HIP FedAVG handles float32 G (DESIGN.md §Scope)")
            G = torch.from_numpy(np.ascontiguousarray(stacked_grad)).cuda()
        wt = torch.from_numpy(np.asarray(w, dtype=np.float32))
        out = codec.weighted_sum_dense(G, wt)
        return out if on_device else out.cpu().numpy()

    def aggregate_packets(self, packets: Sequence["codec.Packet"], out=None) -> torch.Tensor:
        """FedAVG straight from device packets (no dense G): bit-equal to weighted_average on
        the G the reference would build from the same compressed rows."""
        w = self._weights(len(packets), np.float32)
        return codec.decode_accumulate(packets, [float(x) for x in w], out=out)


class FedAvg(GAR):
    def __init__(self, aggregation_config):
        GAR.__init__(self, aggregation_config=aggregation_config)

    def aggregate(self, G, client_ids=None):                               # gar.py:53-56
        return self.weighted_average(stacked_grad=G)
