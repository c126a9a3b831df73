"""Drop-in FedAVG reduce (ftl/gradient_aggregation/gar.py:11-56) on MI355X.

``FedAvg(aggregation_config).aggregate(G, client_ids)`` keeps the reference's contract —
weights default to ``full(M, 1/M, dtype=G.dtype)``, persist across rounds and are asserted
on M (gar.py:37-42) — and computes ``np.sum(G * w[:, None], axis=0)`` (gar.py:44) in HIP
kernels with the reference's exact operation order (bit-exact):

* float32 G and float32 weights (the configured case): ``k_wsum``, fp32 products and sums;
* float64 G (after ``RandomGaussian`` with ``noise_scale == 0``, attack_models.py:105-106) or
  float64 weights (DGA's softmax / RL estimators set ``gradient_weights``,
  aggregation.py:181-198): NumPy promotes ``G * w`` to float64, so ``k_wsum64`` forms
  ``fl64(double(g) * w)`` and sums in fp64 from +0; the result is float64, as in the reference.

``aggregate_packets`` is the compressed fast path: it consumes device packets directly
(``k_decode_sparse``) so the dense M x N matrix G of aggregation.py:61 is never built; it
takes float32 weights (float64 weights go through the dense path of the Aggregator).
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np
import torch

from . import codec

_NP_OF = {torch.float32: np.float32, torch.float64: np.float64}


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
        w = np.asarray(self.gradient_weights)
        if w.dtype not in (np.float32, np.float64):
            raise TypeError(f"gradient_weights must be float32 or float64 (got {w.dtype})")
        return w

    def weighted_average(self, stacked_grad):
        """gar.py:32-46 for an (M, N) float32/float64 G (NumPy array or CUDA tensor).  The
        result has NumPy's promoted dtype of G and the weights; it is a CUDA tensor for a CUDA
        G and a NumPy array otherwise."""
        on_device = isinstance(stacked_grad, torch.Tensor)
        m = int(stacked_grad.shape[0])
        gdt = _NP_OF.get(stacked_grad.dtype) if on_device else stacked_grad.dtype
        if gdt not in (np.float32, np.float64):
            raise TypeError(f"HIP FedAVG handles float32/float64 G (got {stacked_grad.dtype})")
        w = self._weights(m, gdt)
        rdt = np.result_type(gdt, w.dtype)                                 # G * w[:, None]
        if on_device:
            G = stacked_grad
        else:
            G = torch.from_numpy(np.ascontiguousarray(stacked_grad)).cuda()
        out = codec.weighted_sum_dense(G, torch.from_numpy(np.ascontiguousarray(w)),
                                       out_dtype=torch.float64 if rdt == np.float64 else torch.float32)
        return out if on_device else out.cpu().numpy()

    def aggregate_packets(self, packets: Sequence["codec.Packet"], out=None) -> torch.Tensor:
        """FedAVG straight from device packets (no dense G): bit-equal to weighted_average on
        the G the reference would build from the same compressed rows."""
        w = self._weights(len(packets), np.float32)
        if w.dtype != np.float32:
            raise TypeError("aggregate_packets folds with float32 weights; float64 weights "
                            "promote G * w to float64 (use weighted_average on the dense G)")
        return codec.decode_accumulate(packets, [float(x) for x in w], out=out)


class FedAvg(GAR):
    def __init__(self, aggregation_config):
        GAR.__init__(self, aggregation_config=aggregation_config)

    def aggregate(self, G, client_ids=None):                               # gar.py:53-56
        return self.weighted_average(stacked_grad=G)
