"""NumPy restatement of the FedAVG reduce — TEST INFRASTRUCTURE (oracle).

Restates ``ftl/gradient_aggregation/gar.py:32-46`` (``GAR.weighted_average``) and
``gar.py:53-56`` (``FedAvg.aggregate``) and the dense-G build of
``ftl/gradient_aggregation/aggregation.py:61-63``.
"""
from __future__ import annotations

import numpy as np


class FedAvgOracle:
    """gar.py:11-56 — weights persist across calls and are asserted on M (gar.py:41-42)."""

    def __init__(self, aggregation_config: dict | None = None):
        self.aggregation_config = aggregation_config or {}
        self.gradient_weights = None
        self.num_updates = 0

    def weighted_average(self, stacked_grad: np.ndarray) -> np.ndarray:
        if self.gradient_weights is None:                                  # gar.py:37-40
            self.gradient_weights = np.full(stacked_grad.shape[0],
                                            fill_value=1.0 / stacked_grad.shape[0],
                                            dtype=stacked_grad.dtype)
        else:                                                              # gar.py:41-42
            assert len(self.gradient_weights) == stacked_grad.shape[0]
        return np.sum(np.multiply(stacked_grad,                            # gar.py:44
                                  self.gradient_weights[:, np.newaxis]), axis=0)

    def aggregate(self, G: np.ndarray, client_ids=None) -> np.ndarray:    # gar.py:53-56
        return self.weighted_average(stacked_grad=G)


def sequential_weighted_sum(rows, weights) -> np.ndarray:
    """The exact arithmetic of gar.py:44 for an (M,N) fp32 G, spelled out:
    ``acc = fl(w0*g0); acc = fl(acc + fl(wi*gi))`` in row order (probed
    bit-equal to np.sum(axis=0) for M=4,10,128)."""
    acc = None
    for w, r in zip(weights, rows):
        c = np.multiply(r, w)
        acc = c.copy() if acc is None else np.add(acc, c)
    return acc


def build_dense_G(compressed_rows, dtype) -> np.ndarray:
    """aggregation.py:61-63 — rows cast to ``clients[0].grad.dtype`` on assignment."""
    rows = list(compressed_rows)
    G = np.zeros((len(rows), len(rows[0])), dtype=dtype)
    for ix, r in enumerate(rows):
        G[ix, :] = r
    return G
