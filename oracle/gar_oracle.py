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
    ``acc = +0; acc = fl(acc + fl(wi*gi))`` in row order.  NumPy's axis-0 ``add.reduce``
    starts from the additive identity +0 (not from row 0): the two differ only in the sign
    of zero (an all-(-0) column sums to +0), pinned by
    tests/test_oracle_golden.py::test_numpy_axis0_sum_order (SURVEY.md §0.6 probed the
    nonzero values bit-equal for M=4,10,128)."""
    acc = None
    for w, r in zip(weights, rows):
        c = np.multiply(r, w)
        acc = np.add(np.zeros_like(c), c) if acc is None else np.add(acc, c)
    return acc


def cluster_mean(G: np.ndarray, start: int, stop: int) -> np.ndarray:
    """aggregation.py:91 ``np.mean(G[s:e, :], axis=0)`` for fp32 G, spelled out: the +0-started
    row-order sum, then one fp32 division by the row count (probed equal to np.mean)."""
    acc = np.zeros(G.shape[1], dtype=G.dtype)
    for r in range(start, stop):
        acc = np.add(acc, G[r])
    return np.true_divide(acc, G.dtype.type(stop - start))


def merge_gradient(G: np.ndarray, cluster_size: int) -> np.ndarray:
    """aggregation.py:80-93 (``Aggregator.__merge_gradient``): rows averaged over consecutive
    clusters of ``cluster_size``; the last cluster absorbs the remainder."""
    num = G.shape[0] // cluster_size
    assert num > 0, "Too small cluter size: {} // {} == 0".format(G.shape[0], cluster_size)
    bounds = [[i * cluster_size, (i + 1) * cluster_size] for i in range(num)]
    if bounds[-1][1] < G.shape[0]:
        bounds[-1][1] = G.shape[0]
    return np.stack([cluster_mean(G, s, e) for s, e in bounds]).astype(G.dtype)


def build_dense_G(compressed_rows, dtype) -> np.ndarray:
    """aggregation.py:61-63 — rows cast to ``clients[0].grad.dtype`` on assignment."""
    rows = list(compressed_rows)
    G = np.zeros((len(rows), len(rows[0])), dtype=dtype)
    for ix, r in enumerate(rows):
        G[ix, :] = r
    return G
