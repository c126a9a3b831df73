"""Drop-in ``Aggregator.aggregate_grads`` (ftl/gradient_aggregation/aggregation.py:19-93) on MI355X.

The reference builds the dense host matrix ``G`` (M x N) row by row from
``client.C.compress(client.grad)`` (aggregation.py:61-63), optionally merges client clusters
(``__merge_gradient``, aggregation.py:80-93, ``num_hierarchies > 0``) and reduces it with the
GAR (gar.py:44).  Here the rows never become a dense matrix on the common path:

* every client's gradient goes to the GPU once; when all clients compress with ``'top'`` at
  one fraction (the configured codec, client_config.json:48-50) they are encoded in ONE
  batched launch sequence (``fc_topk_encode_batch``) into device packets;
* without hierarchies the packets are folded straight into the FedAVG sum
  (``fc_decode_accumulate``: bit-exact ``np.sum(G * w[:, None], axis=0)``);
* with hierarchies each first-stage cluster mean is the packet fold with weights 1 (the
  +0-started row-order sum ``np.mean`` computes) divided once by the row count
  (``fc_div_scalar``); later stages do the same over the dense merged rows
  (``fc_weighted_sum_dense``); the GAR then reduces the merged rows.
* any other codec mix takes the generic path: the drop-in ``Compression`` per client in row
  order (same NumPy RNG draws as the reference), rows stacked on the device, same reductions.

Results are bit-exact against the reference (tests/golden/make_golden_agg.py pins the merge and
the sign-of-zero semantics; tests/test_gpu_parity.py runs both paths).  Out of the hot path and
not rebuilt: ``pc_analysis`` (randomized SVD of G), ``SpectralFedAvg``, ``update_model`` and the
RL / DGA aggregators — they raise ``NotImplementedError``.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from . import codec
from .compression import Compression, kept_count
from .gar import FedAvg


def _cluster_bounds(m: int, cluster_size: int):
    """aggregation.py:82-87: consecutive clusters, the last one absorbs the remainder."""
    num = m // cluster_size
    assert num > 0, "Too small cluter size: {} // {} == 0".format(m, cluster_size)
    bounds = [[i * cluster_size, (i + 1) * cluster_size] for i in range(num)]
    if bounds[-1][1] < m:
        bounds[-1][1] = m
    return bounds


class Aggregator:
    """aggregation.py:19-93 — the aggregation hot path of the reference's ``Aggregator``.

    Same constructor, attributes and ``aggregate_grads`` contract; ``agg_grad`` is the host
    NumPy array the server loop reads (server.py:98 -> update_model)."""

    def __init__(self, aggregation_config: Dict, model=None, optimizer=None, clip_val=None,
                 lr_scheduler=None, device: Optional[torch.device] = None):
        self.aggregation_config = aggregation_config
        self.model = model
        self.opt = optimizer
        self.clip_val = clip_val if isinstance(clip_val, float) is True else -1.0
        self.lrs = lr_scheduler
        self.gar = self.__get_gar()
        self.curr_G = None
        self.curr_packets = None
        self.agg_grad = None
        self.analyze_pc = self.aggregation_config.get("pc_analysis", False)
        self.num_hierarchies = self.aggregation_config.get("num_hierarchies", 0)
        self.cluster_size_list = self.aggregation_config.get("cluster_size_list", [])
        assert self.num_hierarchies == len(self.cluster_size_list), \
            "Unmatched hierarchial and cluster size list length"
        self.device = device or torch.device("cuda", torch.cuda.current_device())

    def __get_gar(self):                                                  # aggregation.py:44-52
        scheme = self.aggregation_config["aggregation_scheme"]
        if scheme == "fed_avg":
            return FedAvg(aggregation_config=self.aggregation_config)
        if scheme == "fed_spectral_avg":
            raise NotImplementedError("SpectralFedAvg is outside the codec hot path (DESIGN.md §8)")
        raise NotImplementedError

    # ---- aggregation.py:54-78 ---------------------------------------------------------------
    def aggregate_grads(self, clients: List, input_feature: np.ndarray = None,
                        val_loader=None) -> None:
        if len(clients) == 0:
            raise Exception('Client List is Empty')
        if self.analyze_pc is True:
            raise NotImplementedError("pc_analysis (randomized SVD of G) is outside the hot path")
        grad0 = np.asarray(clients[0].grad)
        if grad0.dtype != np.float32:
            raise TypeError("device aggregation handles float32 gradients (DESIGN.md §8)")
        n = grad0.shape[0]
        if any(np.asarray(c.grad).shape != (n,) for c in clients):
            raise ValueError("client gradients must share one length (aggregation.py:61)")
        top_f = self._common_top_fraction(clients)
        if top_f is not None:
            packets = self._encode_top(clients, n, top_f)
            self.curr_packets = packets
            if self.num_hierarchies > 0:
                H = self._merge_packets(packets, self.cluster_size_list[0])
                H = self._merge_stages(H, self.cluster_size_list[1:])
                self.curr_G = H
                agg = self.gar.aggregate(G=H, client_ids=np.arange(H.shape[0]))
            else:
                self.curr_G = None
                agg = self.gar.aggregate_packets(packets)
        else:
            # generic codec mix: the drop-in Compression per client, in row order
            rows = [torch.from_numpy(np.ascontiguousarray(c.C.compress(c.grad), dtype=np.float32))
                    for c in clients]
            G = torch.stack(rows).to(self.device)
            self.curr_packets = None
            if self.num_hierarchies > 0:
                G = self._merge_stages(G, self.cluster_size_list)
                client_ids = np.arange(G.shape[0])
            else:
                client_ids = np.array([c.client_id for c in clients])
            self.curr_G = G
            agg = self.gar.aggregate(G=G, client_ids=client_ids)
        self.agg_grad = agg.cpu().numpy() if isinstance(agg, torch.Tensor) else agg

    # ---- helpers ----------------------------------------------------------------------------
    @staticmethod
    def _common_top_fraction(clients) -> Optional[float]:
        """The fraction when every client compresses with 'top' at one fraction whose k lies in
        [0, N] (f < 0 / f > 1 keep the reference's slice semantics: generic path), else None."""
        fr = None
        for c in clients:
            C = c.C
            if getattr(C, "compression_function", None) != "top":
                return None
            f = C.fraction_coordinates
            if fr is None:
                fr = f
            elif f != fr:
                return None
        n = len(clients[0].grad)
        return fr if 0 <= kept_count(fr, n) <= n else None

    def _encode_top(self, clients, n: int, f: float):
        k = kept_count(f, n)
        grads = [torch.from_numpy(np.ascontiguousarray(c.grad)).to(self.device, non_blocking=True)
                 for c in clients]
        if 0 < k < n:
            packets = codec.encode_top_batch(grads, k)
        else:                                   # trivial k (0, all, or the negative slice)
            packets = [codec.encode_top(g, k) for g in grads]
        return packets

    def _merge_packets(self, packets, cluster_size: int) -> torch.Tensor:
        """First merge stage straight from the packets (aggregation.py:80-93).  Merged rows are
        separate (16-B aligned) buffers while they are written, stacked at the end."""
        bounds = _cluster_bounds(len(packets), cluster_size)
        rows = []
        for s, e in bounds:
            r = codec.decode_accumulate(packets[s:e], [1.0] * (e - s))
            rows.append(codec.div_scalar(r, float(e - s)))
        return torch.stack(rows)

    def _merge_stages(self, G: torch.Tensor, sizes) -> torch.Tensor:
        """Later merge stages over dense device rows: +0-started sums (weights 1), then / count."""
        for cs in sizes:
            bounds = _cluster_bounds(G.shape[0], cs)
            rows = []
            for s, e in bounds:
                r = codec.weighted_sum_dense(G[s:e], torch.ones(e - s, dtype=torch.float32))
                rows.append(codec.div_scalar(r, float(e - s)))
            G = torch.stack(rows)
        return G

    def update_model(self):
        raise NotImplementedError("model update is outside the codec hot path (DESIGN.md §8)")


__all__ = ["Aggregator", "Compression"]
