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
* any other codec mix, float64 gradients (``RandomGaussian`` with ``noise_scale == 0``,
  attack_models.py:105-106) and float64 GAR weights take the generic path: the drop-in
  ``Compression`` per client in row order (same NumPy RNG draws as the reference), rows
  stacked on the device in G's dtype, the same reductions in that dtype.

``aggregate_grads`` is a plain function so that :func:`openmsftl_amd.integration.install` can
bind it onto the REFERENCE ``Aggregator`` class (its ``self.gar`` may then be a reference GAR
with no ``aggregate_packets``: G is then handed over as the host array the reference builds).

Results are bit-exact against the reference (tests/golden/make_golden_agg.py pins the merge and
the sign-of-zero semantics; tests/test_gpu_parity.py runs both paths).  Out of the hot path and
not rebuilt: ``pc_analysis`` (randomized SVD of G), ``SpectralFedAvg``, ``update_model`` and the
RL / DGA aggregators: the device class raises ``NotImplementedError`` for them,
the patched reference class keeps its own code for ``pc_analysis``.
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


def _device_of(agg) -> torch.device:
    dev = getattr(agg, "device", None)
    if isinstance(dev, torch.device) and dev.type == "cuda":
        return dev
    return torch.device("cuda", torch.cuda.current_device())


def common_top_fraction(clients) -> Optional[float]:
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


def encode_top_clients(clients, n: int, f: float, device: torch.device):
    """Every client's top-k packet (one batched launch sequence; exact re-encode of the rare
    RETRY packets).  The packets drop their reference to the device gradient afterwards."""
    k = kept_count(f, n)
    grads = [torch.from_numpy(np.ascontiguousarray(c.grad)).to(device, non_blocking=True)
             for c in clients]
    if 0 < k < n:
        packets = codec.encode_top_batch(grads, k)
    else:                                   # trivial k (0, all, or the negative slice)
        packets = [codec.encode_top(g, k) for g in grads]
    for p in packets:                       # resolved: the gradient is no longer needed
        p.release()
    return packets


def merge_packets(packets, cluster_size: int) -> torch.Tensor:
    """First merge stage straight from the packets (aggregation.py:80-93).  Merged rows are
    separate (16-B aligned) buffers while they are written, stacked at the end."""
    bounds = _cluster_bounds(len(packets), cluster_size)
    rows = []
    for s, e in bounds:
        r = codec.decode_accumulate(packets[s:e], [1.0] * (e - s))
        rows.append(codec.div_scalar(r, float(e - s)))
    return torch.stack(rows)


def merge_stages(G: torch.Tensor, sizes) -> torch.Tensor:
    """Merge stages over dense device rows (fp32 or fp64 G): +0-started sums (weights 1),
    then / count, in G's dtype (np.mean(G[s:e], axis=0), aggregation.py:91)."""
    for cs in sizes:
        bounds = _cluster_bounds(G.shape[0], cs)
        rows = []
        for s, e in bounds:
            r = codec.weighted_sum_dense(G[s:e], torch.ones(e - s, dtype=G.dtype), out_dtype=G.dtype)
            rows.append(codec.div_scalar(r, float(e - s)))
        G = torch.stack(rows)
    return G


def aggregate_grads(self, clients: List, input_feature: np.ndarray = None,
                    val_loader=None) -> None:
    """aggregation.py:54-78 on the device: sets ``self.agg_grad`` (host array) and
    ``self.curr_G`` as the reference does."""
    if len(clients) == 0:
        raise Exception('Client List is Empty')
    self.curr_packets = None                # last round's packets go before this round encodes
    if self.analyze_pc is True:
        ref = getattr(type(self), "_ref_aggregate_grads", None)
        if ref is not None:                 # patched reference class: its own SVD analysis
            return ref(self, clients, input_feature, val_loader)
        raise NotImplementedError("pc_analysis (randomized SVD of G) is outside the hot path")
    dev = _device_of(self)
    grad0 = np.asarray(clients[0].grad)
    n = grad0.shape[0]
    if any(np.asarray(c.grad).shape != (n,) for c in clients):
        raise ValueError("client gradients must share one length (aggregation.py:61)")
    device_gar = hasattr(self.gar, "aggregate_packets")
    w = getattr(self.gar, "gradient_weights", None)
    f32_weights = w is None or np.asarray(w).dtype == np.float32
    top_f = None
    if device_gar and grad0.dtype == np.float32 and f32_weights:
        top_f = common_top_fraction(clients)
    if top_f is not None:
        packets = encode_top_clients(clients, n, top_f, dev)
        self.curr_packets = packets
        if self.num_hierarchies > 0:
            H = merge_packets(packets, self.cluster_size_list[0])
            H = merge_stages(H, self.cluster_size_list[1:])
            self.curr_G = H
            agg = self.gar.aggregate(G=H, client_ids=np.arange(H.shape[0]))
        else:
            self.curr_G = None
            agg = self.gar.aggregate_packets(packets)
    else:
        # generic codec mix / float64: the drop-in Compression per client, in row order; rows
        # take G's dtype (aggregation.py:61-63: G = zeros(..., dtype=clients[0].grad.dtype))
        tdt = torch.float64 if grad0.dtype == np.float64 else torch.float32
        G = torch.empty((len(clients), n), dtype=tdt, device=dev)
        for ix, c in enumerate(clients):
            q = c.C.compress(c.grad)
            q = q if isinstance(q, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(q))
            G[ix].copy_(q)                  # implicit cast to G's dtype, as G[ix, :] = q
        if self.num_hierarchies > 0:
            G = merge_stages(G, self.cluster_size_list)
            client_ids = np.arange(G.shape[0])
        else:
            client_ids = np.array([c.client_id for c in clients])
        if device_gar:
            self.curr_G = G
            agg = self.gar.aggregate(G=G, client_ids=client_ids)
        else:                               # a reference GAR: the host G it expects
            self.curr_G = G.cpu().numpy()
            agg = self.gar.aggregate(G=self.curr_G, client_ids=client_ids)
    self.agg_grad = agg.cpu().numpy() if isinstance(agg, torch.Tensor) else agg


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
        self.device = device                # None: the current device, resolved per call

    def __get_gar(self):                                                  # aggregation.py:44-52
        scheme = self.aggregation_config["aggregation_scheme"]
        if scheme == "fed_avg":
            return FedAvg(aggregation_config=self.aggregation_config)
        if scheme == "fed_spectral_avg":
            raise NotImplementedError("SpectralFedAvg is outside the codec hot path (DESIGN.md §8)")
        raise NotImplementedError

    aggregate_grads = aggregate_grads

    def update_model(self):
        raise NotImplementedError("model update is outside the codec hot path (DESIGN.md §8)")


__all__ = ["Aggregator", "Compression", "aggregate_grads"]
