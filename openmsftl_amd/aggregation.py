"""Drop-in ``Aggregator.aggregate_grads`` (ftl/gradient_aggregation/aggregation.py:19-93) on MI355X.

The reference builds the dense host matrix ``G`` (M x N) row by row from
``client.C.compress(client.grad)`` (aggregation.py:61-63), optionally merges client clusters
(``__merge_gradient``, aggregation.py:80-93, ``num_hierarchies > 0``) and reduces it with the
GAR (gar.py:44).  Here the rows never become a dense matrix on the common path:

* when all clients compress with ``'top'`` at one fraction (the configured codec,
  client_config.json:48-50) their host gradients stream through a bounded device ring
  (openmsftl_amd/pipeline.py): H2D, ``fc_topk_encode`` into packets, and every group of
  packets folded into the FedAVG sum (``fc_decode_accumulate``: bit-exact
  ``np.sum(G * w[:, None], axis=0)``).  On a node with several GPUs the groups go
  round-robin to one pipeline per GPU, driven by one host thread each, and the running sum
  hops between the GPUs in group order (``aggregation_config["devices"]``, default every
  visible GPU: the reference's single-process server loop, server.py:98-100, drives them all);
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

from . import _lib as L
from . import codec
from .compression import Compression, kept_count
from .gar import FedAvg
from .pipeline import HostFedAvg


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


#: default for aggregation_config["devices"] (``integration.install(devices=...)`` sets it):
#: "all" = every visible GPU of this process drives the streamed top-k path
DEFAULT_DEVICES = "all"


def stream_devices(agg) -> List[torch.device]:
    """The GPUs the streamed top-k path fans out over (one process, one pipeline each):
    ``aggregation_config["devices"]`` = "all" (every visible GPU), a count (the first n) or a
    list of device indices (repeats allowed: tests stand two pipelines on one GPU in for two
    GPUs); absent -> :data:`DEFAULT_DEVICES`.  An aggregator constructed with an explicit
    ``device`` and no ``devices`` key stays on that device."""
    cfg = getattr(agg, "aggregation_config", None) or {}
    spec = cfg.get("devices")
    if spec is None:
        if isinstance(getattr(agg, "device", None), torch.device):
            return [_device_of(agg)]
        spec = DEFAULT_DEVICES
    if spec is None or spec == 1:
        return [_device_of(agg)]
    if spec == "all":
        count = torch.cuda.device_count()
        if count <= 1:
            return [_device_of(agg)]
        return [torch.device("cuda", i) for i in range(count)]
    if isinstance(spec, int):
        if not 1 <= spec <= torch.cuda.device_count():
            raise ValueError(f"devices={spec}: {torch.cuda.device_count()} visible GPU(s)")
        return [torch.device("cuda", i) for i in range(spec)]
    devs = [torch.device("cuda", int(i)) for i in spec]
    if not devs:
        raise ValueError("devices: empty list")
    return devs


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


#: device bytes the streamed top-k path may hold (gradient ring + packets + aggregates);
#: aggregation_config["device_budget_bytes"] overrides, default a quarter of the free HBM
DEFAULT_BUDGET_FRACTION = 0.25


def _budget(agg, dev: torch.device) -> int:
    b = agg.aggregation_config.get("device_budget_bytes") if hasattr(agg, "aggregation_config") else None
    if b:
        return int(b)
    free, _ = torch.cuda.mem_get_info(dev)
    return int(free * DEFAULT_BUDGET_FRACTION)


def _stream_pipeline(agg, n: int, k: int, m: int, devs: List[torch.device]):
    """The aggregator's cached streaming pipeline for (n, k) on ``devs``: one HostFedAvg, or
    a DeviceRing of one HostFedAvg (two packet sets) per device; fold groups sized for the
    per-device budget."""
    from .pipeline import DeviceRing, HostFedAvg, plan_group
    cache = agg.__dict__.setdefault("_host_pipelines", {})
    sets = 1 if len(devs) == 1 else 2
    group = min(plan_group(n, m, _budget(agg, d), sets=sets) for d in devs)
    key = (n, k, tuple(d.index for d in devs))
    pipe = cache.get(key)
    if pipe is None or pipe.group < group:
        cache.clear()                       # one shape at a time: release the old buffers
        torch.cuda.empty_cache()
        if len(devs) == 1:
            pipe = HostFedAvg(n, k, group=group, device=devs[0])
        else:
            pipe = DeviceRing([HostFedAvg(n, k, group=group, device=d, sets=2) for d in devs])
        cache[key] = pipe
    return pipe


def stream_top_fold(agg, clients, n: int, f: float, weights: np.ndarray, dev: torch.device,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """FedAVG of the clients' top-k rows (aggregation.py:61-63 + gar.py:44) streamed from
    their host ``client.grad`` through a bounded H2D ring, encoded and folded group by group
    (openmsftl_amd/pipeline.py): device memory stays within the budget for any client count.
    With several devices (:func:`stream_devices`) the groups go round-robin to one pipeline
    per GPU and the running aggregate hops between them in group order (pipeline.DeviceRing):
    the same bits, every GPU's PCIe link busy.  Returns the device aggregate (``out`` if
    given, else on the device that folded the last group)."""
    k = kept_count(f, n)
    w = np.asarray(weights, np.float32)
    if not 0 < k < n:
        # trivial k (0, all rows): the exact engine, one client at a time through one device
        # slot and one packet, so the device bytes stay bounded whatever the client count
        slot = torch.empty(n, dtype=torch.float32, device=dev)
        pkt = codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k)
        acc = out if out is not None else torch.empty(n, dtype=torch.float32, device=dev)
        for i, c in enumerate(clients):
            slot.copy_(torch.from_numpy(np.ascontiguousarray(c.grad)))
            codec.encode_top(slot, k, packet=pkt)
            codec.decode_accumulate([pkt], [float(w[i])], out=acc, continue_sum=i > 0)
        return acc
    devs = stream_devices(agg)
    pipe = _stream_pipeline(agg, n, k, len(clients), devs)
    get = lambda i: clients[i].grad         # noqa: E731
    if isinstance(pipe, HostFedAvg) and (out is None or out.device == pipe.dev):
        return pipe.run(get, len(clients), w, out=out, to_host=False)
    acc = pipe.run(get, len(clients), w, to_host=False)
    if out is None:
        return acc
    out.copy_(acc)
    return out


def merge_streamed(agg, clients, n: int, f: float, cluster_size: int,
                   dev: torch.device) -> torch.Tensor:
    """First merge stage straight from the streamed packets (aggregation.py:80-93): each
    cluster's +0-started row-order sum (weights 1), then one fl32 division by its size."""
    bounds = _cluster_bounds(len(clients), cluster_size)
    H = torch.empty((len(bounds), n), dtype=torch.float32, device=dev)
    for r, (s, e) in enumerate(bounds):
        row = torch.empty(n, dtype=torch.float32, device=dev)   # 16-B aligned while written
        stream_top_fold(agg, clients[s:e], n, f, np.ones(e - s, np.float32), dev, out=row)
        H[r].copy_(codec.div_scalar(row, float(e - s)))
    return H


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
        # streamed from the host gradients, G never built (packets live group by group)
        self.agg_path = "stream-top"
        if self.num_hierarchies > 0:
            H = merge_streamed(self, clients, n, top_f, self.cluster_size_list[0], dev)
            H = merge_stages(H, self.cluster_size_list[1:])
            self.curr_G = H
            agg = self.gar.aggregate(G=H, client_ids=np.arange(H.shape[0]))
        else:
            self.curr_G = None
            w = self.gar._weights(len(clients), np.float32)     # gar.py:37-42 (persisted)
            agg = stream_top_fold(self, clients, n, top_f, w, dev)
    else:
        # generic codec mix / float64: the drop-in Compression per client, in row order; rows
        # take G's dtype (aggregation.py:61-63: G = zeros(..., dtype=clients[0].grad.dtype))
        self.agg_path = "dense"
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
        self.agg_grad = None
        self.agg_path = None                # "stream-top" | "dense": the path the last call took
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
