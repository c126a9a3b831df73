"""Drop-in ``Aggregator.aggregate_grads`` (ftl/gradient_aggregation/aggregation.py:19-93) on MI355X.

The reference builds the dense host matrix ``G`` (M x N) row by row from
``client.C.compress(client.grad)`` (aggregation.py:61-63), optionally merges client clusters
(``__merge_gradient``, aggregation.py:80-93, ``num_hierarchies > 0``) and reduces it with the
GAR (gar.py:44).  Here the rows never become a dense matrix on the common path:

* when every client's codec is one of compression.py's ('full', 'top', 'rand',
  'dropout-biased', 'dropout-unbiased') on float32 gradients, their host gradients stream
  through a bounded device ring (openmsftl_amd/pipeline.py): H2D, each row made on the device
  (top-k packets, mask packets whose masks are drawn on the host from the global
  ``np.random`` in row order exactly as the reference draws them, or the dense gradient for
  'full'), and every group folded into the FedAVG sum in row order (``fc_decode_accumulate``
  / ``fc_weighted_sum_dense_continue``: bit-exact ``np.sum(G * w[:, None], axis=0)``).  G is
  never built and device memory stays within ``device_budget_bytes`` for any client count.
  ``aggregation_config["devices"]`` (or ``integration.install(devices=...)``) fans the groups
  out round-robin over several GPUs, one pipeline and host thread each, the running sum
  hopping between them in group order; the default is the current device only;
* with hierarchies each first-stage cluster mean is the streamed fold with weights 1 (the
  +0-started row-order sum ``np.mean`` computes) divided once by the row count
  (``fc_div_scalar``); later stages do the same over the dense merged rows
  (``fc_weighted_sum_dense``); the GAR then reduces the merged rows.
* 'qsgd' (opt-in) or a codec the reference rejects, float64 gradients (``RandomGaussian``
  with ``noise_scale == 0``, attack_models.py:105-106) and float64 GAR weights take the
  generic path: the drop-in ``Compression`` per client in row order on the device (same NumPy
  RNG draws as the reference, the same exceptions at the same row), each row cast to G's dtype
  and folded at once into the GAR's sum in NumPy's promoted dtype (``fold_rows``: one row of
  device memory); only a merge (hierarchies) or a host GAR stacks the rows into G.

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
from .compression import Compression, bitmask_words, kept_count
from .gar import FedAvg
from .pipeline import HostFedAvg, MtRedraw, RowCodec, RowPlan


def _cluster_bounds(m: int, cluster_size: int):
    """aggregation.py:82-87: consecutive clusters, the last one absorbs the remainder."""
    num = m // cluster_size
    assert num > 0, "Too small cluter size: {} // {} == 0".format(m, cluster_size)
    bounds = [[i * cluster_size, (i + 1) * cluster_size] for i in range(num)]
    if bounds[-1][1] < m:
        bounds[-1][1] = m
    return bounds


def _merge_log(stage: int, cluster_size: int, bounds) -> None:
    """The reference's progress lines for one merge stage (aggregation.py:71, 88, 90), text and
    order included."""
    print("{}-stage gradient aggregation: cluster size={}".format(stage, cluster_size))
    print("#client clusters: {}".format(len(bounds)))
    for s, e in bounds:
        print("Averaging gradient from the {}-th client to the {}=th".format(s, e))


def _device_of(agg) -> torch.device:
    dev = getattr(agg, "device", None)
    if isinstance(dev, torch.device) and dev.type == "cuda":
        return dev
    return torch.device("cuda", torch.cuda.current_device())


#: default for aggregation_config["devices"] (``integration.install(devices=...)`` sets it):
#: None = the current device only; "all" = every visible GPU of this process
DEFAULT_DEVICES = None


def stream_devices(agg) -> List[torch.device]:
    """The GPUs the streamed path fans out over (one process, one pipeline each):
    ``aggregation_config["devices"]`` = "all" (every visible GPU), a count (the first n) or a
    list of device indices (repeats allowed: tests stand two pipelines on one GPU in for two
    GPUs); absent -> :data:`DEFAULT_DEVICES` (None: the current device).  An aggregator
    constructed with an explicit ``device`` and no ``devices`` key stays on that device."""
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


_STREAMED = ("full", "top", "rand", "dropout-biased", "dropout-unbiased")


def _streamable(C, n: int) -> bool:
    """Can this client's codec stream (its row made on the device exactly as compress()
    would make it)?  Anything else — 'qsgd', unknown names, an RNG mode or p the drop-in
    would reject — takes the generic path, which raises where the reference raises."""
    fn = getattr(C, "compression_function", None)
    if fn not in _STREAMED:
        return False
    if fn == "full":
        return True
    rng = getattr(C, "rng", "numpy")           # a reference Compression draws from np.random
    if rng not in ("numpy", "philox"):
        return False
    if fn in ("top", "rand"):
        f = getattr(C, "fraction_coordinates", None)
        return isinstance(f, (int, float, np.floating, np.integer)) and np.isfinite(f)
    p = getattr(C, "dropout_p", None)
    if not isinstance(p, (int, float, np.floating, np.integer)):
        return False
    return rng == "numpy" or 0.0 <= p <= 1.0


#: draw the reference's np.random dropout masks on the device (np.random's MT19937 stream by
#: jump-ahead, openmsftl_amd/csrc/fc_mt.hip) instead of on the host producer thread
DEVICE_MT = True


def _device_mt_ok(clients) -> bool:
    """Can the round's np.random draws be made on the device?  Only if every host-RNG row is a
    dropout row with p in [0, 1]: 'rand' (np.random.permutation) consumes a data-dependent
    number of draws, and an invalid p must raise at its row (the host path does)."""
    for c in clients:
        C = c.C
        fn = C.compression_function
        if getattr(C, "rng", "numpy") != "numpy":
            continue
        if fn == "rand":
            return False
        if fn in ("dropout-biased", "dropout-unbiased"):
            try:
                p = float(C.dropout_p)
            except (TypeError, ValueError):
                return False
            if not 0.0 <= p <= 1.0:
                return False
    return True


def row_plan(clients, n: int, device_mt: Optional[bool] = None) -> Optional[RowPlan]:
    """The streamed round's :class:`~openmsftl_amd.pipeline.RowPlan` (aggregation.py:61-63:
    row ix = compress(clients[ix].grad)), or None when some client's codec cannot stream.

    * 'full' -> the gradient itself (a dense row); 'top' -> a top-k packet (k = n: the
      gradient itself; k = 0: nothing kept);
    * 'rand' -> with ``np.random`` (the reference, and the drop-in default) a host mask from
      ``np.random.permutation(n)[:k]`` (compression.py:43); native Philox -> Philox-key top-k;
    * 'dropout-*' -> a host mask from ``np.random.binomial(1, p, (n,))`` (:51/:58), or device
      Bernoulli(p) (Philox); the unbiased 1/p scaling is applied by the fold
      (fl32(fl64(g) / p), compression.py:59-60 then the cast into G, aggregation.py:63).
    Host draws run in row order on the plan's producer thread, exactly the reference's
    consumption of the global RNG; Philox offsets are taken in row order too.  With
    ``device_mt`` (default :data:`DEVICE_MT`) and no host permutation in the round, the dropout
    masks are np.random's own draws made on the device instead (mask_src "mt": row r of the
    round's MtRound, from np.random's state now; :meth:`RowPlan.close` sets the state after)."""
    if not all(_streamable(c.C, n) for c in clients):
        return None
    use_mt = (DEVICE_MT if device_mt is None else device_mt) and _device_mt_ok(clients)
    mt_rows = 0
    specs, draws = [], {}
    for i, c in enumerate(clients):
        C = c.C
        fn = C.compression_function
        if fn == "full":
            specs.append(RowCodec("dense"))
            continue
        rng = getattr(C, "rng", "numpy")
        if fn in ("top", "rand"):
            k = kept_count(C.fraction_coordinates, n)
            if fn == "rand" and rng == "numpy":
                specs.append(RowCodec("mask", codec=L.FC_CODEC_RAND, mask_src="host"))
                draws[i] = (lambda k=k: bitmask_words(np.random.permutation(n)[:k], n, False))
                continue
            key_mode, seed, off = L.FC_KEY_MAGNITUDE, 0, 0
            if fn == "rand":
                key_mode, seed, off = L.FC_KEY_PHILOX, C.seed, C._next_offset()
            if k == n:
                specs.append(RowCodec("dense"))
            elif k == 0:
                specs.append(RowCodec("mask", codec=L.FC_CODEC_RAND, mask_src="none"))
            else:
                specs.append(RowCodec("top", k=k, key_mode=key_mode, seed=seed, offset=off))
            continue
        cid = L.FC_CODEC_DROPOUT_BIASED if fn == "dropout-biased" else L.FC_CODEC_DROPOUT_UNBIASED
        p = float(C.dropout_p)
        if rng == "numpy" and use_mt:
            specs.append(RowCodec("mask", codec=cid, p=p, mask_src="mt", offset=mt_rows))
            mt_rows += 1
        elif rng == "numpy":
            specs.append(RowCodec("mask", codec=cid, p=p, mask_src="host"))
            draws[i] = (lambda p=C.dropout_p: bitmask_words(np.random.binomial(1, p, (n,)), n, True))
        else:
            specs.append(RowCodec("mask", codec=cid, p=p, mask_src="philox", seed=C.seed,
                                  offset=C._next_offset()))
    return RowPlan(n, specs, draws, mt_rows=mt_rows)


#: device bytes the streamed path may hold (gradient ring + packets + aggregates);
#: aggregation_config["device_budget_bytes"] overrides, default a quarter of the free HBM
DEFAULT_BUDGET_FRACTION = 0.25


def _budget(agg, dev: torch.device) -> int:
    b = agg.aggregation_config.get("device_budget_bytes") if hasattr(agg, "aggregation_config") else None
    if b:
        return int(b)
    free, _ = torch.cuda.mem_get_info(dev)
    return int(free * DEFAULT_BUDGET_FRACTION)


def _stream_pipeline(agg, n: int, m: int, devs: List[torch.device]):
    """The aggregator's cached streaming pipeline for length n on ``devs``: one HostFedAvg, or
    a DeviceRing of one HostFedAvg (two packet sets) per device; fold groups sized for the
    per-device budget."""
    from .pipeline import DeviceRing, HostFedAvg, plan_group
    cache = agg.__dict__.setdefault("_host_pipelines", {})
    sets = 1 if len(devs) == 1 else 2
    group = min(plan_group(n, m, _budget(agg, d), sets=sets) for d in devs)
    key = (n, tuple(d.index for d in devs))
    pipe = cache.get(key)
    if pipe is None or pipe.group < group:
        cache.clear()                       # one shape at a time: release the old buffers
        torch.cuda.empty_cache()
        if len(devs) == 1:
            pipe = HostFedAvg(n, group=group, device=devs[0])
        else:
            pipe = DeviceRing([HostFedAvg(n, group=group, device=d, sets=2) for d in devs])
        cache[key] = pipe
    return pipe


def stream_fold(agg, clients, n: int, plan: RowPlan, weights: np.ndarray, dev: torch.device,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """FedAVG of the clients' rows (aggregation.py:61-63 + gar.py:44) streamed from their host
    ``client.grad`` through a bounded H2D ring, each row made on the device as ``plan`` says
    and every group folded in row order (openmsftl_amd/pipeline.py): device memory stays within
    the budget for any client count.  With several devices (:func:`stream_devices`) the
    groups go round-robin to one pipeline per GPU and the running aggregate hops between them
    in group order (pipeline.DeviceRing): the same bits, every GPU's PCIe link busy.  Returns
    the device aggregate (``out`` if given, else on the device that folded the last group)."""
    w = np.asarray(weights, np.float32)
    devs = stream_devices(agg)
    pipe = _stream_pipeline(agg, n, len(clients), devs)
    get = lambda i: clients[i].grad         # noqa: E731
    if isinstance(pipe, HostFedAvg) and (out is None or out.device == pipe.dev):
        return pipe.run(get, len(clients), w, out=out, to_host=False, plan=plan)
    acc = pipe.run(get, len(clients), w, to_host=False, plan=plan)
    if out is None:
        return acc
    out.copy_(acc)
    return out


def merge_streamed(agg, clients, n: int, plan: RowPlan, cluster_size: int,
                   dev: torch.device) -> torch.Tensor:
    """First merge stage straight from the streamed rows (aggregation.py:80-93): each
    cluster's +0-started row-order sum (weights 1), then one fl32 division by its size."""
    bounds = _cluster_bounds(len(clients), cluster_size)
    _merge_log(0, cluster_size, bounds)
    H = torch.empty((len(bounds), n), dtype=torch.float32, device=dev)
    for r, (s, e) in enumerate(bounds):
        row = torch.empty(n, dtype=torch.float32, device=dev)   # 16-B aligned while written
        stream_fold(agg, clients[s:e], n, plan.shifted(s), np.ones(e - s, np.float32), dev, out=row)
        H[r].copy_(codec.div_scalar(row, float(e - s)))
    return H


def merge_stages(G: torch.Tensor, sizes, first_stage: int = 0) -> torch.Tensor:
    """Merge stages over dense device rows (fp32 or fp64 G): +0-started sums (weights 1),
    then / count, in G's dtype (np.mean(G[s:e], axis=0), aggregation.py:91)."""
    for i, cs in enumerate(sizes):
        bounds = _cluster_bounds(G.shape[0], cs)
        _merge_log(first_stage + i, cs, bounds)
        rows = []
        for s, e in bounds:
            r = codec.weighted_sum_dense(G[s:e], torch.ones(e - s, dtype=G.dtype), out_dtype=G.dtype)
            rows.append(codec.div_scalar(r, float(e - s)))
        G = torch.stack(rows)
    return G


def _client_row(C, grad, dev: torch.device):
    """``C.compress(grad)`` (aggregation.py:63) as a device tensor: the drop-in Compression
    gets the gradient on the device (no D2H of its result); another codec object gets the host
    array it expects and its result is copied up."""
    if isinstance(C, Compression) and not isinstance(grad, torch.Tensor):
        a = np.asarray(grad)
        if a.dtype in (np.float32, np.float64) and a.ndim == 1:
            grad = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    q = C.compress(grad)
    if not isinstance(q, torch.Tensor):
        q = torch.from_numpy(np.ascontiguousarray(q))
    return q


def fold_rows(gar, clients, n: int, tdt: torch.dtype, dev: torch.device) -> torch.Tensor:
    """gar.py:44 over the rows aggregation.py:61-63 would stack, folded one row at a time as
    each client's codec makes it (same NumPy RNG draws, same order; each row cast to G's dtype
    ``tdt`` first, as ``G[ix, :] = q`` does): the +0-started row-order sum in NumPy's promoted
    dtype of G and the GAR's (persisted) weights, without the M x N matrix."""
    gdt = np.float64 if tdt == torch.float64 else np.float32
    w = gar._weights(len(clients), gdt)
    odt = torch.float64 if np.result_type(gdt, w.dtype) == np.float64 else torch.float32
    wt = torch.from_numpy(np.ascontiguousarray(w))
    acc = torch.empty(n, dtype=odt, device=dev)
    row = torch.empty(n, dtype=tdt, device=dev)
    for ix, c in enumerate(clients):
        row.copy_(_client_row(c.C, c.grad, dev))        # G[ix, :] = q (cast to G's dtype)
        codec.weighted_sum_dense([row], wt[ix:ix + 1], out=acc, out_dtype=odt,
                                 continue_sum=ix > 0)
    return acc


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
    plan = None
    # stream only when EVERY row is a float32 gradient: a float64 client after a float32 one
    # (RandomGaussian Byzantine noise, attack_models.py:105-118) is compressed in its own dtype
    # and cast into G's float32 row by the generic path, as aggregation.py:63 does
    all_f32 = all(np.asarray(c.grad).dtype == np.float32 for c in clients)
    streamable = device_gar and all_f32 and f32_weights and n > 0
    if streamable:
        plan = row_plan(clients, n)
    if plan is not None:
        # streamed from the host gradients, G never built (rows live group by group)
        self.agg_path = "stream"
        while True:
            try:
                if self.num_hierarchies > 0:
                    H = merge_streamed(self, clients, n, plan, self.cluster_size_list[0], dev)
                    H = merge_stages(H, self.cluster_size_list[1:], first_stage=1)
                    self.curr_G = H
                    agg = self.gar.aggregate(G=H, client_ids=np.arange(H.shape[0]))
                else:
                    self.curr_G = None
                    w = self.gar._weights(len(clients), np.float32)     # gar.py:37-42 (persisted)
                    agg = stream_fold(self, clients, n, plan, w, dev)
            except BaseException:
                plan.close(wait=False)
                raise
            try:
                plan.close()                # every draw done: the RNG is where the reference leaves it
            except MtRedraw:                # NumPy would redraw somewhere (~2^-52 per element):
                plan = row_plan(clients, n, device_mt=False)   # the reference's host draws
                continue
            break
        self.agg_draws = "device-mt" if plan.mt_rows else ("host" if plan.draws else None)
    else:
        # generic codec mix / float64: the drop-in Compression per client, in row order; rows
        # take G's dtype (aggregation.py:61-63: G = zeros(..., dtype=clients[0].grad.dtype))
        tdt = torch.float64 if grad0.dtype == np.float64 else torch.float32
        if device_gar and self.num_hierarchies == 0:
            # nothing reads G but the GAR: fold each row as it is made (bounded: one row)
            self.agg_path = "dense-fold"
            self.curr_G = None
            agg = fold_rows(self.gar, clients, n, tdt, dev)
            self.agg_grad = agg.cpu().numpy()
            return
        self.agg_path = "dense"
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
        self.agg_path = None                # "stream" | "dense-fold" | "dense": the last call's path
        self.agg_draws = None               # streamed np.random draws: "device-mt" | "host" | None
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
