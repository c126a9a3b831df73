"""Device-resident codec API over libfedcodec.so (torch tensors in HBM, torch's stream).

    pkt = encode_top(g, k)                 # compression.py:31-37   (one read of g)
    pkt = encode_rand_philox(g, k, seed)   # compression.py:39-45   native RNG
    pkt = encode_mask(g, codec, p, ...)    # compression.py:47-60 / rand parity
    q   = decode(pkt)                      # the dense vector compress() returns
    agg = decode_accumulate(pkts, w)       # aggregation.py:61-63 + gar.py:44, bit-exact fp32

Packets live on the GPU in the slotted layout of include/fedcodec.h: chunk c (8192 elements)
lists its entries, ascending, at ``[c*8192, c*8192 + cnt[c])`` of ``idx``/``val`` (or
``bitmap``/``val``); ``idx`` holds the chunk-local index as uint16 (element c*8192 + idx).
Plus per-chunk counts and quarter offsets and a 96-byte device header (``fc_packet_hdr``).
"""
from __future__ import annotations

import ctypes
import threading
import weakref
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib as L

_U32 = torch.int32  # uint32 payloads are stored in int32 tensors (bit-identical)
_U16 = torch.int16  # uint16 chunk-local indices in int16 tensors (bit-identical)


def _vp(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_cuda_f32(g: torch.Tensor, name="g", align: int = 16, dtype=torch.float32):
    if not isinstance(g, torch.Tensor) or not g.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) tensor")
    if g.dtype != dtype:
        raise TypeError(f"{name} must be {dtype} (got {g.dtype})")
    if g.dim() != 1 or not g.is_contiguous():
        raise ValueError(f"{name} must be a contiguous 1-D tensor")
    if g.data_ptr() % align:
        raise ValueError(f"{name} must be {align}-byte aligned")


# ---------------------------------------------------------------------------------------
class Workspace:
    """Per-(device, stream) encoder scratch (self-cleaning after one memset)."""

    _cache: dict = {}

    def __init__(self, n: int, device: torch.device):
        lib = L.load()
        self.n = n
        self.nbytes = int(lib.fc_workspace_bytes(n))
        self.buf = torch.empty(self.nbytes, dtype=torch.uint8, device=device)
        L.check(lib.fc_workspace_init(_vp(self.buf), self.nbytes, _stream(device)),
                "fc_workspace_init")

    @classmethod
    def get(cls, n: int, device: torch.device) -> "Workspace":
        key = (device.index if device.index is not None else torch.cuda.current_device(),
               torch.cuda.current_stream(device).cuda_stream)
        ws = cls._cache.get(key)
        if ws is None or ws.n < n:
            ws = cls(n, device)
            cls._cache[key] = ws
        return ws


@dataclass
class Packet:
    """A compressed gradient resident in HBM (see include/fedcodec.h)."""
    n: int
    fmt: int
    val: torch.Tensor
    cnt: torch.Tensor                      # int32[num_chunks]: entries per chunk slot
    hdr: torch.Tensor                      # uint8[96] (may be a row of a batch tensor)
    idx: Optional[torch.Tensor] = None
    bitmap: Optional[torch.Tensor] = None
    k: int = 0
    qoff: Optional[torch.Tensor] = None    # int64[num_chunks]: quarter offsets (FC_FMT_IDXVAL)

    @classmethod
    def alloc(cls, n: int, fmt: int, device, hdr: Optional[torch.Tensor] = None,
              k: int = 0) -> "Packet":
        lib = L.load()
        nch = int(lib.fc_num_chunks(n))
        cap = int(lib.fc_packet_capacity(n))
        return cls(n=n, fmt=fmt, k=k,
                   val=torch.empty(cap, dtype=torch.float32, device=device),
                   cnt=torch.empty(nch, dtype=_U32, device=device),
                   hdr=hdr if hdr is not None else torch.empty(L.HDR_BYTES, dtype=torch.uint8,
                                                               device=device),
                   idx=torch.empty(cap, dtype=_U16, device=device) if fmt == L.FC_FMT_IDXVAL else None,
                   bitmap=torch.empty(nch * 256, dtype=_U32, device=device)
                   if fmt == L.FC_FMT_BITMAP else None,
                   qoff=torch.empty(nch, dtype=torch.int64, device=device)
                   if fmt == L.FC_FMT_IDXVAL else None)

    @classmethod
    def alloc_batch(cls, n: int, m: int, fmt: int, device, k: int = 0) -> list:
        """``m`` packets of length n whose fields are the rows of per-field slabs (one (m, cap)
        value tensor, one index tensor, ...): the layout a batch of G's rows would have.  The
        128-client 16 M batched compaction writes them 2-3 % faster than m separate allocations
        (profiles/r05_stagger_probe.jsonl); the packets are ordinary Packet objects."""
        lib = L.load()
        nch = int(lib.fc_num_chunks(n))
        cap = int(lib.fc_packet_capacity(n))
        val = torch.empty((m, cap), dtype=torch.float32, device=device)
        idx = torch.empty((m, cap), dtype=_U16, device=device) if fmt == L.FC_FMT_IDXVAL else None
        bitmap = torch.empty((m, nch * 256), dtype=_U32, device=device) if fmt == L.FC_FMT_BITMAP else None
        cnt = torch.empty((m, nch), dtype=_U32, device=device)
        qoff = torch.empty((m, nch), dtype=torch.int64, device=device) if fmt == L.FC_FMT_IDXVAL else None
        hdr = torch.empty((m, L.HDR_BYTES), dtype=torch.uint8, device=device)
        return [cls(n=n, fmt=fmt, k=k, val=val[i], cnt=cnt[i], hdr=hdr[i],
                    idx=idx[i] if idx is not None else None,
                    bitmap=bitmap[i] if bitmap is not None else None,
                    qoff=qoff[i] if qoff is not None else None) for i in range(m)]

    @property
    def capacity(self) -> int:
        return self.val.numel()

    def release(self) -> None:
        """Drop the reference to the source gradient kept for the exact re-encode (call once
        :func:`resolve` has seen the packet OK), so the gradient's memory can be reused."""
        self._enc = None

    def _decodable(self) -> None:
        if getattr(self, "_dense_only", False):
            raise ValueError("this packet was scratch of compress_top_dense (header format "
                             "FC_FMT_DENSE): it lists no entries; decode the dense q instead")

    def view(self, weight: float = 1.0) -> L.PacketView:
        self._decodable()
        return L.PacketView(idx=self.idx.data_ptr() if self.idx is not None else 0,
                            val=self.val.data_ptr(),
                            bitmap=self.bitmap.data_ptr() if self.bitmap is not None else 0,
                            cnt=self.cnt.data_ptr(), hdr=self.hdr.data_ptr(),
                            qoff=self.qoff.data_ptr() if self.qoff is not None else 0,
                            weight=float(np.float32(weight)), reserved=0)

    def header(self) -> L.PacketHdr:
        """Synchronous D2H read of the device header."""
        raw = self.hdr.cpu().numpy().tobytes()
        return L.PacketHdr.from_buffer_copy(raw)

    def raw_entries(self):
        """(idx uint32 = global element index, val float32, header) of every LISTED entry,
        ascending — includes the sampled-bracket slack (comp < thresh); inspection / test
        helper (synchronises)."""
        self._decodable()
        h = self.header()
        cnt = self.cnt.cpu().numpy().astype(np.int64)
        pos = np.arange(self.capacity, dtype=np.int64)
        listed = (pos % L.FC_CHUNK) < cnt[pos // L.FC_CHUNK]
        val = self.val.cpu().numpy()[listed]
        if self.fmt == L.FC_FMT_IDXVAL:
            local = self.idx.cpu().numpy().view(np.uint16)[listed].astype(np.uint32)
            idx = (pos[listed] // L.FC_CHUNK * L.FC_CHUNK).astype(np.uint32) + local
        else:
            bits = np.unpackbits(self.bitmap.cpu().numpy().view(np.uint8), bitorder="little")
            idx = np.nonzero(bits[: self.n])[0].astype(np.uint32)
        return idx, val, h


def headers(packets: Sequence[Packet]) -> list:
    """Read many device headers with ONE synchronising copy (stacked on the device first)."""
    if not packets:
        return []
    raw = torch.stack([p.hdr for p in packets]).cpu().numpy()
    return [L.PacketHdr.from_buffer_copy(raw[i].tobytes()) for i in range(len(packets))]


# ---------------------------------------------------------------------------------------
def encode_top(g: torch.Tensor, k: int, *, key_mode: int = L.FC_KEY_MAGNITUDE, seed: int = 0,
               offset: int = 0, packet: Optional[Packet] = None,
               check: bool = True, exact: bool = False) -> Packet:
    """Top-k (|g|) or native rand-k (Philox keys) into an idx/val packet.

    ``check=True`` synchronises, reads the header and falls back to the exact device path
    if the sampled bracket missed (FC_STATUS_RETRY_EXACT).  With ``check=False`` call
    :func:`resolve` on the batch later (one sync per batch)."""
    _require_cuda_f32(g)
    lib = L.load()
    n = g.numel()
    if not 0 <= k <= n:
        raise ValueError(f"k={k} outside [0, {n}]")
    ws = Workspace.get(n, g.device)
    if packet is None:
        packet = Packet.alloc(n, L.FC_FMT_IDXVAL, g.device, k=k)
    packet.k = k
    fn = lib.fc_topk_encode_exact if exact else lib.fc_topk_encode
    L.check(fn(_vp(g), n, k, key_mode, seed, offset, _vp(packet.idx), _vp(packet.val),
               packet.capacity, _vp(packet.cnt), _vp(packet.qoff), _vp(packet.hdr), _vp(ws.buf),
               ws.nbytes, _stream(g.device)), "fc_topk_encode")
    packet._enc = (g, k, key_mode, seed, offset)
    packet._dense_only = False
    if check:
        resolve([packet])
    return packet


def encode_decode_top(g: torch.Tensor, k: int, *, packet: Optional[Packet] = None,
                      out: Optional[torch.Tensor] = None, check: bool = True):
    """compression.py:31-37 as a packet AND its dense decode (fc_topk_encode_decode): the
    packet fc_topk_encode writes (entries, counts, quarter offsets, header with T64), and
    ``out`` = decode(packet), with the resolve's gather and finish done by the decode launch
    itself (k_fused_mag -> k_beta -> k_decode_res; no gather launch in between).  Returns
    (packet, out).  ``check=False`` skips the status read (call :func:`resolve` and, if it
    re-encoded, :func:`decode` yourself)."""
    _require_cuda_f32(g)
    n = g.numel()
    if not 0 <= k <= n:
        raise ValueError(f"k={k} outside [0, {n}]")
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=g.device)
    _require_cuda_f32(out, "out")
    if out.numel() != n:
        raise ValueError("out must have n elements")
    if packet is None:
        packet = Packet.alloc(n, L.FC_FMT_IDXVAL, g.device, k=k)
    if k == 0 or k >= n:                       # trivial thresholds: the exact engine's packet
        encode_top(g, k, packet=packet, check=check)
        return packet, decode(packet, out=out)
    lib = L.load()
    ws = Workspace.get(n, g.device)
    packet.k = k
    L.check(lib.fc_topk_encode_decode(_vp(g), n, k, _vp(packet.idx), _vp(packet.val),
                                      packet.capacity, _vp(packet.cnt), _vp(packet.qoff),
                                      _vp(packet.hdr), _vp(ws.buf), ws.nbytes, _vp(out),
                                      _stream(g.device)), "fc_topk_encode_decode")
    packet._enc = (g, k, L.FC_KEY_MAGNITUDE, 0, 0)
    packet._dense_only = False
    if check and resolve([packet]):            # bracket missed: exact packet, then decode
        decode(packet, out=out)
    return packet, out


def compress_top_dense(g: torch.Tensor, k: int, out: Optional[torch.Tensor] = None,
                       packet: Optional[Packet] = None, check: bool = True) -> torch.Tensor:
    """compression.py:31-37 on the device, straight to the dense q (fc_topk_encode_dense):
    one pass streams q (the packet buffers are scratch: no entries are written, the header
    says FC_FMT_DENSE), the resolve zeroes the slack.  Same bytes as
    ``decode(encode_top(g, k))``.  ``check=False`` skips the status read (call :func:`resolve`
    — it re-encodes a full packet — + :func:`decode` yourself if the header reports a retry)."""
    _require_cuda_f32(g)
    n = g.numel()
    if not 0 <= k <= n:
        raise ValueError(f"k={k} outside [0, {n}]")
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=g.device)
    _require_cuda_f32(out, "out")
    if out.numel() != n:
        raise ValueError("out must have n elements")
    if packet is None:
        packet = Packet.alloc(n, L.FC_FMT_IDXVAL, g.device, k=k)
    if k == 0 or k >= n:                       # trivial thresholds: packet path
        return decode(encode_top(g, k, packet=packet), out=out)
    lib = L.load()
    ws = Workspace.get(n, g.device)
    packet.k = k
    L.check(lib.fc_topk_encode_dense(_vp(g), n, k, _vp(packet.idx), _vp(packet.val),
                                     packet.capacity, _vp(packet.cnt), _vp(packet.qoff),
                                     _vp(packet.hdr), _vp(ws.buf), ws.nbytes, _vp(out),
                                     _stream(g.device)), "fc_topk_encode_dense")
    packet._enc = (g, k, L.FC_KEY_MAGNITUDE, 0, 0)
    packet._dense_only = True
    if check and resolve([packet]):            # bracket missed: exact packet, then decode
        decode(packet, out=out)
    return out


class BatchWorkspace:
    """Scratch for fc_topk_encode_batch: one encoder state per client (zeroed once)."""

    _cache: dict = {}

    def __init__(self, n: int, m: int, device: torch.device):
        lib = L.load()
        self.n, self.m = n, m
        self.nbytes = int(lib.fc_workspace_bytes_batch(n, m))
        self.buf = torch.empty(self.nbytes, dtype=torch.uint8, device=device)
        L.check(lib.fc_workspace_init(_vp(self.buf), self.nbytes, _stream(device)),
                "fc_workspace_init")

    @classmethod
    def get(cls, n: int, m: int, device: torch.device, slot: int = 0) -> "BatchWorkspace":
        """One workspace per (device, stream, n, slot): ``slot`` = the sub-batch index, so two
        sub-batches dealt to one stream never share encoder state between a SAMPLE part and
        its FINISH part."""
        key = (device.index if device.index is not None else torch.cuda.current_device(),
               torch.cuda.current_stream(device).cuda_stream, n, slot)
        ws = cls._cache.get(key)
        if ws is None or ws.m < m:
            ws = cls(n, m, device)
            cls._cache[key] = ws
        return ws


_SIDE: dict = {}
_MAX_SIDE = 4          # GPU_MAX_HW_QUEUES is 4: more forked streams would share queues
# k_fused_mag / k_fused64 (the lone magnitude encodes) hold workgroups in a bounded in-kernel
# wait; the library orders those launches per device itself (include/fedcodec.h, Concurrency),
# so any stream may issue them.  A graph replay is bracketed by fc_fused_order_begin / _end.


def _side_streams(dev: torch.device, count: int = 2) -> list:
    """Forked streams for :func:`encode_top_batch` sub-batches (created once per device)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    lst = _SIDE.setdefault(key, [])
    while len(lst) < count:
        lst.append(torch.cuda.Stream(device=dev))
    return lst[:count]


def encode_jobs(grads: Sequence[torch.Tensor], packets: Sequence[Packet], seeds=None,
                offsets=None) -> torch.Tensor:
    """Device array of fc_encode_job (build once, reuse while the buffers live)."""
    m = len(grads)
    seeds = seeds if seeds is not None else [0] * m
    offsets = offsets if offsets is not None else [0] * m
    arr = (L.EncodeJob * m)(*[
        L.EncodeJob(g=g.data_ptr(), idx=p.idx.data_ptr(), val=p.val.data_ptr(),
                    cnt=p.cnt.data_ptr(), hdr=p.hdr.data_ptr(), seed=int(s), offset=int(o),
                    qoff=p.qoff.data_ptr() if p.qoff is not None else 0)
        for g, p, s, o in zip(grads, packets, seeds, offsets)])
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.to(grads[0].device)


def encode_top_batch(grads: Sequence[torch.Tensor], k: int, *,
                     key_mode: int = L.FC_KEY_MAGNITUDE, seeds=None, offsets=None,
                     packets: Optional[Sequence[Packet]] = None,
                     jobs: Optional[torch.Tensor] = None, check: bool = True,
                     streams: int = 1, groups: Optional[Sequence[int]] = None,
                     part: int = L.FC_PART_SAMPLE | L.FC_PART_FINISH, fork: bool = True,
                     join: bool = True) -> list:
    """Top-k (or native rand-k) of M equal-length gradients in ONE launch per pipeline stage
    (fc_topk_encode_batch).  Same packets, bit for bit, as M calls of :func:`encode_top`.
    ``jobs``: a prebuilt :func:`encode_jobs` array for these exact grads/packets.
    ``streams``: sub-batches launched on that many forked streams (joined before return),
    free to run concurrently (the batched kernels never wait in-kernel);
    ``groups``: sub-batch sizes (default: ``streams`` equal parts), dealt to the streams in turn.
    Pipelining (bench.py): ``part`` = FC_PART_SAMPLE or FC_PART_FINISH runs one half of the
    pipeline (fc_topk_encode_batch_part; the same ``groups`` / ``streams`` for both halves, so
    each sub-batch's halves share a stream and its own workspace, keyed by the sub-batch index
    even when more sub-batches than streams share one stream); ``fork=False``: the forked
    streams do not wait for the caller's stream first; ``join=False``: the caller's stream does
    not wait for them (the caller orders later work itself)."""
    if not grads:
        raise ValueError("no gradients")
    lib = L.load()
    n, dev = grads[0].numel(), grads[0].device
    # per-tensor checks once per (jobs table, gradient / packet set): a 128-client step spent
    # ~1 ms of host time in them, which shows as GPU idle time when a step is short (16 M).  The
    # table remembers the checked objects by weak reference and compares identity (not id():
    # CPython reuses the ids of collected objects; a per-tensor signature tuple cost ~1.3 ms
    # per 128-client call, which doubled configs[2]'s step)
    def _same(refs, objs):
        return refs is not None and len(refs) == len(objs) and all(r() is o for r, o in zip(refs, objs))
    checked = (jobs is not None and getattr(jobs, "_fc_checked_n", None) == n
               and _same(getattr(jobs, "_fc_grefs", None), grads)
               and (packets is None or _same(getattr(jobs, "_fc_prefs", None), packets)))
    if not checked:
        for g in grads:
            _require_cuda_f32(g)
            if g.numel() != n or g.device != dev:
                raise ValueError("batched gradients must share length and device")
    if not 0 <= k <= n:
        raise ValueError(f"k={k} outside [0, {n}]")
    m = len(grads)
    seeds = seeds if seeds is not None else [0] * m
    offsets = offsets if offsets is not None else [0] * m
    if packets is None:
        packets = [Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k) for _ in range(m)]
    if len(packets) != m:
        raise ValueError("one packet per gradient")
    if part != (L.FC_PART_SAMPLE | L.FC_PART_FINISH) and (k == 0 or k == n or n < 2 or check):
        raise ValueError("a partial batch encode needs 0 < k < n and check=False")
    if k == 0 or k == n or n < 2:                    # trivial thresholds: exact engine per client
        return [encode_top(g, k, key_mode=key_mode, seed=s, offset=o, packet=p, check=check)
                for g, p, s, o in zip(grads, packets, seeds, offsets)]
    cap = int(lib.fc_packet_capacity(n))
    for p, g, s, o in zip(packets, grads, seeds, offsets):
        if not checked and (p.capacity < cap or p.fmt != L.FC_FMT_IDXVAL):
            raise ValueError("packet too small or not idx/val")
        p.k = k
        p._enc = (g, k, key_mode, s, o)
        p._dense_only = False
    if jobs is None:
        jobs = encode_jobs(grads, packets, seeds, offsets)
    elif not checked:
        jobs._fc_checked_n = n
        jobs._fc_grefs = [weakref.ref(g) for g in grads]
        jobs._fc_prefs = [weakref.ref(p) for p in packets]
    nside = max(1, min(int(streams), m, _MAX_SIDE))
    if groups is None:
        groups = [(i + 1) * m // nside - i * m // nside for i in range(nside)]
    groups = [int(x) for x in groups]
    if any(x < 1 for x in groups) or sum(groups) != m:
        raise ValueError(f"groups {groups} must be positive sizes summing to {m} clients")
    if nside == 1 or len(groups) == 1:
        ws = BatchWorkspace.get(n, m, dev)
        L.check(lib.fc_topk_encode_batch_part(_vp(jobs), m, n, k, key_mode, packets[0].capacity,
                                              _vp(ws.buf), ws.nbytes, part, _stream(dev)),
                "fc_topk_encode_batch")
    else:
        # Sub-batches on forked streams (group i on stream i % streams), free to overlap.
        # Packets are identical; the caller's stream joins every fork before this returns, so
        # later work (and frees) stay ordered.
        main = torch.cuda.current_stream(dev)
        job_bytes = ctypes.sizeof(L.EncodeJob)
        base = jobs.data_ptr()
        sides = _side_streams(dev, nside)
        if fork:
            ev = torch.cuda.Event()
            ev.record(main)
            for side in sides:
                side.wait_event(ev)
        lo = 0
        for i, size in enumerate(groups):
            side = sides[i % nside]
            with torch.cuda.stream(side):
                ws = BatchWorkspace.get(n, size, dev, slot=i)
                L.check(lib.fc_topk_encode_batch_part(ctypes.c_void_p(base + lo * job_bytes),
                                                      size, n, k, key_mode, packets[0].capacity,
                                                      _vp(ws.buf), ws.nbytes, part, _stream(dev)),
                        "fc_topk_encode_batch")
            lo += size
        if join:
            for side in sides:
                main.wait_stream(side)
    if check:
        resolve(packets)
    return list(packets)


def encode_fold_batch(grads: Sequence[torch.Tensor], k: int, weights, out: torch.Tensor, *,
                      packets: Sequence[Packet], jobs: Optional[torch.Tensor] = None,
                      views: Optional[torch.Tensor] = None, streams: int = 2,
                      status: Optional[tuple] = None) -> "torch.cuda.Event":
    """Batched top-k encode of M gradients AND their packet FedAVG fold (gar.py:44), pipelined:
    sub-batch i is encoded on forked stream i and folded there as soon as it is encoded,
    continuing sub-batch i-1's partial sum (an event orders the folds, so the rows are added
    in G's order: bit-identical to :func:`encode_top_batch` + :func:`decode_accumulate`), while
    sub-batch i+1 encodes on its own stream.  ``out`` holds the aggregate once the
    caller's stream (joined at return) reaches it.  Returns an event recorded once every
    sub-batch is ENCODED (the folds may still run); ``status=(src, dst)``: ``dst.copy_(src)``
    (e.g. the packet headers' status words into pinned host memory) is queued right then, so
    the host can check the statuses while the last fold runs.  No re-encode here: call
    :func:`resolve` and, if it re-encoded anything, fold again (bench.py does)."""
    lib = L.load()
    m = len(grads)
    if m == 0 or len(packets) != m:
        raise ValueError("one packet per gradient, at least one")
    n, dev = grads[0].numel(), grads[0].device
    if not 0 < k < n:
        raise ValueError("encode_fold_batch needs 0 < k < n")
    weights = [float(x) for x in weights]
    if len(weights) != m:
        raise ValueError("one weight per gradient")
    if jobs is None:
        jobs = encode_jobs(grads, packets)
    if views is None:
        views = views_tensor(packets, weights, dev)
    nside = max(1, min(int(streams), m, _MAX_SIDE))
    groups = [(i + 1) * m // nside - i * m // nside for i in range(nside)]
    jb, vb = ctypes.sizeof(L.EncodeJob), ctypes.sizeof(L.PacketView)
    main = torch.cuda.current_stream(dev)
    sides = _side_streams(dev, nside)
    start = torch.cuda.Event()
    start.record(main)
    prev = None
    encoded = []
    lo = 0
    for i, size in enumerate(groups):
        hi = lo + size
        side = sides[i]
        with torch.cuda.stream(side):
            side.wait_event(start)
            ws = BatchWorkspace.get(n, size, dev, slot=i)
            L.check(lib.fc_topk_encode_batch(ctypes.c_void_p(jobs.data_ptr() + lo * jb), size, n,
                                             k, L.FC_KEY_MAGNITUDE, packets[0].capacity,
                                             _vp(ws.buf), ws.nbytes, _stream(dev)),
                    "fc_topk_encode_batch")
            for p, g in zip(packets[lo:hi], grads[lo:hi]):
                p.k = k
                p._enc = (g, k, L.FC_KEY_MAGNITUDE, 0, 0)
            ev = torch.cuda.Event()
            ev.record(side)
            encoded.append(ev)
            if i == len(groups) - 1:                       # every sub-batch is encoded here
                for e in encoded[:-1]:
                    side.wait_event(e)
                if status is not None:
                    status[1].copy_(status[0], non_blocking=True)
                done = torch.cuda.Event()
                done.record(side)
            if prev is not None:
                side.wait_event(prev)                      # folds in G's row order
            fn = lib.fc_decode_accumulate_continue if i else lib.fc_decode_accumulate
            L.check(fn(ctypes.c_void_p(views.data_ptr() + lo * vb), size, L.FC_FMT_IDXVAL, n,
                       _vp(out), _stream(dev)), "fc_decode_accumulate")
            prev = torch.cuda.Event()
            prev.record(side)
        lo = hi
    main.wait_event(prev)
    for side in sides:                                     # later frees stay ordered
        main.wait_stream(side)
    return done


class GraphedCalls:
    """A sequence of codec calls on fixed tensors, captured once into one HIP graph and replayed
    (the hipGraph form of a launch-bound inner loop).  Replays launch the same kernels on the
    same buffers without the host's per-call work and with cheaper kernel boundaries: a lone
    16 M drop-in dense top-k 48.6 -> 45.0 us per call, the packet encode + decode 60.1 -> 56.7 us
    (tools/graph_probe.py, profiles/r05_graph_probe.jsonl).

    ``fn`` issues the calls (``check=False`` throughout: a status check synchronises, which a
    capture cannot; call :func:`resolve` after a replay).  Every tensor ``fn`` touches must stay
    alive at the same address.  The encoder state in the workspaces is self-cleaning, so each
    replay computes what the eager calls would; the workspace is the capture stream's, so do not
    run eager encodes of the same size on that stream concurrently with a replay."""

    def __init__(self, fn, device: Optional[torch.device] = None, warmup: int = 2):
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.stream = torch.cuda.Stream(dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self.stream):
            for _ in range(warmup):                      # workspaces, packets, first-call setup
                fn()
        self.stream.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: another thread's stream work (e.g. a process group's watchdog polling
        # its events) is not an error during this capture
        with torch.cuda.graph(self.graph, stream=self.stream, capture_error_mode="thread_local"):
            fn()
        torch.cuda.current_stream(dev).wait_stream(self.stream)

    def replay(self) -> None:
        """Launch the captured calls on the current stream, ordered after the device's last
        in-kernel-waiting encode (fc_fused_order_begin / _end: the library's own ordering does
        not see launches inside a graph)."""
        lib = L.load()
        s = _stream(self.stream.device)
        L.check(lib.fc_fused_order_begin(s), "fc_fused_order_begin")
        self.graph.replay()
        L.check(lib.fc_fused_order_end(s), "fc_fused_order_end")


def resolve(packets: Sequence[Packet]) -> int:
    """Re-encode (exact path) every top/rand packet whose sampled bracket missed.
    Returns the number of packets that needed the exact path."""
    lib = L.load()
    redo = 0
    for p, h in zip(packets, headers(packets)):       # one sync for the whole batch
        if h.status == L.FC_STATUS_OK:
            continue
        if h.status != L.FC_STATUS_RETRY_EXACT or getattr(p, "_enc", None) is None:
            raise L.FedCodecError(f"packet status {h.status}")
        g, k, key_mode, seed, offset = p._enc
        ws = Workspace.get(g.numel(), g.device)
        L.check(lib.fc_topk_encode_exact(_vp(g), g.numel(), k, key_mode, seed, offset,
                                         _vp(p.idx), _vp(p.val), p.capacity, _vp(p.cnt),
                                         _vp(p.qoff), _vp(p.hdr), _vp(ws.buf), ws.nbytes,
                                         _stream(g.device)), "fc_topk_encode_exact")
        redo += 1
        p._dense_only = False                        # a full packet now
        h2 = p.header()
        if h2.status != L.FC_STATUS_OK:
            raise L.FedCodecError(f"exact encode status {h2.status}")
    return redo


def encode_mask(g: torch.Tensor, codec: int, *, p: float = 0.5,
                mask_bits: Optional[torch.Tensor] = None, seed: int = 0, offset: int = 0,
                fmt: int = L.FC_FMT_BITMAP, packet: Optional[Packet] = None) -> Packet:
    """Mask codecs: dropout-biased / dropout-unbiased (Philox or host mask) and rand-k with a
    host-drawn permutation mask (parity mode).  ``mask_bits``: int32 device tensor, bit i of
    word i//32 = element i."""
    _require_cuda_f32(g)
    lib = L.load()
    n = g.numel()
    ws = Workspace.get(n, g.device)
    if mask_bits is not None and (mask_bits.dtype != _U32 or not mask_bits.is_cuda
                                  or mask_bits.numel() * 32 < n):
        raise ValueError("mask_bits must be an int32 CUDA tensor of ceil(n/32) words")
    if packet is None:
        packet = Packet.alloc(n, fmt, g.device)
    L.check(lib.fc_mask_encode(_vp(g), n, codec, _vp(mask_bits), float(p), seed, offset, fmt,
                               _vp(packet.idx), _vp(packet.val), _vp(packet.bitmap),
                               packet.capacity, _vp(packet.cnt), _vp(packet.qoff),
                               _vp(packet.hdr), _vp(ws.buf), ws.nbytes, _stream(g.device)),
            "fc_mask_encode")
    return packet


def decode(packet: Packet, out: Optional[torch.Tensor] = None,
           dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """Dense reconstruction (the array compress() returns)."""
    lib = L.load()
    dev = packet.val.device
    if out is None:
        out = torch.empty(packet.n, dtype=dtype, device=dev)
    if out.dtype not in (torch.float32, torch.float64) or out.numel() != packet.n:
        raise ValueError("out must be float32/float64 with n elements")
    v = packet.view()
    L.check(lib.fc_decode_dense(ctypes.byref(v), packet.fmt, packet.n, _vp(out),
                                int(out.dtype == torch.float64), _stream(dev)),
            "fc_decode_dense")
    return out


def views_tensor(packets: Sequence[Packet], weights, device) -> torch.Tensor:
    """Device array of fc_packet_view (client order = G row order)."""
    arr = (L.PacketView * len(packets))(*[p.view(w) for p, w in zip(packets, weights)])
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.to(device)


def decode_accumulate(packets: Sequence[Packet], weights, out: Optional[torch.Tensor] = None,
                      views: Optional[torch.Tensor] = None,
                      continue_sum: bool = False) -> torch.Tensor:
    """FedAVG over packets: bit-exact ``np.sum(G * w[:, None], axis=0)`` (gar.py:44).

    ``continue_sum=True`` folds the packets into the partial sum already in ``out`` (rows of
    G that an earlier call, or an earlier rank of the chained reduce, has summed)."""
    lib = L.load()
    if not packets:
        raise ValueError("no packets")
    fmt, n, dev = packets[0].fmt, packets[0].n, packets[0].val.device
    if any(p.fmt != fmt or p.n != n for p in packets):
        raise ValueError("packets must share n and format")
    if out is None:
        if continue_sum:
            raise ValueError("continue_sum needs the partial sum in `out`")
        out = torch.empty(n, dtype=torch.float32, device=dev)
    _require_cuda_f32(out, "out")
    if out.numel() != n:
        raise ValueError("out must have n elements")
    if views is None:
        views = views_tensor(packets, weights, dev)
    fn = lib.fc_decode_accumulate_continue if continue_sum else lib.fc_decode_accumulate
    L.check(fn(_vp(views), len(packets), fmt, n, _vp(out), _stream(dev)),
            "fc_decode_accumulate")
    return out


def weighted_sum_dense(rows, weights: torch.Tensor, out: Optional[torch.Tensor] = None,
                       out_dtype: Optional[torch.dtype] = None, continue_sum: bool = False):
    """gar.py:44 on dense device rows (a (M, N) tensor or a list of 1-D tensors).

    float32 rows and float32 weights: fp32 arithmetic (k_wsum).  Anything float64 (rows,
    weights or ``out_dtype``): NumPy's promotion of ``G * w`` to float64, fp64 arithmetic
    (k_wsum64); the result is float64.  ``continue_sum``: ``out`` holds the sum of earlier
    rows and these rows continue it (same bits as one call over all rows)."""
    lib = L.load()
    if isinstance(rows, torch.Tensor):
        rows = list(rows.unbind(0))
    rdt = rows[0].dtype
    if rdt not in (torch.float32, torch.float64) or any(r.dtype != rdt for r in rows):
        raise TypeError("rows must all be float32 or all float64")
    f64 = rdt == torch.float64 or weights.dtype == torch.float64 or out_dtype == torch.float64
    for r in rows:
        _require_cuda_f32(r, "row", align=4 if rdt == torch.float32 else 8, dtype=rdt)
    n, dev = rows[0].numel(), rows[0].device
    if any(r.numel() != n for r in rows):
        raise ValueError("rows must have equal length")
    ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64).to(dev)
    odt = torch.float64 if f64 else torch.float32
    if out is None:
        if continue_sum:
            raise ValueError("continue_sum needs the partial sum in `out`")
        out = torch.empty(n, dtype=odt, device=dev)
    if out.dtype != odt or out.numel() != n or not out.is_cuda:
        raise ValueError(f"out must be a CUDA {odt} tensor of {n} elements")
    if f64:
        w = weights.to(device=dev, dtype=torch.float64).contiguous()   # exact for fp32 weights
        L.check(lib.fc_weighted_sum_dense_f64(_vp(ptrs), int(rdt == torch.float64), _vp(w),
                                              len(rows), n, _vp(out), int(continue_sum),
                                              _stream(dev)), "fc_weighted_sum_dense_f64")
        return out
    w = weights.to(device=dev, dtype=torch.float32).contiguous()
    fn = lib.fc_weighted_sum_dense_continue if continue_sum else lib.fc_weighted_sum_dense
    L.check(fn(_vp(ptrs), _vp(w), len(rows), n, _vp(out), _stream(dev)), "fc_weighted_sum_dense")
    return out


def div_scalar(x: torch.Tensor, d: float) -> torch.Tensor:
    """x = fl(x / d) in place, in x's dtype (the count division of np.mean, aggregation.py:91)."""
    lib = L.load()
    if x.dtype == torch.float64:
        _require_cuda_f32(x, "x", align=8, dtype=torch.float64)
        L.check(lib.fc_div_scalar_f64(_vp(x), x.numel(), float(d), _stream(x.device)),
                "fc_div_scalar_f64")
        return x
    _require_cuda_f32(x, "x")
    L.check(lib.fc_div_scalar(_vp(x), x.numel(), ctypes.c_float(d), _stream(x.device)),
            "fc_div_scalar")
    return x


# ---- float64 gradients (attack_models.py:105-106 -> aggregation.py:61) ----------------------
def _f64_status(out: torch.Tensor) -> torch.Tensor:
    """The device status word of ONE output (k_compact64 sets it OK, k_resolve64 raises it to
    RETRY): each output keeps its own, so several unchecked encodes are each resolvable."""
    st = getattr(out, "_fc_f64_status", None)
    if st is None or st.device != out.device:
        st = torch.empty(1, dtype=_U32, device=out.device)
        out._fc_f64_status = st
    return st


def compress_top_dense_f64(g: torch.Tensor, k: int, *, key_mode: int = L.FC_KEY_MAGNITUDE,
                           seed: int = 0, offset: int = 0,
                           out: Optional[torch.Tensor] = None, check: bool = True,
                           exact: bool = False) -> torch.Tensor:
    """compression.py:31-37 ('top') / native 'rand' (PHILOX keys) on a float64 gradient: the
    dense float64 q (same tie rule as fp32).  'top' with 0 < k < n takes the sampled path
    (fc_topk_dense_f64_sampled: one streaming pass); ``check=True`` reads its status (one
    sync) and re-runs a missed bracket exactly; with ``check=False`` call
    :func:`resolve_f64` on the output later (each output has its own status word).  Native rand-k, trivial k and
    ``exact=True``: the exact radix select (fc_topk_dense_f64)."""
    _require_cuda_f32(g, align=8, dtype=torch.float64)
    n = g.numel()
    if not 0 <= k <= n:
        raise ValueError(f"k={k} outside [0, {n}]")
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=g.device)
    _require_cuda_f32(out, "out", align=8, dtype=torch.float64)
    if out.numel() != n:
        raise ValueError("out must have n elements")
    lib = L.load()
    ws = Workspace.get(n, g.device)
    sampled = (not exact and key_mode == L.FC_KEY_MAGNITUDE and 0 < k < n
               and g.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0)
    if sampled:
        st = _f64_status(out)
        L.check(lib.fc_topk_dense_f64_sampled(_vp(g), n, k, _vp(out), _vp(ws.buf), ws.nbytes,
                                              _vp(st), _stream(g.device)),
                "fc_topk_dense_f64_sampled")
        out._fc_f64_enc = (g, k)
        if check:
            resolve_f64(out)
        return out
    L.check(lib.fc_topk_dense_f64(_vp(g), n, k, key_mode, seed, offset, _vp(out), _vp(ws.buf),
                                  ws.nbytes, _stream(g.device)), "fc_topk_dense_f64")
    return out


def resolve_f64(out: torch.Tensor) -> int:
    """After a sampled fp64 encode into ``out`` (check=False): if its bracket missed (the
    output's own status word), redo it exactly into ``out``.  Returns 1 if it did, else 0."""
    st = getattr(out, "_fc_f64_status", None)
    if st is None or getattr(out, "_fc_f64_enc", None) is None:
        return 0                                   # not a sampled encode's output
    if int(st.item()) == L.FC_STATUS_OK:
        return 0
    g, k = out._fc_f64_enc
    compress_top_dense_f64(g, k, out=out, exact=True)
    return 1


def mask_dense_f64(g: torch.Tensor, codec: int, *, p: float = 0.5,
                   mask_bits: Optional[torch.Tensor] = None, seed: int = 0, offset: int = 0,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """'rand' (host permutation mask) and 'dropout-*' on a float64 OR float32 gradient, with
    the reference's float64 arithmetic (g * mask, (g * mask) / p; a float32 g is promoted
    exactly, as NumPy does): fc_mask_dense_f64 / fc_mask_dense_f32.  Result: float64."""
    f32 = isinstance(g, torch.Tensor) and g.dtype == torch.float32
    if f32:
        _require_cuda_f32(g, align=4)
    else:
        _require_cuda_f32(g, align=8, dtype=torch.float64)
    n = g.numel()
    if mask_bits is not None and (mask_bits.dtype != _U32 or not mask_bits.is_cuda
                                  or mask_bits.numel() * 32 < n):
        raise ValueError("mask_bits must be an int32 CUDA tensor of ceil(n/32) words")
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=g.device)
    _require_cuda_f32(out, "out", align=8, dtype=torch.float64)
    if out.numel() != n:
        raise ValueError("out must have n elements")
    lib = L.load()
    fn = lib.fc_mask_dense_f32 if f32 else lib.fc_mask_dense_f64
    L.check(fn(_vp(g), n, codec, _vp(mask_bits), float(p), seed, offset, _vp(out),
               _stream(g.device)), "fc_mask_dense_f32" if f32 else "fc_mask_dense_f64")
    return out


# ---- QSGD (compression.py:62-74; opt-in, parity unpinned: oracle/qsgd_oracle.py) ----------
@dataclass
class QsgdPacket:
    codes: torch.Tensor          # uint32[fc_qsgd_code_words(n, bits)]
    hdr: torch.Tensor            # uint8[HDR_BYTES]
    n: int
    bits: int

    @classmethod
    def alloc(cls, n: int, bits: int, device) -> "QsgdPacket":
        lib = L.load()
        words = int(lib.fc_qsgd_code_words(n, bits))
        if words == 0:
            raise ValueError(f"bits={bits} outside [1, 14]")
        return cls(torch.empty(words, dtype=torch.int32, device=device),
                   torch.zeros(L.HDR_BYTES, dtype=torch.uint8, device=device), n, bits)

    def view(self, weight: float = 1.0) -> L.PacketView:
        v = L.PacketView()
        v.idx = self.codes.data_ptr()
        v.hdr = self.hdr.data_ptr()
        v.weight = weight
        return v

    def header(self) -> L.PacketHdr:
        return L.PacketHdr.from_buffer_copy(bytes(self.hdr.cpu().numpy()))


_QSGD_WS = {}


def encode_qsgd(g: torch.Tensor, bits: int, *, seed: int = 0, offset: int = 0,
                packet: Optional[QsgdPacket] = None) -> QsgdPacket:
    """QSGD codes of a device gradient (two streaming passes: ||g||, then quantise)."""
    lib = L.load()
    _require_cuda_f32(g)
    n, dev = g.numel(), g.device
    if packet is None:
        packet = QsgdPacket.alloc(n, bits, dev)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(),
           torch.cuda.current_stream(dev).cuda_stream)        # k_qsgd_norm's ticket: per stream
    ws = _QSGD_WS.get(key)
    if ws is None:
        ws = _QSGD_WS[key] = torch.zeros(int(lib.fc_qsgd_workspace_bytes()), dtype=torch.uint8,
                                         device=dev)
    L.check(lib.fc_qsgd_encode(_vp(g), n, bits, seed, offset, _vp(packet.codes),
                               packet.codes.numel(), _vp(packet.hdr), _vp(ws), ws.numel(),
                               _stream(dev)), "fc_qsgd_encode")
    return packet


def decode_qsgd(packet: QsgdPacket, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    lib = L.load()
    dev = packet.codes.device
    if out is None:
        out = torch.empty(packet.n, dtype=torch.float32, device=dev)
    _require_cuda_f32(out, "out")
    v = packet.view()
    L.check(lib.fc_qsgd_decode(ctypes.byref(v), packet.n, _vp(out), _stream(dev)), "fc_qsgd_decode")
    return out


def decode_accumulate_qsgd(packets: Sequence[QsgdPacket], weights, out: Optional[torch.Tensor] = None,
                           continue_sum: bool = False) -> torch.Tensor:
    """FedAVG over QSGD packets: gar.py:44 on the dense rows they decode to (bit-exact)."""
    lib = L.load()
    if not packets:
        raise ValueError("no packets")
    n, dev = packets[0].n, packets[0].codes.device
    if any(p.n != n for p in packets):
        raise ValueError("packets must share n")
    if out is None:
        if continue_sum:
            raise ValueError("continue_sum needs the partial sum in `out`")
        out = torch.empty(n, dtype=torch.float32, device=dev)
    _require_cuda_f32(out, "out")
    arr = (L.PacketView * len(packets))(*[p.view(float(w)) for p, w in zip(packets, weights)])
    views = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
    L.check(lib.fc_qsgd_decode_accumulate(_vp(views), len(packets), n, _vp(out),
                                          int(continue_sum), _stream(dev)),
            "fc_qsgd_decode_accumulate")
    return out


# ---- NumPy's legacy MT19937 stream on the device (the reference's dropout draws) -------------
class MtPlan:
    """The jump polynomials of gradient length n on one device (fc_mt_plan), for up to
    ``rows`` rows per round; kept per (device, n) and grown on demand."""

    _cache: dict = {}
    _lock = threading.Lock()

    def __init__(self, n: int, rows: int, device: torch.device):
        lib = L.load()
        self.n, self.rows = n, rows
        self.nbytes = int(lib.fc_mt_plan_bytes(n, rows))
        self.buf = torch.empty(self.nbytes, dtype=torch.uint8, device=device)
        L.check(lib.fc_mt_plan(n, rows, _vp(self.buf), self.nbytes, _stream(device)), "fc_mt_plan")

    @classmethod
    def get(cls, n: int, rows: int, device: torch.device) -> "MtPlan":
        key = (device.index if device.index is not None else torch.cuda.current_device(), n)
        with cls._lock:
            p = cls._cache.get(key)
            if p is None or p.rows < rows:
                p = cls(n, max(rows, 2 * p.rows if p is not None else rows), device)
                cls._cache[key] = p
            return p


class MtRound:
    """``rows`` consecutive ``np.random.binomial(1, p_r, (n,))`` draws (compression.py:51, :58)
    generated on the device from the legacy state (key, pos) of ``np.random.get_state()``
    (fc_mt_begin / fc_mt_binomial): row r's mask words equal the host draw's
    ``bitmask_words(mask, n, True)``.  :meth:`end_state` gives the state np.random is left in
    (and whether NumPy would have redrawn somewhere: the caller then draws on the host)."""

    def __init__(self, n: int, rows: int, key: np.ndarray, pos: int,
                 device: Optional[torch.device] = None):
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        lib = L.load()
        self.n, self.rows, self.dev = n, rows, dev
        self.plan = MtPlan.get(n, rows, dev)
        self.nbytes = int(lib.fc_mt_workspace_bytes(rows))
        self.ws = torch.empty(self.nbytes, dtype=torch.uint8, device=dev)
        self._key = np.ascontiguousarray(np.asarray(key, dtype=np.uint32))
        if self._key.shape != (624,):
            raise ValueError("an MT19937 key has 624 words")
        with torch.cuda.device(dev):
            L.check(lib.fc_mt_begin(_vp(self.plan.buf), self.plan.nbytes, n, rows,
                                    self._key.ctypes.data_as(ctypes.c_void_p), int(pos),
                                    _vp(self.ws), self.nbytes, _stream(dev)), "fc_mt_begin")
        self._events = []                   # after begin and each row: end_state() waits on them
        self._mark()
        self._begin = (self._events[0], torch.cuda.current_stream(dev))

    def _mark(self) -> None:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        self._events.append(ev)
        if len(self._events) > 8:
            self._events = [e for e in self._events if not e.query()] or self._events[-1:]

    def binomial(self, row: int, p: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Row ``row``'s mask as int32 bit words (ceil(n/32)) on the current stream."""
        if out is None:
            out = torch.empty((self.n + 31) // 32, dtype=torch.int32, device=self.dev)
        cur = torch.cuda.current_stream(self.dev)
        if cur != self._begin[1]:           # rows may be drawn on other streams (DeviceRing)
            cur.wait_event(self._begin[0])
        lib = L.load()
        L.check(lib.fc_mt_binomial(_vp(self.plan.buf), self.plan.nbytes, self.n, self.rows, int(row),
                                   float(p), _vp(out), _vp(self.ws), self.nbytes,
                                   _stream(self.dev)), "fc_mt_binomial")
        self._mark()
        return out

    def end_state(self):
        """(key uint32[624], pos, redraw) after the round: waits for begin and every row
        launched so far (the redraw flag covers those rows)."""
        for ev in self._events:
            ev.synchronize()
        raw = self.ws[:624 * 4 + 16].cpu().numpy()
        words = raw.view(np.uint32)
        return words[:624].copy(), int(words[624]), bool(words[625])


def mt_state():
    """np.random's legacy state as (key, pos, has_gauss, gauss); ValueError if not MT19937."""
    st = np.random.get_state()
    if st[0] != "MT19937":
        raise ValueError("np.random is not an MT19937 RandomState")
    return np.asarray(st[1], dtype=np.uint32), int(st[2]), int(st[3]), float(st[4])


def mt_set_state(key: np.ndarray, pos: int, has_gauss: int, gauss: float) -> None:
    np.random.set_state(("MT19937", np.asarray(key, dtype=np.uint32), int(pos), int(has_gauss),
                         float(gauss)))
