"""Host-resident FedAVG round: H2D -> top-k encode -> decode-accumulate -> D2H (BASELINE.json
configs[4], the path that "starts and ends in host memory").

The reference's round starts from client gradients in host memory (client.py:53 flattens to
NumPy) and hands the aggregate back to the server loop (aggregation.py:61-78 -> update_model,
aggregation.py:99).  :class:`HostFedAvg` streams the clients' host gradients through the GPU
without ever holding more than ``ring`` of them on the device:

* a copy stream moves client i's gradient into a device slot of the ring (H2D overlapped
  with the encodes of earlier clients); the compute stream waits for that copy, encodes
  (``fc_topk_encode``) into a packet of the current fold group and signals the slot free again;
* a gradient that is not already in pinned memory (the reference's ``client.grad`` is a plain
  NumPy array) is first copied by host threads into one of ``stage`` pinned buffers, which is
  reused once its H2D has completed — the host copy of client i+1 overlaps the H2D and encode
  of client i; ``pin="register"`` instead page-locks the caller's array in place for its DMA
  (hipHostRegister) and releases it after the copy;
* every ``group`` packets are folded into the running aggregate with
  ``fc_decode_accumulate_continue`` (one status read per group; a packet whose sampled bracket
  missed is re-encoded exactly from its host copy), so the sum is the same left-to-right fp32
  fold as gar.py:44 over all rows, bit for bit;
* the aggregate is copied D2H once at the end.

Device memory is bounded by ``ring`` gradients + ``sets`` x ``group`` packets + two aggregates
whatever the client count (:func:`plan_group` sizes ``group`` for a byte budget), so the device
``Aggregator.aggregate_grads`` (openmsftl_amd/aggregation.py) runs any number of sampled
clients through it.

Every codec of compression.py streams (:class:`RowCodec` per row of G, a :class:`RowPlan` for
the round): ``'top'`` and native ``'rand'`` rows are ``fc_topk_encode`` packets, ``'rand'`` with
the host permutation and ``'dropout-*'`` rows are ``fc_mask_encode`` idx/val packets (the mask
drawn on the host from the global ``np.random`` in row order, or Philox Bernoulli on the
device), and ``'full'`` rows are the gradient itself, copied H2D straight into the group's
packet value buffer and folded by ``fc_weighted_sum_dense_continue``.  A group's rows are folded
in row order, runs of packets by ``fc_decode_accumulate`` and runs of dense rows by the dense
sum, each continuing the running aggregate: one left-to-right fp32 fold (gar.py:44).

More than one GPU, still bit-exact (:class:`DeviceRing` in one process, :class:`RankRing`
across processes): the fold groups — rows ``[t*group, (t+1)*group)`` of G — are dealt to the
devices round-robin, and the running aggregate travels device to device in group order.  Each
device encodes its next group (the PCIe-bound part) while the aggregate is elsewhere; the fold
of group t continues exactly where group t-1's left it, so the result is one left-to-right
fold over all rows (gar.py:44), whatever the device count.  Only the folds (~0.1 ms) and the
4N-byte hops of the aggregate (~2 ms over xGMI at 25.5 M) are serial; the encodes (~117 ms per
64-client group at PCIe rate) overlap across devices.

Used also by tools/e2e_bench.py (the PCIe-inclusive rate, configs[4] at N ranks) and
tests/test_fullsize_parity.py / tests/test_e2e_multirank.py (the configs[4] digest).
"""
from __future__ import annotations

import ctypes
import threading
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Union

import numpy as np
import torch

from . import _lib as L
from . import codec
from .distributed import fedavg_weights

HostSource = Union[Sequence, Callable[[int], object]]


def packet_bytes(n: int) -> int:
    """Device bytes one idx/val packet of length n reserves (codec.Packet.alloc)."""
    lib = L.load()
    cap, nch = int(lib.fc_packet_capacity(n)), int(lib.fc_num_chunks(n))
    return cap * 6 + nch * 12 + L.HDR_BYTES


def plan_group(n: int, clients: int, budget_bytes: int, ring: int = 4,
               max_group: int = 64, sets: int = 1) -> int:
    """Packets per fold group so that ring gradients + ``sets`` x group packets + the
    aggregate and a scratch row (4N each) + one encoder workspace fit in ``budget_bytes``
    (at least 1)."""
    lib = L.load()
    fixed = (ring + 2) * 4 * n + int(lib.fc_workspace_bytes(n))
    g = (budget_bytes - fixed) // (packet_bytes(n) * max(1, sets))
    return int(max(1, min(max_group, clients, g)))


def group_bounds(clients: int, group: int) -> List[range]:
    """G's rows cut into fold groups of ``group`` (the last one shorter)."""
    return [range(g0, min(g0 + group, clients)) for g0 in range(0, clients, group)]


@dataclass(frozen=True)
class RowCodec:
    """How one row of G is made on the device from its client's gradient (compression.py:23-77).

    kind "top": fc_topk_encode packet of the k largest keys (``key_mode`` MAGNITUDE = 'top',
    PHILOX = native 'rand' keyed by ``seed``/``offset``); "mask": fc_mask_encode idx/val packet
    of codec ``codec`` (FC_CODEC_RAND / DROPOUT_*) with ``mask_src`` "host" (bits drawn on the
    host, :meth:`RowPlan.take_mask`), "mt" (np.random.binomial's own MT19937 draws made on the
    device, row ``offset`` of the plan's :class:`~openmsftl_amd.codec.MtRound`), "philox"
    (device Bernoulli(p)) or "none" (nothing kept: 'top' with k = 0); "dense": the gradient
    itself ('full', or 'top' with k = n)."""
    kind: str
    k: int = 0
    key_mode: int = 0
    seed: int = 0
    offset: int = 0
    codec: int = 0
    p: float = 0.0
    mask_src: str = "none"


class MtRedraw(RuntimeError):
    """NumPy's binomial would have redrawn a variate (probability ~2^-52 per element) in a
    device MT19937 round: its masks from that element on are not the reference's; redo the
    round with host draws (np.random is still at the round's start)."""


class RowPlan:
    """The row codecs of one round, and the host RNG draws of its 'rand' / 'dropout-*' rows.

    ``draws[i]()`` returns row i's mask as little-endian uint32 words (ceil(n/32)); the draws run
    on ONE producer thread in increasing row order — the order in which the reference's loop
    (aggregation.py:61-63) consumes the process-global ``np.random`` stream — at most
    ``lookahead`` rows ahead of the pipeline, into pinned buffers that the pipeline copies H2D.
    Several pipeline threads (:class:`DeviceRing`) may take masks; the draw order never
    changes.  :meth:`close` waits for the producer (every draw done: the RNG is then where the
    reference leaves it) and re-raises a draw's exception (e.g. NumPy's ValueError for p > 1).

    Error path: if the round fails for another reason (a FedCodecError, an H2D or
    allocation error) and the plan is closed with ``wait=False``, host draws may already have
    run up to ``lookahead`` rows past the failing row, so np.random is then further along than
    the reference's loop would have left it; device MT19937 rows ("mt") leave np.random at the
    round's start instead.  A caller that must resume the stream exactly after such an error
    saves ``np.random.get_state()`` before the round and restores it."""

    def __init__(self, n: int, specs: Sequence[RowCodec], draws: Optional[dict] = None,
                 lookahead: int = 8, base: int = 0, parent: "RowPlan" = None,
                 mt_rows: int = 0):
        self.n, self.specs, self.base = n, specs, base
        self._root = parent if parent is not None else self
        if parent is not None:
            return
        # device MT19937 rows ("mt"): the round's start state is np.random's now; close() leaves
        # np.random where the reference's loop would (the state after mt_rows binomial draws)
        self.mt_rows = mt_rows
        self._mt_start = codec.mt_state() if mt_rows else None
        self._mt_rounds = {}
        self._mt_lock = threading.Lock()
        self._mt_redraw = False
        self.draws = dict(draws or {})
        self.nwords = (n + 31) // 32
        self._cv = threading.Condition()
        self._ready = {}
        self._free = []
        self._pool = max(1, min(int(lookahead), len(self.draws)))
        self._made = 0
        self._err = None
        self._stop = False
        self._thread = None
        self._started = False
        self._keep = None

    def restrict(self, keep) -> None:
        """Only rows with ``keep(i)`` will be taken (a rank's own rows): the others are still
        drawn, in order, and dropped.  Call before the first :meth:`take_mask`."""
        if self._root._started:
            raise RuntimeError("restrict() after the draws started")
        self._root._keep = keep

    def _start(self) -> None:
        r = self._root
        with r._cv:
            if r._started or not r.draws:
                r._started = True
                return
            r._started = True
            r._thread = threading.Thread(target=r._produce, name="fc-row-draws", daemon=True)
            r._thread.start()

    def __call__(self, i: int) -> RowCodec:
        return self.specs[self.base + i]

    def __len__(self) -> int:
        return len(self.specs) - self.base

    def shifted(self, start: int) -> "RowPlan":
        """The plan of rows [start, ...) re-indexed from 0 (a merge cluster's rows)."""
        return RowPlan(self.n, self.specs, base=self.base + start, parent=self._root)

    # ---- producer -----------------------------------------------------------------------
    def _buffer(self):
        with self._cv:
            while not self._free and self._made >= self._pool and not self._stop:
                self._cv.wait()
            if self._stop:
                return None
            if self._free:
                return self._free.pop()
            self._made += 1
        buf = torch.empty(self.nwords, dtype=torch.int32)
        return (buf.pin_memory() if torch.cuda.is_available() else buf), None

    def _produce(self) -> None:
        for i in sorted(self.draws):
            if self._keep is not None and not self._keep(i):
                try:
                    self.draws[i]()                  # consumed from the RNG stream, not used
                except BaseException as e:
                    with self._cv:
                        self._err = (i, e)
                        self._cv.notify_all()
                    return
                continue
            got = self._buffer()
            if got is None:
                return
            buf, ev = got
            if ev is not None:
                ev.synchronize()                     # its previous H2D has read it
            try:
                words = self.draws[i]()
                np.copyto(buf.numpy().view(np.uint32), words)
            except BaseException as e:               # raised to the pipeline at row i
                with self._cv:
                    self._err = (i, e)
                    self._cv.notify_all()
                return
            with self._cv:
                self._ready[i] = buf
                self._cv.notify_all()

    # ---- consumers ----------------------------------------------------------------------
    def take_mask(self, i: int) -> torch.Tensor:
        """Row i's pinned mask words (blocks until drawn); hand the buffer back with
        :meth:`release` once a copy from it has been queued."""
        r, row = self._root, self.base + i
        r._start()
        with r._cv:
            while row not in r._ready:
                if r._err is not None and r._err[0] <= row:
                    raise r._err[1]
                if r._stop:
                    raise RuntimeError("row plan closed")
                r._cv.wait()
            return r._ready.pop(row)

    def release(self, buf: torch.Tensor, event) -> None:
        r = self._root
        with r._cv:
            r._free.append((buf, event))
            r._cv.notify_all()

    def close(self, wait: bool = True) -> None:
        """wait=True: every draw has run (raises the first draw error; a device MT round
        sets np.random to the state after its draws, or raises :class:`MtRedraw`); False:
        stop early (np.random keeps the state it had when the plan was made)."""
        r = self._root
        if wait:
            r._start()
        if r._thread is not None:
            if not wait:
                with r._cv:
                    r._stop = True
                    r._cv.notify_all()
            r._thread.join()
            r._thread = None
        if wait and r._err is not None:
            raise r._err[1]
        if wait and r.mt_rows:
            r._mt_finish()

    # ---- device MT19937 rows --------------------------------------------------------------
    def mt_round(self, dev: torch.device) -> "codec.MtRound":
        """The round's :class:`~openmsftl_amd.codec.MtRound` on ``dev`` (begun on the current
        stream the first time a pipeline of that device asks)."""
        r = self._root
        key = dev.index if dev.index is not None else torch.cuda.current_device()
        with r._mt_lock:
            R = r._mt_rounds.get(key)
            if R is None:
                k, pos, _, _ = r._mt_start
                R = codec.MtRound(r.n, r.mt_rows, k, pos, dev)
                r._mt_rounds[key] = R
            return R

    def mt_redraw_seen(self) -> bool:
        """Did a row drawn so far on any device hit NumPy's redraw (synchronises)?"""
        return any(R.end_state()[2] for R in list(self._root._mt_rounds.values()))

    def _mt_finish(self) -> None:
        rounds = list(self._mt_rounds.values()) or [self.mt_round(
            torch.device("cuda", torch.cuda.current_device()))]
        ends = [R.end_state() for R in rounds]          # synchronises
        if self._mt_redraw or any(e[2] for e in ends):
            raise MtRedraw("NumPy would redraw a binomial variate in this round")
        key, pos, _ = ends[0]
        _, _, has_gauss, gauss = self._mt_start
        codec.mt_set_state(key, pos, has_gauss, gauss)


def top_plan(n: int, k: int, clients: int) -> RowPlan:
    """Every row a magnitude top-k packet (the configured codec, client_config.json:48-50)."""
    return RowPlan(n, [RowCodec("top", k=k)] * clients)


def _getter(host: HostSource):
    return host if callable(host) else (lambda i: host[i])


def _weights(clients: int, weights) -> np.ndarray:
    w = fedavg_weights(clients) if weights is None else np.asarray(weights)
    if w.shape != (clients,):
        raise AssertionError("one weight per client (gar.py:41-42)")
    if w.dtype != np.float32:
        raise TypeError("HostFedAvg folds with float32 weights")
    return w


class HostFedAvg:
    """A reusable H2D -> encode -> fold -> D2H pipeline for clients of length n.

    Rows are made as their :class:`RowCodec` says (``plan`` of :meth:`run`; without one every
    row is a top-k packet of ``k``).  ``sets`` packet sets of ``group`` packets each: with 2,
    one group encodes into one set while the previous group, in the other, waits for the
    running aggregate (the rings).  A dense row ('full') occupies its packet's value buffer."""

    def __init__(self, n: int, k: Optional[int] = None, *, group: int = 64, ring: int = 4,
                 stage: int = 2, copy_threads: int = 4, pin: str = "stage",
                 device: Optional[torch.device] = None, sets: int = 1):
        if k is not None and not 0 < k < n:
            raise ValueError("HostFedAvg needs 0 < k < n")
        if pin not in ("stage", "register"):
            raise ValueError("pin must be 'stage' or 'register'")
        if group < 1 or ring < 1 or sets < 1:
            raise ValueError("group, ring and sets must be >= 1")
        self.n, self.k, self.group, self.ring, self.sets = n, k, group, ring, sets
        self.pin = pin
        self.dev = device or torch.device("cuda", torch.cuda.current_device())
        self.slots = [torch.empty(n, dtype=torch.float32, device=self.dev) for _ in range(ring)]
        self.hdrs = [torch.empty((group, L.HDR_BYTES), dtype=torch.uint8, device=self.dev)
                     for _ in range(sets)]
        self.pktsets = [[codec.Packet.alloc(n, L.FC_FMT_IDXVAL, self.dev, hdr=h[j], k=k or 0)
                         for j in range(group)] for h in self.hdrs]
        self.pkts = self.pktsets[0]
        self.status_host = [torch.empty((group, 4), dtype=torch.uint8).pin_memory()
                            for _ in range(sets)]
        self.encoded = [torch.cuda.Event() for _ in range(sets)]
        self.set_free = [torch.cuda.Event() for _ in range(sets)]   # the set's last fold read it
        self.rows_of = [None] * sets                # (row codecs) of the group encoded in a set
        self.acc = torch.empty(n, dtype=torch.float32, device=self.dev)
        self.scratch = torch.empty(n, dtype=torch.float32, device=self.dev)
        self.out_host = torch.empty(n, dtype=torch.float32).pin_memory()
        self.copy = torch.cuda.Stream(self.dev)
        self.h2d_done = [torch.cuda.Event() for _ in range(ring)]
        self.enc_done = [torch.cuda.Event() for _ in range(ring)]
        self._slot = 0
        self.mslots = None                          # host-drawn mask words per ring slot
        self.zero_mask = None
        # pinned staging for pageable sources (allocated on first use)
        self.nstage = max(1, stage)
        self.stage_bufs = None
        self.stage_free = [torch.cuda.Event() for _ in range(self.nstage)]
        self.copy_threads = max(1, copy_threads)
        self._pool = None
        self._registered = []                       # (ptr, event) awaiting unregister
        self._views = {}
        self.exact_fallbacks = 0
        self.staged_copies = 0

    def _default_plan(self, clients: int) -> RowPlan:
        if self.k is None:
            raise ValueError("no row plan and no default k")
        return top_plan(self.n, self.k, clients)

    # ---- host side ------------------------------------------------------------------
    def _as_cpu_tensor(self, src) -> torch.Tensor:
        if isinstance(src, np.ndarray):
            if src.dtype != np.float32 or src.ndim != 1:
                raise ValueError("host gradients must be 1-D float32")
            src = torch.from_numpy(np.ascontiguousarray(src))
        if not isinstance(src, torch.Tensor) or src.is_cuda:
            raise ValueError("host gradients must be CPU tensors or NumPy arrays")
        if src.dtype != torch.float32 or src.numel() != self.n:
            raise ValueError("host gradients must be fp32 of n elements")
        return src.contiguous()

    def _host_copy(self, dst: torch.Tensor, src: torch.Tensor) -> None:
        """dst <- src (CPU -> pinned CPU) in ``copy_threads`` slices (NumPy releases the GIL)."""
        d, s = dst.numpy(), src.numpy()
        t = self.copy_threads
        if t == 1 or self.n < (1 << 20):
            np.copyto(d, s)
            return
        if self._pool is None:
            self._pool = ThreadPoolExecutor(t)
        cuts = [i * self.n // t for i in range(t + 1)]
        list(self._pool.map(lambda i: np.copyto(d[cuts[i]:cuts[i + 1]], s[cuts[i]:cuts[i + 1]]),
                            range(t)))

    def _register(self, t: torch.Tensor) -> bool:
        rt = torch.cuda.cudart()
        return int(rt.cudaHostRegister(t.data_ptr(), t.numel() * 4, 0)) == 0

    def _release_registered(self, wait: bool = False) -> None:
        rt = torch.cuda.cudart()
        keep = []
        for ptr, ev, ref in self._registered:
            if wait:
                ev.synchronize()
            if ev.query():
                rt.cudaHostUnregister(ptr)
            else:
                keep.append((ptr, ev, ref))
        self._registered = keep

    def _h2d(self, src, dst: torch.Tensor, wait=None, done=None) -> None:
        """Queue one client's gradient into the device buffer ``dst`` on the copy stream, after
        event ``wait`` (the buffer's previous reader); record ``done`` after the copy."""
        t = self._as_cpu_tensor(src)
        if wait is not None:
            self.copy.wait_event(wait)
        if not t.is_pinned():
            if self.pin == "register" and self._register(t):
                with torch.cuda.stream(self.copy):
                    dst.copy_(t, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.copy)
                self._registered.append((t.data_ptr(), ev, t))
                if done is not None:
                    done.record(self.copy)
                self._release_registered()
                return
            if self.stage_bufs is None:
                self.stage_bufs = [torch.empty(self.n, dtype=torch.float32).pin_memory()
                                   for _ in range(self.nstage)]
                for e in self.stage_free:
                    e.record(self.copy)
            b = self.staged_copies % self.nstage
            self.staged_copies += 1
            self.stage_free[b].synchronize()           # its previous H2D has read it
            self._host_copy(self.stage_bufs[b], t)
            t = self.stage_bufs[b]
            with torch.cuda.stream(self.copy):
                dst.copy_(t, non_blocking=True)
                self.stage_free[b].record(self.copy)
        else:
            with torch.cuda.stream(self.copy):
                dst.copy_(t, non_blocking=True)
        if done is not None:
            done.record(self.copy)

    def _mslot(self, slot: int) -> torch.Tensor:
        if self.mslots is None:
            words = (self.n + 31) // 32
            self.mslots = [torch.empty(words, dtype=torch.int32, device=self.dev)
                           for _ in range(self.ring)]
        return self.mslots[slot]

    def _mask_slot(self, slot: int, plan: RowPlan, i: int) -> torch.Tensor:
        """Row i's host-drawn mask into the ring slot's device mask words (copy stream, after
        the slot's previous encode: queue it after :meth:`_h2d` of the same slot)."""
        self._mslot(slot)
        buf = plan.take_mask(i)
        with torch.cuda.stream(self.copy):
            self.mslots[slot].copy_(buf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy)
        plan.release(buf, ev)
        return self.mslots[slot]

    def _views_for(self, weights: np.ndarray, rows: range, ps: int, j0: int = 0) -> torch.Tensor:
        key = ("v", weights.tobytes(), rows.start, len(rows), ps, j0)
        v = self._views.get(key)
        if v is None:
            v = codec.views_tensor(self.pktsets[ps][j0:j0 + len(rows)],
                                   [float(x) for x in weights[rows.start:rows.stop]], self.dev)
            self._cache(key, v)
        return v

    def _dense_args(self, weights: np.ndarray, rows: range, ps: int, j0: int):
        """(row pointers, weights) device arrays of a run of dense rows held in the set's
        packet value buffers."""
        key = ("d", weights.tobytes(), rows.start, len(rows), ps, j0)
        v = self._views.get(key)
        if v is None:
            ptrs = [p.val.data_ptr() for p in self.pktsets[ps][j0:j0 + len(rows)]]
            v = (torch.tensor(ptrs, dtype=torch.int64).to(self.dev),
                 torch.from_numpy(np.ascontiguousarray(weights[rows.start:rows.stop])).to(self.dev))
            self._cache(key, v)
        return v

    def _cache(self, key, v) -> None:
        self._views = {key: v} if len(self._views) > 64 else {**self._views, key: v}

    # ---- one fold group (rows of G) ---------------------------------------------------
    def begin(self) -> None:
        """Start of a round on the caller's (compute) stream: every ring slot is free."""
        comp = torch.cuda.current_stream(self.dev)
        for e in self.enc_done:
            e.record(comp)

    def encode_group(self, get, rows: range, ps: int = 0, plan: Optional[RowPlan] = None) -> None:
        """Queue H2D + encode of ``rows`` into packet set ``ps`` on the current stream, then
        the copy of their status words to pinned host memory (:meth:`check_group` reads
        them; the host does not wait here).  Dense rows are copied straight into their
        packet's value buffer (after the set's previous fold, ``set_free``)."""
        if len(rows) > self.group:
            raise ValueError(f"a fold group holds at most {self.group} rows")
        plan = plan if plan is not None else self._default_plan(rows.stop)
        comp = torch.cuda.current_stream(self.dev)
        pk = self.pktsets[ps]
        specs = [plan(i) for i in rows]
        dense_h2d = None
        for j, (i, rc) in enumerate(zip(rows, specs)):
            if rc.kind == "dense":
                if dense_h2d is None:
                    dense_h2d = torch.cuda.Event()
                    self.copy.wait_event(self.set_free[ps])
                self._h2d(get(i), pk[j].val[:self.n])
                continue
            s = self._slot
            self._slot = (s + 1) % self.ring
            self._h2d(get(i), self.slots[s], wait=self.enc_done[s])
            mask = self._mask_slot(s, plan, i) if rc.mask_src == "host" else None
            self.h2d_done[s].record(self.copy)
            if rc.mask_src == "mt":                 # np.random.binomial's draws, on the device,
                # made while the row's gradient is still on its way (the slot's previous
                # encode, its last reader, is earlier on this stream)
                mask = plan.mt_round(self.dev).binomial(rc.offset, rc.p, out=self._mslot(s))
            comp.wait_event(self.h2d_done[s])
            if rc.kind == "top":
                codec.encode_top(self.slots[s], rc.k, key_mode=rc.key_mode, seed=rc.seed,
                                 offset=rc.offset, packet=pk[j], check=False)
            elif rc.kind == "mask":
                if rc.mask_src == "none":
                    if self.zero_mask is None:
                        self.zero_mask = torch.zeros((self.n + 31) // 32, dtype=torch.int32,
                                                     device=self.dev)
                    mask = self.zero_mask
                codec.encode_mask(self.slots[s], rc.codec, p=rc.p, mask_bits=mask, seed=rc.seed,
                                  offset=rc.offset, fmt=L.FC_FMT_IDXVAL, packet=pk[j])
            else:
                raise ValueError(f"unknown row kind {rc.kind!r}")
            self.enc_done[s].record(comp)
        if dense_h2d is not None:
            dense_h2d.record(self.copy)
            comp.wait_event(dense_h2d)
        self.rows_of[ps] = specs
        m = len(rows)
        self.status_host[ps][:m].copy_(self.hdrs[ps][:m, 36:40], non_blocking=True)
        self.encoded[ps].record(comp)

    def check_group(self, get, rows: range, ps: int = 0) -> torch.cuda.Event:
        """Wait for the group's status words; a top-k packet whose sampled bracket missed is
        re-encoded exactly from its host copy (current stream).  Returns an event after
        which the group's rows are final."""
        self.encoded[ps].synchronize()
        specs = self.rows_of[ps]
        st = self.status_host[ps][:len(rows)].numpy().view(np.uint32).ravel()
        bad = [int(j) for j in np.nonzero(st)[0] if specs[int(j)].kind != "dense"]
        if not bad:
            return self.encoded[ps]
        for j in bad:
            rc = specs[j]
            if rc.kind != "top" or st[j] != L.FC_STATUS_RETRY_EXACT:
                raise L.FedCodecError(f"row {rows.start + j}: packet status {int(st[j])}")
            self.scratch.copy_(self._as_cpu_tensor(get(rows.start + j)))
            codec.encode_top(self.scratch, rc.k, key_mode=rc.key_mode, seed=rc.seed,
                             offset=rc.offset, packet=self.pktsets[ps][j], exact=True)
            self.exact_fallbacks += 1
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        return ev

    def fold_group(self, weights: np.ndarray, rows: range, ps: int, acc: torch.Tensor,
                   continue_sum: bool) -> None:
        """acc (+)= the group's rows in row order, current stream: each run of packets by
        fc_decode_accumulate[_continue], each run of dense rows by
        fc_weighted_sum_dense[_continue] (the same left-to-right fp32 sum, gar.py:44)."""
        lib = L.load()
        specs = self.rows_of[ps]
        stream = codec._stream(self.dev)
        j = 0
        while j < len(rows):
            dense = specs[j].kind == "dense"
            j1 = j + 1
            while j1 < len(rows) and (specs[j1].kind == "dense") == dense:
                j1 += 1
            sub = range(rows.start + j, rows.start + j1)
            cont = continue_sum or j > 0
            if dense:
                ptrs, w = self._dense_args(weights, sub, ps, j)
                fn = lib.fc_weighted_sum_dense_continue if cont else lib.fc_weighted_sum_dense
                L.check(fn(ctypes.c_void_p(ptrs.data_ptr()), ctypes.c_void_p(w.data_ptr()),
                           len(sub), self.n, ctypes.c_void_p(acc.data_ptr()), stream),
                        "fc_weighted_sum_dense")
            else:
                codec.decode_accumulate(self.pktsets[ps][j:j1], None, out=acc,
                                        views=self._views_for(weights, sub, ps, j),
                                        continue_sum=cont)
            j = j1
        self.set_free[ps].record(torch.cuda.current_stream(self.dev))

    def finish(self) -> None:
        if self._registered:
            self._release_registered(wait=True)

    # ---- one device, sequential groups -----------------------------------------------
    def run(self, host: HostSource, clients: int, weights: Optional[np.ndarray] = None,
            sync: bool = True, out: Optional[torch.Tensor] = None,
            to_host: bool = True, continue_sum: bool = False,
            plan: Optional[RowPlan] = None) -> torch.Tensor:
        """FedAVG of ``clients`` host gradients (``host[i]`` or ``host(i)``: fp32 CPU tensors
        or NumPy arrays of n elements; pinned ones are copied directly) with float32 weights
        (default fl32(1/M), gar.py:37-40), row i made as ``plan(i)`` says (default: top-k of
        ``k``).  Returns the pinned host aggregate (valid after the stream syncs; ``sync``
        does it), or with ``to_host=False`` the device aggregate (``out`` if given: a float32
        CUDA tensor of n elements).  ``continue_sum``: ``out`` already holds the left-to-right
        sum of earlier rows (another device's or rank's shard) and these rows continue it, so
        a chain of runs is one fold over all rows (gar.py:44)."""
        get = _getter(host)
        w = _weights(clients, weights)
        plan = plan if plan is not None else self._default_plan(clients)
        acc = self.acc if out is None else out
        if acc.dtype != torch.float32 or acc.numel() != self.n or not acc.is_cuda:
            raise ValueError("out must be a float32 CUDA tensor of n elements")
        if continue_sum and out is None:
            raise ValueError("continue_sum needs the running sum in out")
        self.begin()
        for rows in group_bounds(clients, self.group):
            self.encode_group(get, rows, 0, plan)
            self.check_group(get, rows, 0)
            self.fold_group(w, rows, 0, acc, continue_sum or rows.start > 0)
        if clients == 0 and not continue_sum:
            acc.zero_()                                     # no rows: np.sum's +0
        self.finish()
        if not to_host:
            return acc
        self.out_host.copy_(acc, non_blocking=True)
        if sync:
            torch.cuda.synchronize(self.dev)
        return self.out_host


def host_fold(pipe: HostFedAvg, host: HostSource, plan: Optional[RowPlan] = None):
    """A :data:`openmsftl_amd.distributed.Fold` over host gradients: the rows ``rows`` of G
    (global client indices, ``host[i]`` / ``host(i)``) streamed through ``pipe`` into the
    device partial sum ``out``.  Composes the host-resident round (configs[4]) with
    :class:`~openmsftl_amd.distributed.ShardedFedAvg`: each rank streams its contiguous shard,
    then the partial sums are reduced (RCCL) or chained (bit-exact, serial)."""
    get = _getter(host)

    def fold(rows: range, w: np.ndarray, out, continue_sum: bool):
        r0 = rows.start
        return pipe.run(lambda j: get(r0 + j), len(rows), np.asarray(w, np.float32), sync=False,
                        out=out, to_host=False, continue_sum=continue_sum,
                        plan=plan.shifted(r0) if plan is not None else None)
    return fold


# ---- the running aggregate travels between devices in group order -------------------------
def _ring_worker(pipe: HostFedAvg, get, w: np.ndarray, groups: List[range], mine: List[int],
                 acc: torch.Tensor, comp, fold_s, take, give, plan: RowPlan) -> None:
    """One device's share of a ring round: its groups ``mine`` (indices into ``groups``,
    increasing).  Group t's successor on this device encodes into the other packet set while
    group t waits for the aggregate of the rows before it: ``take(t)`` (called with the fold
    stream current) returns ``(tensor, event)`` holding it — ``(None, None)`` when ``acc``
    already holds it or t == 0 — and ``give(t, acc, event)`` hands the result on."""
    if pipe.sets < 2:
        raise ValueError("ring pipelines need sets=2 (one set encodes, one waits)")
    done = [None] * pipe.sets
    with torch.cuda.device(pipe.dev), torch.cuda.stream(comp):
        pipe.begin()

        def finish(t, ps):
            rows = groups[t]
            with torch.cuda.stream(fold_s):
                src, ev = take(t)               # (a receive is queued before the host waits)
            ready = pipe.check_group(get, rows, ps)
            with torch.cuda.stream(fold_s):
                fold_s.wait_event(ready)
                if ev is not None:
                    fold_s.wait_event(ev)
                if src is not None and src is not acc:
                    acc.copy_(src, non_blocking=True)          # the aggregate's hop (D2D / P2P)
                pipe.fold_group(w, rows, ps, acc, continue_sum=t > 0)
                e = torch.cuda.Event()
                e.record(fold_s)
            done[ps] = e
            give(t, acc, e)

        pending = None
        for idx, t in enumerate(mine):
            ps = idx % pipe.sets
            if done[ps] is not None:
                comp.wait_event(done[ps])             # the set's previous group is folded
            pipe.encode_group(get, groups[t], ps, plan)
            if pending is not None:
                finish(*pending)
            pending = (t, ps)
        if pending is not None:
            finish(*pending)
        pipe.finish()


class DeviceRing:
    """FedAVG of host gradients over several devices of ONE process, bit-exact to gar.py:44.

    Fold groups are dealt round-robin to the pipelines (one :class:`HostFedAvg` per device,
    two packet sets each), each driven by its own host thread; the running aggregate hops from
    device to device in group order (stream events order every hop, no host round trip).
    ``pipes`` may share a device (tests stand two pipelines on one GPU in for two GPUs)."""

    def __init__(self, pipes: Sequence[HostFedAvg]):
        if not pipes:
            raise ValueError("no pipelines")
        n, k, grp = pipes[0].n, pipes[0].k, pipes[0].group
        if any(p.n != n or p.k != k or p.group != grp for p in pipes):
            raise ValueError("pipelines must share n, k and group")
        if any(p.sets < 2 for p in pipes):
            raise ValueError("ring pipelines need sets=2 (one set encodes, one waits)")
        self.pipes = list(pipes)
        self.n, self.k, self.group = n, k, grp
        self.comp = [torch.cuda.Stream(p.dev) for p in pipes]
        self.fold = [torch.cuda.Stream(p.dev) for p in pipes]
        self.accs = [torch.empty(n, dtype=torch.float32, device=p.dev) for p in pipes]
        self.out_host = torch.empty(n, dtype=torch.float32).pin_memory()
        self._pool = ThreadPoolExecutor(len(pipes))

    @property
    def devices(self) -> list:
        return [p.dev for p in self.pipes]

    @property
    def exact_fallbacks(self) -> int:
        return sum(p.exact_fallbacks for p in self.pipes)

    def run(self, host: HostSource, clients: int, weights: Optional[np.ndarray] = None,
            to_host: bool = True, plan: Optional[RowPlan] = None) -> torch.Tensor:
        """The FedAVG aggregate of ``clients`` host gradients (row i made as ``plan(i)`` says,
        default top-k of ``k``): the pinned host array (synced), or with ``to_host=False`` the
        device tensor holding it (on the last group's device, ordered before later work on
        that device's current stream; the next run writes it only after the work the caller
        has queued on its devices' current streams by then)."""
        get = _getter(host)
        w = _weights(clients, weights)
        plan = plan if plan is not None else self.pipes[0]._default_plan(clients)
        for d, p in enumerate(self.pipes):       # the last run's result may still be read there
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(p.dev))
            self.fold[d].wait_event(ev)
        groups = group_bounds(clients, self.group)
        D = len(self.pipes)
        if not groups:
            raise Exception("Empty gradient list")               # aggregation.py:59-60
        tokens = {}
        cv = threading.Condition()
        failed = []

        def take(t):
            if t == 0:
                return None, None
            with cv:
                while t - 1 not in tokens and not failed:
                    cv.wait(timeout=1.0)
                if t - 1 not in tokens:
                    raise RuntimeError("another device of the ring failed")
                return tokens[t - 1]

        def give(t, acc, ev):
            with cv:
                tokens[t] = (acc, ev)
                cv.notify_all()

        def work(d):
            try:
                mine = list(range(d, len(groups), D))
                if mine:
                    _ring_worker(self.pipes[d], get, w, groups, mine, self.accs[d],
                                 self.comp[d], self.fold[d], take, give, plan)
            except BaseException:
                with cv:
                    failed.append(d)
                    cv.notify_all()
                raise

        for f in [self._pool.submit(work, d) for d in range(D)]:
            f.result()
        acc, ev = tokens[len(groups) - 1]
        with torch.cuda.device(acc.device):
            cur = torch.cuda.current_stream(acc.device)
            cur.wait_event(ev)
            if not to_host:
                return acc
            self.out_host.copy_(acc, non_blocking=True)
            cur.synchronize()
        return self.out_host


class RankRing:
    """:class:`DeviceRing` across processes (one rank per GPU, ``torch.distributed``): rank r
    encodes the fold groups t = r, r+W, ...; the running aggregate goes rank to rank in group
    order by point-to-point send/recv (RCCL over xGMI with ``nccl``; staged through host
    memory with gloo), and the last group's rank sends it to ``dst``.  Bit-exact to gar.py:44
    over all M rows, with every rank's encodes running in parallel.

    Every rank issues its receives and sends in increasing group order, so each pair's
    operations match one for one (rank t % W sends group t's aggregate, rank (t+1) % W
    receives it next) and the ring cannot deadlock."""

    def __init__(self, pipe: HostFedAvg, dst: int = 0, group=None):
        if pipe.sets < 2:
            raise ValueError("RankRing needs a pipeline with sets=2")
        import torch.distributed as dist
        self.pipe, self.dst, self.pg = pipe, dst, group
        init = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if init else 1
        self.rank = dist.get_rank(group) if init else 0
        self.comp = torch.cuda.Stream(pipe.dev)
        self.fold = torch.cuda.Stream(pipe.dev)
        self.acc = torch.empty(pipe.n, dtype=torch.float32, device=pipe.dev)

    def _gloo(self) -> bool:
        import torch.distributed as dist
        return dist.get_backend(self.pg) == "gloo"

    def _send(self, t: torch.Tensor, peer: int) -> None:
        import torch.distributed as dist
        dist.send(t.cpu() if self._gloo() else t, dst=peer, group=self.pg)

    def _recv(self, t: torch.Tensor, peer: int) -> None:
        import torch.distributed as dist
        if self._gloo():
            h = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(h, src=peer, group=self.pg)
            t.copy_(h)
        else:
            dist.recv(t, src=peer, group=self.pg)

    def run(self, host: HostSource, clients: int, weights: Optional[np.ndarray] = None,
            plan: Optional[RowPlan] = None) -> Optional[torch.Tensor]:
        """Returns the device aggregate on ``dst`` (ordered before later work on the current
        stream), None on the other ranks.  ``host(i)`` is called for this rank's rows only.
        A ``plan`` with host draws must be the same on every rank (each rank draws every
        row's mask in order, so all ranks leave the RNG where the reference does)."""
        get = _getter(host)
        w = _weights(clients, weights)
        plan = plan if plan is not None else self.pipe._default_plan(clients)
        G_, W_, r_ = self.pipe.group, self.world, self.rank
        plan.restrict(lambda i: (i // G_) % W_ == r_)
        groups = group_bounds(clients, self.pipe.group)
        if not groups:
            raise Exception("Empty gradient list")               # aggregation.py:59-60
        W, r = self.world, self.rank
        last_owner = (len(groups) - 1) % W
        acc = self.acc

        def take(t):                            # fold stream is current here
            if t > 0 and W > 1:
                self._recv(acc, (t - 1) % W)
            return None, None

        def give(t, a, ev):
            if W == 1:
                return
            if t + 1 < len(groups):
                peer = (t + 1) % W
            elif last_owner != self.dst:
                peer = self.dst
            else:
                return
            with torch.cuda.device(self.pipe.dev), torch.cuda.stream(self.fold):
                self._send(a, peer)

        mine = list(range(r, len(groups), W))
        if mine:
            _ring_worker(self.pipe, get, w, groups, mine, acc, self.comp, self.fold, take, give,
                         plan)
        cur = torch.cuda.current_stream(self.pipe.dev)
        if r == self.dst and last_owner != self.dst:
            with torch.cuda.device(self.pipe.dev), torch.cuda.stream(self.fold):
                self._recv(acc, last_owner)
        cur.wait_stream(self.fold)
        root = plan._root
        if root.mt_rows and W > 1:
            # a redraw seen by one rank must send every rank to the host draws (MtRedraw at
            # close), or the ranks would leave np.random in different states
            import torch.distributed as dist
            flag = torch.tensor([int(root.mt_redraw_seen())], dtype=torch.int32)
            if not self._gloo():
                flag = flag.to(self.pipe.dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.pg)
            root._mt_redraw = bool(int(flag.item()))
        return acc if r == self.dst else None
