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

import threading
from concurrent.futures import ThreadPoolExecutor
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
    """A reusable H2D -> encode -> fold -> D2H pipeline for clients of length n, top-k k.

    ``sets`` packet sets of ``group`` packets each: with 2, one group encodes into one set
    while the previous group, in the other, waits for the running aggregate (the rings)."""

    def __init__(self, n: int, k: int, *, group: int = 64, ring: int = 4, stage: int = 2,
                 copy_threads: int = 4, pin: str = "stage",
                 device: Optional[torch.device] = None, sets: int = 1):
        if not 0 < k < n:
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
        self.pktsets = [[codec.Packet.alloc(n, L.FC_FMT_IDXVAL, self.dev, hdr=h[j], k=k)
                         for j in range(group)] for h in self.hdrs]
        self.pkts = self.pktsets[0]
        self.status_host = [torch.empty((group, 4), dtype=torch.uint8).pin_memory()
                            for _ in range(sets)]
        self.encoded = [torch.cuda.Event() for _ in range(sets)]
        self.acc = torch.empty(n, dtype=torch.float32, device=self.dev)
        self.scratch = torch.empty(n, dtype=torch.float32, device=self.dev)
        self.out_host = torch.empty(n, dtype=torch.float32).pin_memory()
        self.copy = torch.cuda.Stream(self.dev)
        self.h2d_done = [torch.cuda.Event() for _ in range(ring)]
        self.enc_done = [torch.cuda.Event() for _ in range(ring)]
        self._slot = 0
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

    def _h2d(self, src, slot: int) -> None:
        """Queue one client's gradient into device slot ``slot`` on the copy stream."""
        t = self._as_cpu_tensor(src)
        self.copy.wait_event(self.enc_done[slot])
        if not t.is_pinned():
            if self.pin == "register" and self._register(t):
                with torch.cuda.stream(self.copy):
                    self.slots[slot].copy_(t, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.copy)
                self._registered.append((t.data_ptr(), ev, t))
                self.h2d_done[slot].record(self.copy)
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
                self.slots[slot].copy_(t, non_blocking=True)
                self.stage_free[b].record(self.copy)
        else:
            with torch.cuda.stream(self.copy):
                self.slots[slot].copy_(t, non_blocking=True)
        self.h2d_done[slot].record(self.copy)

    def _views_for(self, weights: np.ndarray, rows: range, ps: int) -> torch.Tensor:
        key = (weights.tobytes(), rows.start, len(rows), ps)
        v = self._views.get(key)
        if v is None:
            v = codec.views_tensor(self.pktsets[ps][:len(rows)],
                                   [float(x) for x in weights[rows.start:rows.stop]], self.dev)
            self._views = {key: v} if len(self._views) > 64 else {**self._views, key: v}
        return v

    # ---- one fold group (rows of G) ---------------------------------------------------
    def begin(self) -> None:
        """Start of a round on the caller's (compute) stream: every ring slot is free."""
        comp = torch.cuda.current_stream(self.dev)
        for e in self.enc_done:
            e.record(comp)

    def encode_group(self, get, rows: range, ps: int = 0) -> None:
        """Queue H2D + encode of ``rows`` into packet set ``ps`` on the current stream, then
        the copy of their status words to pinned host memory (:meth:`check_group` reads
        them; the host does not wait here)."""
        if len(rows) > self.group:
            raise ValueError(f"a fold group holds at most {self.group} rows")
        comp = torch.cuda.current_stream(self.dev)
        pk = self.pktsets[ps]
        for j, i in enumerate(rows):
            s = self._slot
            self._slot = (s + 1) % self.ring
            self._h2d(get(i), s)
            comp.wait_event(self.h2d_done[s])
            codec.encode_top(self.slots[s], self.k, packet=pk[j], check=False)
            self.enc_done[s].record(comp)
        m = len(rows)
        self.status_host[ps][:m].copy_(self.hdrs[ps][:m, 36:40], non_blocking=True)
        self.encoded[ps].record(comp)

    def check_group(self, get, rows: range, ps: int = 0) -> torch.cuda.Event:
        """Wait for the group's status words; a packet whose sampled bracket missed is
        re-encoded exactly from its host copy (current stream).  Returns an event after
        which the group's packets are final."""
        self.encoded[ps].synchronize()
        st = self.status_host[ps][:len(rows)].numpy().view(np.uint32).ravel()
        bad = np.nonzero(st)[0]
        if len(bad) == 0:
            return self.encoded[ps]
        for j in bad:
            self.scratch.copy_(self._as_cpu_tensor(get(rows.start + int(j))))
            codec.encode_top(self.scratch, self.k, packet=self.pktsets[ps][int(j)], exact=True)
            self.exact_fallbacks += 1
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        return ev

    def fold_group(self, weights: np.ndarray, rows: range, ps: int, acc: torch.Tensor,
                   continue_sum: bool) -> None:
        """acc (+)= the group's rows in order (fc_decode_accumulate[_continue]), current stream."""
        codec.decode_accumulate(self.pktsets[ps][:len(rows)], None, out=acc,
                                views=self._views_for(weights, rows, ps),
                                continue_sum=continue_sum)

    def finish(self) -> None:
        if self._registered:
            self._release_registered(wait=True)

    # ---- one device, sequential groups -----------------------------------------------
    def run(self, host: HostSource, clients: int, weights: Optional[np.ndarray] = None,
            sync: bool = True, out: Optional[torch.Tensor] = None,
            to_host: bool = True, continue_sum: bool = False) -> torch.Tensor:
        """FedAVG of ``clients`` host gradients (``host[i]`` or ``host(i)``: fp32 CPU tensors
        or NumPy arrays of n elements; pinned ones are copied directly) with float32 weights
        (default fl32(1/M), gar.py:37-40).  Returns the pinned host aggregate (valid after the
        stream syncs; ``sync`` does it), or with ``to_host=False`` the device aggregate
        (``out`` if given: a float32 CUDA tensor of n elements).  ``continue_sum``: ``out``
        already holds the left-to-right sum of earlier rows (another device's or rank's shard)
        and these rows continue it, so a chain of runs is one fold over all rows (gar.py:44)."""
        get = _getter(host)
        w = _weights(clients, weights)
        acc = self.acc if out is None else out
        if acc.dtype != torch.float32 or acc.numel() != self.n or not acc.is_cuda:
            raise ValueError("out must be a float32 CUDA tensor of n elements")
        if continue_sum and out is None:
            raise ValueError("continue_sum needs the running sum in out")
        self.begin()
        for rows in group_bounds(clients, self.group):
            self.encode_group(get, rows, 0)
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


def host_fold(pipe: HostFedAvg, host: HostSource):
    """A :data:`openmsftl_amd.distributed.Fold` over host gradients: the rows ``rows`` of G
    (global client indices, ``host[i]`` / ``host(i)``) streamed through ``pipe`` into the
    device partial sum ``out``.  Composes the host-resident round (configs[4]) with
    :class:`~openmsftl_amd.distributed.ShardedFedAvg`: each rank streams its contiguous shard,
    then the partial sums are reduced (RCCL) or chained (bit-exact, serial)."""
    get = _getter(host)

    def fold(rows: range, w: np.ndarray, out, continue_sum: bool):
        r0 = rows.start
        return pipe.run(lambda j: get(r0 + j), len(rows), np.asarray(w, np.float32), sync=False,
                        out=out, to_host=False, continue_sum=continue_sum)
    return fold


# ---- the running aggregate travels between devices in group order -------------------------
def _ring_worker(pipe: HostFedAvg, get, w: np.ndarray, groups: List[range], mine: List[int],
                 acc: torch.Tensor, comp, fold_s, take, give) -> None:
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
            pipe.encode_group(get, groups[t], ps)
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
            to_host: bool = True) -> torch.Tensor:
        """The FedAVG aggregate of ``clients`` host gradients: the pinned host array (synced),
        or with ``to_host=False`` the device tensor holding it (on the last group's device,
        ordered before later work on that device's current stream)."""
        get = _getter(host)
        w = _weights(clients, weights)
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
                                 self.comp[d], self.fold[d], take, give)
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

    def run(self, host: HostSource, clients: int, weights: Optional[np.ndarray] = None
            ) -> Optional[torch.Tensor]:
        """Returns the device aggregate on ``dst`` (ordered before later work on the current
        stream), None on the other ranks.  ``host(i)`` is called for this rank's rows only."""
        get = _getter(host)
        w = _weights(clients, weights)
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
            _ring_worker(self.pipe, get, w, groups, mine, acc, self.comp, self.fold, take, give)
        cur = torch.cuda.current_stream(self.pipe.dev)
        if r == self.dst and last_owner != self.dst:
            with torch.cuda.device(self.pipe.dev), torch.cuda.stream(self.fold):
                self._recv(acc, last_owner)
        cur.wait_stream(self.fold)
        return acc if r == self.dst else None
