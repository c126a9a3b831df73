"""Host-resident FedAVG round: H2D -> top-k encode -> decode-accumulate -> D2H (BASELINE.json
configs[4], the path that "starts and ends in host memory").

The reference's round starts from client gradients in host memory (client.py:53 flattens to
NumPy) and hands the aggregate back to the server loop (aggregation.py:61-78 -> update_model,
aggregation.py:99).  :class:`HostFedAvg` streams the clients' host gradients through the GPU
without ever holding more than ``ring`` of them on the device:

* a copy stream moves client i's gradient into device slot ``i % ring`` (H2D overlapped with
  the encodes of earlier clients); the compute stream waits for that copy, encodes
  (``fc_topk_encode``) into packet ``i % group`` and signals the slot free again;
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

Device memory is bounded by ``ring`` gradients + ``group`` packets + two aggregates whatever
the client count (:func:`plan_group` sizes ``group`` for a byte budget), so the device
``Aggregator.aggregate_grads`` (openmsftl_amd/aggregation.py) runs any number of sampled
clients through it.  Used also by tools/e2e_bench.py (the PCIe-inclusive rate in DESIGN.md)
and tests/test_fullsize_parity.py (the configs[4] digest, ``group`` 64 so the continued fold
is crossed).
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Optional, Sequence, Union

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
               max_group: int = 64) -> int:
    """Packets per fold group so that ring gradients + group packets + the aggregate and a
    scratch row (4N each) + one encoder workspace fit in ``budget_bytes`` (at least 1)."""
    lib = L.load()
    fixed = (ring + 2) * 4 * n + int(lib.fc_workspace_bytes(n))
    g = (budget_bytes - fixed) // packet_bytes(n)
    return int(max(1, min(max_group, clients, g)))


class HostFedAvg:
    """A reusable H2D -> encode -> fold -> D2H pipeline for clients of length n, top-k k."""

    def __init__(self, n: int, k: int, *, group: int = 64, ring: int = 4, stage: int = 2,
                 copy_threads: int = 4, pin: str = "stage",
                 device: Optional[torch.device] = None):
        if not 0 < k < n:
            raise ValueError("HostFedAvg needs 0 < k < n")
        if pin not in ("stage", "register"):
            raise ValueError("pin must be 'stage' or 'register'")
        self.n, self.k, self.group, self.ring = n, k, group, ring
        self.pin = pin
        self.dev = device or torch.device("cuda", torch.cuda.current_device())
        self.slots = [torch.empty(n, dtype=torch.float32, device=self.dev) for _ in range(ring)]
        self.hdrs = torch.empty((group, L.HDR_BYTES), dtype=torch.uint8, device=self.dev)
        self.pkts = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, self.dev, hdr=self.hdrs[j], k=k)
                     for j in range(group)]
        self.acc = torch.empty(n, dtype=torch.float32, device=self.dev)
        self.scratch = torch.empty(n, dtype=torch.float32, device=self.dev)
        self.out_host = torch.empty(n, dtype=torch.float32).pin_memory()
        self.copy = torch.cuda.Stream(self.dev)
        self.h2d_done = [torch.cuda.Event() for _ in range(ring)]
        self.enc_done = [torch.cuda.Event() for _ in range(ring)]
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

    def _h2d(self, i: int, src, slot: int) -> None:
        """Queue client i's gradient into device slot ``slot`` on the copy stream."""
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

    def _views_for(self, weights: np.ndarray, g0: int, m: int) -> torch.Tensor:
        key = (weights.tobytes(), g0, m)
        v = self._views.get(key)
        if v is None:
            v = codec.views_tensor(self.pkts[:m], [float(x) for x in weights[g0:g0 + m]], self.dev)
            self._views = {key: v} if len(self._views) > 64 else {**self._views, key: v}
        return v

    def run(self, host: HostSource, clients: int, weights: Optional[np.ndarray] = None,
            sync: bool = True, out: Optional[torch.Tensor] = None,
            to_host: bool = True) -> torch.Tensor:
        """FedAVG of ``clients`` host gradients (``host[i]`` or ``host(i)``: fp32 CPU tensors
        or NumPy arrays of n elements; pinned ones are copied directly) with float32 weights
        (default fl32(1/M), gar.py:37-40).  Returns the pinned host aggregate (valid after the
        stream syncs; ``sync`` does it), or with ``to_host=False`` the device aggregate
        (``out`` if given: a float32 CUDA tensor of n elements)."""
        get = host if callable(host) else (lambda i: host[i])
        w = fedavg_weights(clients) if weights is None else np.asarray(weights)
        if w.shape != (clients,):
            raise AssertionError("one weight per client (gar.py:41-42)")
        if w.dtype != np.float32:
            raise TypeError("HostFedAvg folds with float32 weights")
        acc = self.acc if out is None else out
        if acc.dtype != torch.float32 or acc.numel() != self.n or not acc.is_cuda:
            raise ValueError("out must be a float32 CUDA tensor of n elements")
        comp = torch.cuda.current_stream(self.dev)
        for e in self.enc_done:
            e.record(comp)
        for g0 in range(0, clients, self.group):
            m = min(self.group, clients - g0)
            for j in range(m):
                i = g0 + j
                s = i % self.ring
                self._h2d(i, get(i), s)
                comp.wait_event(self.h2d_done[s])
                codec.encode_top(self.slots[s], self.k, packet=self.pkts[j], check=False)
                self.enc_done[s].record(comp)
            status = self.hdrs[:m, 36:40].cpu()                 # one sync per group
            if bool((status != 0).any()):                       # exact re-encode, host copy
                for j in np.nonzero(status.numpy().view(np.uint32).ravel())[0]:
                    self.scratch.copy_(self._as_cpu_tensor(get(g0 + int(j))))
                    codec.encode_top(self.scratch, self.k, packet=self.pkts[int(j)], exact=True)
                    self.exact_fallbacks += 1
            codec.decode_accumulate(self.pkts[:m], None, out=acc,
                                    views=self._views_for(w, g0, m), continue_sum=g0 > 0)
        if self._registered:
            self._release_registered(wait=True)
        if not to_host:
            return acc
        self.out_host.copy_(acc, non_blocking=True)
        if sync:
            torch.cuda.synchronize(self.dev)
        return self.out_host
