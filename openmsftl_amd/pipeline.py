"""Host-resident FedAVG round: H2D -> top-k encode -> decode-accumulate -> D2H (BASELINE.json
configs[4], the path that "starts and ends in host memory").

The reference's round starts from client gradients in host memory (client.py:53 flattens to
NumPy) and hands the aggregate back to the server loop (aggregation.py:61-78 -> update_model,
aggregation.py:99).  :class:`HostFedAvg` streams the clients' pinned host gradients through the
GPU without ever holding more than ``ring`` of them on the device:

* a copy stream moves client i's gradient into device slot ``i % ring`` (H2D overlapped with
  the encodes of earlier clients); the compute stream waits for that copy, encodes
  (``fc_topk_encode``) into packet ``i % group`` and signals the slot free again;
* every ``group`` packets are folded into the running aggregate with
  ``fc_decode_accumulate_continue`` (one status read per group; a packet whose sampled bracket
  missed is re-encoded exactly from its host copy), so the sum is the same left-to-right fp32
  fold as gar.py:44 over all rows, bit for bit;
* the aggregate is copied D2H once at the end.

Used by tools/e2e_bench.py (the PCIe-inclusive rate in DESIGN.md) and by
tests/test_fullsize_parity.py (the configs[4] digest, ``group`` 64 so the continued fold is
crossed).
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence, Union

import numpy as np
import torch

from . import _lib as L
from . import codec
from .distributed import fedavg_weights

HostSource = Union[Sequence[torch.Tensor], Callable[[int], torch.Tensor]]


class HostFedAvg:
    """A reusable H2D -> encode -> fold -> D2H pipeline for M clients of length n, top-k k."""

    def __init__(self, n: int, k: int, *, group: int = 64, ring: int = 4,
                 device: Optional[torch.device] = None):
        if not 0 < k < n:
            raise ValueError("HostFedAvg needs 0 < k < n")
        self.n, self.k, self.group, self.ring = n, k, group, ring
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
        self._views = {}
        self.exact_fallbacks = 0

    def _views_for(self, weights: np.ndarray, g0: int, m: int) -> torch.Tensor:
        key = (weights.tobytes(), g0, m)
        v = self._views.get(key)
        if v is None:
            v = codec.views_tensor(self.pkts[:m], [float(x) for x in weights[g0:g0 + m]], self.dev)
            self._views = {key: v} if len(self._views) > 64 else {**self._views, key: v}
        return v

    def run(self, host: HostSource, clients: int, weights: Optional[np.ndarray] = None,
            sync: bool = True) -> torch.Tensor:
        """FedAVG of ``clients`` host gradients (``host[i]`` or ``host(i)``: pinned fp32 CPU
        tensors of n elements) with float32 weights (default fl32(1/M), gar.py:37-40).
        Returns the pinned host aggregate (valid after the stream syncs; ``sync`` does it)."""
        get = host if callable(host) else (lambda i: host[i])
        w = fedavg_weights(clients) if weights is None else np.asarray(weights, np.float32)
        if w.shape != (clients,):
            raise AssertionError("one weight per client (gar.py:41-42)")
        comp = torch.cuda.current_stream(self.dev)
        for e in self.enc_done:
            e.record(comp)
        for g0 in range(0, clients, self.group):
            m = min(self.group, clients - g0)
            for j in range(m):
                i = g0 + j
                s = i % self.ring
                src = get(i)
                if src.dtype != torch.float32 or src.numel() != self.n or src.is_cuda:
                    raise ValueError("host gradients must be fp32 CPU tensors of n elements")
                self.copy.wait_event(self.enc_done[s])
                with torch.cuda.stream(self.copy):
                    self.slots[s].copy_(src, non_blocking=True)
                    self.h2d_done[s].record(self.copy)
                comp.wait_event(self.h2d_done[s])
                codec.encode_top(self.slots[s], self.k, packet=self.pkts[j], check=False)
                self.enc_done[s].record(comp)
            status = self.hdrs[:m, 36:40].cpu()                 # one sync per group
            if bool((status != 0).any()):                       # exact re-encode, host copy
                for j in np.nonzero(status.numpy().view(np.uint32).ravel())[0]:
                    self.scratch.copy_(get(g0 + int(j)))
                    codec.encode_top(self.scratch, self.k, packet=self.pkts[int(j)], exact=True)
                    self.exact_fallbacks += 1
            codec.decode_accumulate(self.pkts[:m], None, out=self.acc,
                                    views=self._views_for(w, g0, m), continue_sum=g0 > 0)
        self.out_host.copy_(self.acc, non_blocking=True)
        if sync:
            torch.cuda.synchronize(self.dev)
        return self.out_host
