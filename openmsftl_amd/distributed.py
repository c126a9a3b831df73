"""Multi-GPU FedAVG over client packets: one process per GPU.

The reference runs every client in one process and reduces a dense host matrix
(``aggregation.py:61-63`` -> ``gar.py:44``).  Here the sampled clients (``server.py:74``
order) are split into contiguous shards, rank r owning rows ``shard_range(M, W, r)`` of that
G.  Each rank encodes and decode-accumulates its own shard with no collective on the data
path, then combines the per-rank partial sums in one of two ways:

``mode="reduce"`` (default)
    one fp32 sum-reduce of the 4N-byte partial aggregates to ``dst`` (RCCL over xGMI with the
    ``nccl`` backend).  The M-row left-to-right sum is reassociated at the W shard
    boundaries only: ``|agg - gar.py:44| <= (M + W) * 2**-24 * sum_i |fl(w_i * d_i)|``.
``mode="chain"``
    bit-identical to one GPU: rank r receives rank r-1's partial sum, continues the same
    left-to-right fold over its own rows (``fc_decode_accumulate_continue``) and passes it
    on; the last rank sends the result to ``dst``.  Costs W-1 point-to-point hops of 4N
    bytes, serialised behind each rank's fold.

The local fold is a callable so the same orchestration drives the HIP packets
(:func:`packet_fold`) and, in the CPU tests, a plain sequential sum over gloo.

Backends: with ``nccl`` (RCCL over xGMI) the device tensors travel directly; gloo has no
device ``reduce``/``send``/``recv``, so for a device ``out`` on a gloo group the partial sums
are staged through host memory (same bytes, same order of additions: the chain stays
bit-exact; tests/test_distributed_gpu.py runs two gloo ranks on one GPU that way).
``aggregate(..., async_op=True)`` (reduce mode, RCCL) returns the collective's work handle
instead of waiting, so a caller with a second ``out`` buffer overlaps the reduce of step i
with the encodes of step i+1 (bench.py does).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

#: local_fold(rows: range, weights: np.ndarray (float32, per row), out, continue_sum) -> out
Fold = Callable[[range, np.ndarray, object, bool], object]


def shard_range(num_clients: int, world: int, rank: int) -> range:
    """Contiguous, balanced shard of G's rows for ``rank`` (the first M % W ranks get one
    extra row).  Shards are in rank order, so concatenating them gives rows 0..M-1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    if num_clients < 0:
        raise ValueError("num_clients < 0")
    base, rem = divmod(num_clients, world)
    start = rank * base + min(rank, rem)
    return range(start, start + base + (1 if rank < rem else 0))


def fedavg_weights(num_clients: int) -> np.ndarray:
    """``np.full(M, 1/M, dtype=G.dtype)`` for float32 G (gar.py:37-40)."""
    if num_clients < 1:
        raise Exception("Empty gradient list")   # aggregation.py:59-60 (same exception type)
    return np.full(num_clients, fill_value=1.0 / num_clients, dtype=np.float32)


class ShardedFedAvg:
    """Per-rank fold + cross-rank combine of FedAVG partial sums."""

    def __init__(self, mode: str = "reduce", dst: int = 0, group=None,
                 always_collective: bool = False):
        """``always_collective``: issue the reduce even in a world of one (an initialised
        process group of one rank: RCCL's one-rank reduce is a device copy), so one GPU runs
        the multi-GPU code path — the collective, its async work handle and its stream
        ordering against the next encodes (bench.py / tools/e2e_bench.py ``--force-pg``)."""
        if mode not in ("reduce", "chain"):
            raise ValueError(f"mode must be 'reduce' or 'chain' (got {mode!r})")
        self.mode, self.dst, self.group = mode, dst, group
        self.always_collective = always_collective

    def _staged(self, t) -> bool:
        """gloo group + device tensor: communicate through a host copy."""
        import torch.distributed as dist
        return t.is_cuda and dist.get_backend(self.group) == "gloo"

    def _reduce(self, out, async_op: bool):
        import torch.distributed as dist
        if self._staged(out):
            h = out.cpu()
            dist.reduce(h, dst=self.dst, op=dist.ReduceOp.SUM, group=self.group)
            if dist.get_rank(self.group) == self.dst:
                out.copy_(h)
            return None
        return dist.reduce(out, dst=self.dst, op=dist.ReduceOp.SUM, group=self.group,
                           async_op=async_op)

    def _send(self, out, dst: int):
        import torch.distributed as dist
        dist.send(out.cpu() if self._staged(out) else out, dst=dst, group=self.group)

    def _recv(self, out, src: int):
        import torch.distributed as dist
        if self._staged(out):
            h = _host_like(out)
            dist.recv(h, src=src, group=self.group)
            out.copy_(h)
        else:
            dist.recv(out, src=src, group=self.group)

    @staticmethod
    def _initialized() -> bool:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized()

    def _world(self):
        import torch.distributed as dist
        if not dist.is_available() or not dist.is_initialized():
            return 1, 0
        return dist.get_world_size(self.group), dist.get_rank(self.group)

    def aggregate(self, local_fold: Fold, num_clients: int, out, weights=None,
                  async_op: bool = False):
        """Fold this rank's shard into ``out`` and combine across ranks.  The complete
        aggregate is valid on ``dst`` only (``out`` elsewhere holds scratch).  ``weights``:
        float32 per G row (default 1/M each, gar.py:37-40).  ``async_op`` (reduce mode):
        return the reduce's work handle (``None`` when there is nothing to wait for) and
        leave ``out`` in flight until ``handle.wait()``."""
        world, rank = self._world()
        w = fedavg_weights(num_clients) if weights is None else np.asarray(weights, np.float32)
        if w.shape != (num_clients,):
            raise AssertionError("weights must have one entry per client")   # gar.py:41-42
        rows = shard_range(num_clients, world, rank)
        if world == 1 and not (self.always_collective and self.mode == "reduce"
                               and self._initialized()):
            local_fold(rows, w[rows.start:rows.stop], out, False)
            return None if async_op else out
        if self.mode == "reduce":
            if len(rows):
                local_fold(rows, w[rows.start:rows.stop], out, False)
            else:
                out.zero_()                      # empty shard adds nothing
            work = self._reduce(out, async_op)
            return work if async_op else out
        if async_op:
            raise ValueError("async_op is for mode='reduce' (the chain is serial by design)")
        # chain: rank r continues rank r-1's left-to-right fold (bit-identical to 1 GPU)
        first = min(r for r in range(world) if len(shard_range(num_clients, world, r)))
        last = max(r for r in range(world) if len(shard_range(num_clients, world, r)))
        if len(rows):
            if rank != first:
                self._recv(out, self._prev(rank, num_clients, world))
            local_fold(rows, w[rows.start:rows.stop], out, rank != first)
            if rank != last:
                self._send(out, self._next(rank, num_clients, world))
        if last != self.dst:
            if rank == last:
                self._send(out, self.dst)
            elif rank == self.dst:
                self._recv(out, last)
        return out

    @staticmethod
    def _prev(rank, m, world):
        return max(r for r in range(rank) if len(shard_range(m, world, r)))

    @staticmethod
    def _next(rank, m, world):
        return min(r for r in range(rank + 1, world) if len(shard_range(m, world, r)))


def _host_like(t):
    import torch
    return torch.empty(t.shape, dtype=t.dtype)


def packet_fold(packets, views=None) -> Fold:
    """Local fold over this rank's device packets (HIP ``k_decode<ACC>``).  ``packets`` are
    the shard's packets in row order; ``views`` an optional prebuilt view array."""
    from . import codec

    def fold(rows: range, w: np.ndarray, out, continue_sum: bool):
        if len(rows) != len(packets):
            raise ValueError(f"shard has {len(rows)} rows but {len(packets)} packets")
        return codec.decode_accumulate(packets, [float(x) for x in w], out=out,
                                       views=views, continue_sum=continue_sum)
    return fold
