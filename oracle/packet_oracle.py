"""CPU restatement of the HIP codec's packet semantics — TEST INFRASTRUCTURE (oracle).

The reference has no wire format (``compression.py:33-37`` returns a dense vector), so the
packet is the build's own.  This module states its rules on the CPU so the GPU packet can
be checked field by field; the selection rule itself is pinned to the reference by
``compression_oracle.topk_indices`` (stable argsort, reversed) — see
``tests/test_oracle_golden.py::test_composite_rule_equals_stable_argsort``.

Composite key (fc_common.h):
  key(x)  = bits(x) & 0x7fffffff, with every NaN mapped to 0x7f800001 (above +inf)
  IB      = index bits = max(1, ceil(log2 N))
  comp(i) = key(g[i]) << IB | i          (unique per element)
  top-k   = the k largest comps  <=>  argsort(|g|, stable)[::-1][:k]
  T64     = the k-th largest comp; selected  <=>  comp >= T64
A packet lists, in ascending index order, every element whose comp >= L64 (a lower bound
found by the sampled bracket, L64 <= T64); the decoder keeps entries with comp >= T64.
"""
from __future__ import annotations

import numpy as np

NAN_KEY = np.uint32(0x7F800001)
NOTHING = np.uint64(1) << np.uint64(63)       # T64 that selects nothing (k == 0)


def index_bits(n: int) -> int:
    return max(1, int(n - 1).bit_length()) if n > 1 else 1


def mag_key(g: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(g, dtype=np.float32).view(np.uint32) & np.uint32(0x7FFFFFFF)
    return np.where(u > np.uint32(0x7F800000), NAN_KEY, u).astype(np.uint32)


def comps(keys: np.ndarray) -> np.ndarray:
    n = keys.shape[0]
    ib = np.uint64(index_bits(n))
    return (keys.astype(np.uint64) << ib) | np.arange(n, dtype=np.uint64)


def threshold(keys: np.ndarray, k: int) -> np.uint64:
    """T64 for ``k`` kept coordinates (0 <= k <= N)."""
    n = keys.shape[0]
    if k <= 0:
        return NOTHING
    if k >= n:
        return np.uint64(0)
    c = comps(keys)
    return np.partition(c, n - k)[n - k]


def selected_indices(keys: np.ndarray, k: int) -> np.ndarray:
    """Ascending indices of the k largest comps."""
    t = threshold(keys, k)
    return np.nonzero(comps(keys) >= t)[0].astype(np.uint32)


def topk_packet(g: np.ndarray, k: int):
    """(idx ascending uint32, val float32 bit-copies) of the exact top-k packet."""
    idx = selected_indices(mag_key(g), k)
    return idx, np.ascontiguousarray(g, dtype=np.float32)[idx]


def decode_dense(n: int, idx: np.ndarray, val: np.ndarray) -> np.ndarray:
    out = np.zeros(n, dtype=np.float32)
    out[idx] = val
    return out
