"""Philox4x32-10 counter-based RNG in NumPy — TEST INFRASTRUCTURE (oracle).

Published algorithm: J. Salmon, M. Moraes, R. Dror, D. Shaw, "Parallel random numbers: as
easy as 1, 2, 3", SC'11 (Random123).  The reference codec draws from NumPy's legacy MT19937
(``compression.py:43,51,58``); the HIP codec's *native* RNG mode uses Philox instead, so its
streams are pinned here (KAT vectors below) and NOT against the reference — "parity
unpinned" w.r.t. the reference for native-RNG mode; the numpy-RNG parity mode is exact.

Stream layout used by the HIP kernels (openmsftl_amd/csrc/fc_common.h):
  codec keys / Bernoulli masks (``element_words``):
      element i  ->  block b = ((i >> 8) << 6) | (i & 63),  word (i >> 6) & 3
  QSGD dither (``linear_words``):
      element i  ->  block b = i >> 2,  word i & 3
  with ctr = (lo32 b, hi32 b, lo32 offset, hi32 offset), key = (lo32 seed, hi32 seed).
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

#: Random123 known-answer vectors for philox4x32-10: (ctr[4], key[2]) -> out[4].
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over uint32 arrays; returns four uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint32) for c in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint32) + np.zeros_like(c0)
    k1 = np.asarray(k1, dtype=np.uint32) + np.zeros_like(c0)
    for r in range(10):
        if r:
            k0 = ((k0.astype(np.uint64) + np.uint64(W0)) & MASK32).astype(np.uint32)
            k1 = ((k1.astype(np.uint64) + np.uint64(W1)) & MASK32).astype(np.uint32)
        p0 = c0.astype(np.uint64) * M0
        p1 = c2.astype(np.uint64) * M1
        hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
        lo0 = (p0 & MASK32).astype(np.uint32)
        hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
        lo1 = (p1 & MASK32).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def _words(idx: np.ndarray, b: np.ndarray, word: np.ndarray, seed: int, offset: int):
    blocks, inv = np.unique(b, return_inverse=True)
    outs = philox4x32_10(blocks & MASK32, blocks >> np.uint64(32),
                         np.uint32(offset & 0xFFFFFFFF), np.uint32((offset >> 32) & 0xFFFFFFFF),
                         np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF))
    table = np.stack(outs, axis=1)                      # (nblocks, 4)
    return table[inv, word.astype(np.int64)]


def element_words(n: int, seed: int, offset: int = 0, start: int = 0) -> np.ndarray:
    """The 32-bit Philox word the HIP codec assigns to elements ``start .. start+n-1`` (rand-k
    keys, Bernoulli masks): block ((i >> 8) << 6) | (i & 63), word (i >> 6) & 3."""
    if n == 0:
        return np.zeros(0, dtype=np.uint32)
    idx = np.arange(start, start + n, dtype=np.uint64)
    b = ((idx >> np.uint64(8)) << np.uint64(6)) | (idx & np.uint64(63))
    return _words(idx, b, (idx >> np.uint64(6)) & np.uint64(3), seed, offset)


def linear_words(n: int, seed: int, offset: int = 0, start: int = 0) -> np.ndarray:
    """Linear word map: word i = word i & 3 of counter block i >> 2.  QSGD dithers element e
    with the 16-bit half (e & 1) of word e >> 1 (fc_qsgd.hip, oracle/qsgd_oracle.py)."""
    if n == 0:
        return np.zeros(0, dtype=np.uint32)
    idx = np.arange(start, start + n, dtype=np.uint64)
    return _words(idx, idx >> np.uint64(2), idx & np.uint64(3), seed, offset)


def bernoulli_threshold(p: float) -> int:
    """keep iff word < thr, thr = round(p * 2**32) in [0, 2**32] (fc_common.h)."""
    return int(min(max(round(p * 4294967296.0), 0), 4294967296))


def bernoulli_mask(n: int, p: float, seed: int, offset: int = 0) -> np.ndarray:
    return element_words(n, seed, offset).astype(np.uint64) < np.uint64(bernoulli_threshold(p))
