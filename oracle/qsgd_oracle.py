"""NumPy restatement of the QSGD codec — TEST INFRASTRUCTURE (oracle).

The reference's ``'qsgd'`` branch raises ``NotImplementedError`` (``compression.py:62-64``)
and keeps the quantiser only as a comment (``compression.py:65-74``):

    s = 2 ** bits;  tau = 1 + min(sqrt(d) / s, d / s**2)
    q = (sign(x) * ||x||) / (s * tau) * floor(s * |x| / ||x|| + U),  U ~ Uniform[0, 1)

(Alistarh et al., "QSGD: Communication-efficient SGD via gradient quantization and
encoding", NeurIPS 2017).  There is no reference output to pin against: **parity unpinned**
with respect to the reference.  This module states the exact arithmetic the HIP codec
(openmsftl_amd/csrc/fc_qsgd.hip) implements, so the GPU is pinned to it bit for bit:

    U_i   = h_i * 2**-16,  h_i = 16-bit half (i & 1) of linear word (i >> 1)
            (oracle/philox.py linear_words: one Philox block per 8 elements)
    l_i   = min(s, floor(fl32(|g_i| * c) + U_i))  (the sum exact, in fp64);  0 if NaN,
            c = fl32(fl64(s / norm));  if that overflows, fl64(|g_i| * c) with c = fl64(s / norm)
            (round 5: the sum used to be an fp32 round-to-nearest add, which could reach s + 1,
            and a level above s was dropped to 0)
    code  = signbit(g_i) << (W - 1) | l_i,  W = 4 / 8 / 16 bits for bits <= 2 / 6 / 14
    value = fl32(+-(norm / (s * tau)) * l_i)         (fp64 product, one rounding)

``norm`` is ||g||_2 in fp64; the GPU sums the squares in its own fixed order and records the
result in the packet header, and the tests check it against :func:`norm64` with a relative
tolerance of 1e-12 (fp64 reassociation), then feed the header's norm to :func:`encode`.
"""
from __future__ import annotations

import math

import numpy as np

from . import philox as ph


def width(bits: int) -> int:
    return 4 if bits <= 2 else 8 if bits <= 6 else 16


def tau(n: int, s: float) -> float:
    return 1.0 + min(math.sqrt(n) / s, n / (s * s))


def norm64(g: np.ndarray) -> float:
    return math.sqrt(float(np.sum(np.square(g.astype(np.float64)))))


def levels_and_signs(g: np.ndarray, bits: int, seed: int, offset: int, norm: float):
    n = g.shape[0]
    w = ph.linear_words((n + 1) // 2, seed, offset)
    h = (w[np.arange(n) >> 1] >> ((np.arange(n) & 1) * 16).astype(np.uint32)) & np.uint32(0xFFFF)
    return levels_from_dither(g, h, bits, norm), np.signbit(g).astype(np.uint32)


def levels_from_dither(g: np.ndarray, h: np.ndarray, bits: int, norm: float) -> np.ndarray:
    """The levels for given 16-bit dither values h (U = h / 2**16)."""
    s = float(2 ** bits)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        c = s / norm if norm != 0.0 else math.inf            # fl64(s / norm), once
        c32 = np.float32(c)
        u = h.astype(np.float64) * 2.0 ** -16                # exact
        if np.isfinite(c32):                                 # fp32 product, exact sum
            p = (np.abs(g.astype(np.float32)) * c32).astype(np.float64)
        else:                                                # s / norm above FLT_MAX
            p = np.abs(g.astype(np.float64)) * c
        f = np.floor(p + u)
        # NaN -> 0; the fp32 product may overshoot s (the exact s|g|/norm + U is < s + 1): s
        return np.where(f >= 0, np.minimum(f, s), 0).astype(np.uint32)


def encode(g: np.ndarray, bits: int, seed: int, offset: int, norm: float) -> np.ndarray:
    """Packed codes (uint32 words, little-endian W-bit fields, groups of 8 elements)."""
    W = width(bits)
    lev, sign = levels_and_signs(g, bits, seed, offset, norm)
    codes = (sign << np.uint32(W - 1)) | lev
    n = g.shape[0]
    groups = (n + 7) // 8
    c = np.zeros(groups * 8, dtype=np.uint64)
    c[:n] = codes
    per = 32 // W
    c = c.reshape(-1, per)
    shifts = (np.arange(per, dtype=np.uint64) * np.uint64(W))
    words = np.bitwise_or.reduce(c << shifts, axis=1).astype(np.uint32)
    return words


def unpack(words: np.ndarray, n: int, bits: int) -> np.ndarray:
    W = width(bits)
    per = 32 // W
    w = np.asarray(words, dtype=np.uint64).reshape(-1, 1)
    shifts = (np.arange(per, dtype=np.uint64) * np.uint64(W)).reshape(1, -1)
    c = ((w >> shifts) & np.uint64((1 << W) - 1)).reshape(-1)
    return c[:n].astype(np.uint32)


def decode(words: np.ndarray, n: int, bits: int, norm: float) -> np.ndarray:
    W = width(bits)
    s = float(2 ** bits)
    c = unpack(words, n, bits)
    lev = (c & np.uint32((1 << (W - 1)) - 1)).astype(np.float64)
    with np.errstate(invalid="ignore", over="ignore"):
        v = (norm / (s * tau(n, s))) * lev
    v = np.where((c >> np.uint32(W - 1)) & np.uint32(1), -v, v)
    return v.astype(np.float32)


def compress(g: np.ndarray, bits: int, seed: int, offset: int, norm: float | None = None):
    """The dense array the reference's commented formula returns (float32)."""
    if norm is None:
        norm = norm64(g)
    return decode(encode(g, bits, seed, offset, norm), g.shape[0], bits, norm)
