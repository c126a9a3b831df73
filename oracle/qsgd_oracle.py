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
    l_i   = floor(fl32(fl32(|g_i| * c) + U_i))   in [0, s];  0 if not finite,
            c = fl32(fl64(s / norm));  if that overflows, the same in fp64 with c = fl64(s / norm)
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
    s = float(2 ** bits)
    n = g.shape[0]
    w = ph.linear_words((n + 1) // 2, seed, offset)
    h = (w[np.arange(n) >> 1] >> ((np.arange(n) & 1) * 16).astype(np.uint32)) & np.uint32(0xFFFF)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        c = s / norm if norm != 0.0 else math.inf            # fl64(s / norm), once
        c32 = np.float32(c)
        if np.isfinite(c32):                                 # fp32 arithmetic
            u = h.astype(np.float32) * np.float32(2.0 ** -16)
            f = np.floor(np.abs(g.astype(np.float32)) * c32 + u)
        else:                                                # s / norm above FLT_MAX
            u = h.astype(np.float64) * 2.0 ** -16
            f = np.floor(np.abs(g.astype(np.float64)) * c + u)
    ok = np.isfinite(f) & (f >= 0) & (f <= s)
    lev = np.where(ok, f, 0).astype(np.uint32)
    sign = np.signbit(g).astype(np.uint32)
    return lev, sign


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
