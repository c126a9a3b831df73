"""NumPy's legacy MT19937 stream and ``binomial(1, p, n)`` — TEST INFRASTRUCTURE (oracle).

The reference's dropout codecs draw ``np.random.binomial(1, p, (N,))`` from the process-global
legacy ``RandomState`` (ftl/compression/compression.py:51, :58).  The algorithm lives in NumPy
(third-party, unpinned in the reference's requirements.txt:1; 2.2.6 here and on the GPU box),
so this file restates NumPy's published C code and is pinned against NumPy itself
(tests/test_mt19937.py: masks and RNG states byte-equal to ``np.random``):

* MT19937 (Matsumoto & Nishimura 1998; numpy/random/src/mt19937/mt19937.c): the raw word
  sequence x[k + 624] = x[k + 397] ^ (y >> 1) ^ (0x9908b0df if y & 1), with
  y = (x[k] & 0x80000000) | (x[k + 1] & 0x7fffffff); output = temper(x[k]).  NumPy's state
  (``get_state()``) is ('MT19937', key = x[b .. b + 624), pos, has_gauss, gauss): the next
  output is temper(x[b + pos]); key is re-twisted (b += 624) when pos reaches 624.
* ``random_sample`` (``mt19937_next_double``): U = ((a >> 5) * 2**26 + (b >> 6)) / 2**53 from two
  consecutive outputs a, b.
* ``binomial(1, p)`` (numpy/random/src/distributions/distributions.c ``random_binomial`` ->
  ``random_binomial_inversion``, used for every p when n = 1 since n*p <= 30): with
  q = 1 - p, qn = exp(n log q), X = 0, px = qn, U = next_double; while U > px: X += 1; if
  X > bound (= 1 for n = 1): X = 0, px = qn, U = next_double (a redraw); else U -= px,
  px = ((n - X + 1) * p * px) / (X * q).  For p > 0.5 the result is n - inversion(n, 1 - p).
  So for n = 1: X = (U > qn), except that U - qn > (p * qn) / q asks for a redraw — an event
  of probability ~2**-52 per draw that :func:`binomial_mask` reproduces and the device path
  flags (it then falls back to the host draw).
* Jump-ahead (Haramoto, Matsumoto, Nishimura, L'Ecuyer, Panneton 2008): the 19937-bit state
  transition A has characteristic polynomial chi (found here by Berlekamp-Massey on one bit of
  the raw sequence); with z**D = sum c_i z**i (mod chi), A**D S = sum c_i A**i S, and every raw
  word is a linear function of the state, so x[D + t] = XOR_{c_i = 1} x[i + t] for t >= 1 — the
  device's jump kernel (openmsftl_amd/csrc/fc_mt.hip) computes exactly this sum.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline import this module.
"""
from __future__ import annotations

import math
from functools import lru_cache

import numpy as np

NW, MM = 624, 397
MATRIX_A = np.uint32(0x9908B0DF)
UPPER = np.uint32(0x80000000)
LOWER = np.uint32(0x7FFFFFFF)
NBITS = 19937


def raw_sequence(key, length: int) -> np.ndarray:
    """x[0 .. length) from the 624 words x[0 .. 624) (uint32): the MT19937 recurrence, 227 new
    words at a time (x[m] needs x[m - 227], so 227 consecutive new words are independent)."""
    x = np.empty(max(length, NW), dtype=np.uint32)
    x[:NW] = np.asarray(key, dtype=np.uint32)
    m = NW
    while m < length:
        e = min(m + 227, length)
        k = np.arange(m - NW, e - NW)
        y = (x[k] & UPPER) | (x[k + 1] & LOWER)
        x[m:e] = x[k + MM] ^ (y >> np.uint32(1)) ^ np.where((y & np.uint32(1)) != 0, MATRIX_A,
                                                            np.uint32(0))
        m = e
    return x[:length]


def temper(y: np.ndarray) -> np.ndarray:
    y = np.asarray(y, dtype=np.uint32).copy()
    y ^= y >> np.uint32(11)
    y ^= (y << np.uint32(7)) & np.uint32(0x9D2C5680)
    y ^= (y << np.uint32(15)) & np.uint32(0xEFC60000)
    y ^= y >> np.uint32(18)
    return y


def state_key_pos(state=None):
    """(key uint32[624], pos) of a legacy ``get_state()`` tuple (default: np.random's)."""
    st = np.random.get_state() if state is None else state
    if st[0] != "MT19937":
        raise ValueError("not an MT19937 state")
    return np.asarray(st[1], dtype=np.uint32), int(st[2])


def outputs(key, pos: int, count: int) -> np.ndarray:
    """The next ``count`` 32-bit outputs of the state (key, pos)."""
    return temper(raw_sequence(key, pos + count)[pos:pos + count])


def doubles(words: np.ndarray) -> np.ndarray:
    """``random_sample``: one double from each consecutive pair of outputs."""
    a = (words[0::2] >> np.uint32(5)).astype(np.float64)
    b = (words[1::2] >> np.uint32(6)).astype(np.float64)
    return (a * 67108864.0 + b) / 9007199254740992.0


def binomial_params(p: float):
    """(invert, T, px2, qn) for binomial(1, p): with m = U * 2**53 (an integer),
    X = m > T; a redraw when U - qn > px2 (only possible when X = 1); the result is X, or
    1 - X when ``invert`` (p > 0.5: n - inversion(n, 1 - p))."""
    p = float(p)
    if not 0.0 <= p <= 1.0:
        raise ValueError("binomial p outside [0, 1]")
    invert = p > 0.5
    pp = 1.0 - p if invert else p
    q = 1.0 - pp
    qn = math.exp(1 * math.log(q))
    px2 = ((1 - 1 + 1) * pp * qn) / (1 * q) if q > 0 else math.inf
    return invert, math.floor(qn * 9007199254740992.0), px2, qn


def binomial_mask(key, pos: int, n: int, p: float):
    """``np.random.binomial(1, p, (n,))`` from the state (key, pos) -> (mask uint8[n], the
    state (key, pos) after the call), redraws included."""
    invert, T, px2, qn = binomial_params(p)
    words = outputs(key, pos, 2 * n)
    a = (words[0::2] >> np.uint32(5)).astype(np.uint64)
    b = (words[1::2] >> np.uint32(6)).astype(np.uint64)
    m = (a << np.uint64(26)) | b
    x = m > np.uint64(T)
    u = m.astype(np.float64) / 9007199254740992.0
    redraw = np.nonzero(x & ((u - qn) > px2))[0]
    used = 2 * n
    if redraw.size:                       # ~2**-52 per draw: replay sequentially from the first
        x = x.copy()
        stream = pos + 2 * int(redraw[0])
        for e in range(int(redraw[0]), n):
            while True:
                w = outputs(key, stream, 2)
                stream += 2
                mm = (int(w[0] >> np.uint32(5)) << 26) | int(w[1] >> np.uint32(6))
                if not (mm > T and (mm / 9007199254740992.0 - qn) > px2):
                    x[e] = mm > T
                    break
        used = stream - pos
    mask = (~x if invert else x).astype(np.uint8)
    return mask, advance(key, pos, used)


def advance(key, pos: int, count: int):
    """The state (key, pos) after ``count`` more outputs, in NumPy's form (pos in [1, 624]
    after at least one output; key re-twisted lazily)."""
    if count == 0:
        return np.asarray(key, np.uint32).copy(), pos
    end = pos + count                                # stream index of the next output
    b = NW * ((end - 1) // NW)
    x = raw_sequence(key, b + NW)
    return x[b:b + NW].copy(), end - b


# ---- GF(2) polynomials: characteristic polynomial and jumps -------------------------------------
def _bits_of_raw(x: np.ndarray) -> int:
    """Bit 31 of each raw word, as an integer (bit k = bit 31 of x[k])."""
    bits = ((x >> np.uint32(31)) & np.uint32(1)).astype(np.uint8)
    return int.from_bytes(np.packbits(bits, bitorder="little").tobytes(), "little")


@lru_cache(maxsize=1)
def charpoly() -> int:
    """chi as an integer (bit i = coefficient of z**i), degree 19937, by Berlekamp-Massey over
    the top bit of 2 * 19937 raw words of an arbitrary seed's state (MT19937's chi is
    primitive, so any non-zero bit sequence of the generator has it as minimal polynomial)."""
    rs = np.random.RandomState(12345)
    key, _ = state_key_pos(rs.get_state())
    n = 2 * NBITS + 64
    s = _bits_of_raw(raw_sequence(key, n))
    C, B = 1, 1                       # connection polynomials (bit i = coefficient of D**i)
    L, m = 0, 1
    R = 0                             # bit i = s[k - i]
    for k in range(n):
        R = (R << 1) | ((s >> k) & 1)
        if (C & R).bit_count() & 1 == 0:
            m += 1
        elif 2 * L <= k:
            C, B, L, m = C ^ (B << m), C, k + 1 - L, 1
        else:
            C ^= B << m
            m += 1
    if L != NBITS:
        raise RuntimeError(f"Berlekamp-Massey found degree {L}")
    return int(bin(C)[2:].zfill(L + 1)[::-1], 2)    # chi(z) = z**L C(1/z)


def _mod(a: int, P: int) -> int:
    dp = P.bit_length() - 1
    while a.bit_length() - 1 >= dp:
        a ^= P << (a.bit_length() - 1 - dp)
    return a


def _square(a: int) -> int:
    """a(z)**2 over GF(2): spread the bits."""
    b = np.frombuffer(a.to_bytes((a.bit_length() + 7) // 8 or 1, "little"), dtype=np.uint8)
    bits = np.unpackbits(b, bitorder="little")
    sp = np.zeros(bits.size * 2, dtype=np.uint8)
    sp[0::2] = bits
    return int.from_bytes(np.packbits(sp, bitorder="little").tobytes(), "little")


def jump_poly(D: int) -> int:
    """z**D mod chi (bit i = c_i)."""
    P = charpoly()
    r = 1
    for bit in bin(D)[2:]:
        r = _mod(_square(r), P)
        if bit == "1":
            r = _mod(r << 1, P)
    return r


def jump_words(x: np.ndarray, c: int, t_count: int = NW + 1) -> np.ndarray:
    """XOR_{c_i = 1} x[i + t] for t = 0 .. t_count - 1 (x must hold 19937 + t_count words):
    = x[D + t] for t >= 1 when c = z**D mod chi and x is a raw sequence."""
    out = np.zeros(t_count, dtype=np.uint32)
    bits = np.unpackbits(np.frombuffer(c.to_bytes(NBITS // 8 + 1, "little"), dtype=np.uint8),
                         bitorder="little")[:NBITS]
    for i in np.nonzero(bits)[0]:
        out ^= x[i:i + t_count]
    return out
