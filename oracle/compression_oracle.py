"""NumPy restatement of the reference gradient codec — TEST INFRASTRUCTURE (oracle).

Restates ``ftl/compression/compression.py:8-77`` (OpenMSFTL) with the same NumPy calls, so
that it both checks the HIP codec and serves as the timed CPU baseline (kind "port").

Deliberate, documented difference: the reference's ``top``
uses NumPy's default (unstable) ``argsort``; its choice inside a group of tied magnitudes is
implementation-defined.  The oracle fixes ONE rule, ``argsort(kind="stable")[::-1]``: every
|g| above the k-th magnitude is kept, and inside the tied group the HIGHEST indices are kept
first.  NaN sorts above +inf (NumPy puts NaN last, so ``[::-1]`` takes it first).  On inputs
without a tie at the k-th magnitude this equals the reference bit for bit (pinned by
``tests/test_oracle_golden.py``).
"""
from __future__ import annotations

import numpy as np

#: Codec names understood by the reference's dispatcher (compression.py:27-77).
CODECS = ("full", "top", "rand", "dropout-biased", "dropout-unbiased", "qsgd")


def config_fields(cfg: dict):
    """compression.py:18-21 — keys and defaults, read verbatim (no validation)."""
    return (cfg.get("compression_function", "full"),
            cfg.get("num_bits", 8),
            cfg.get("fraction_coordinate", 0.5),
            cfg.get("dropout_p", 0.5))


def num_kept(fraction: float, n: int) -> int:
    """compression.py:34/42 — ``k = round(f * N)``: Python banker's rounding of the f64 product."""
    return round(fraction * n)


def effective_k(k: int, n: int) -> int:
    """How many coordinates ``idx[:k]`` really keeps (Python slice semantics, incl. k<0, k>N)."""
    return len(range(n)[:k])


def topk_indices(grad: np.ndarray, k: int, kind: str | None = "stable") -> np.ndarray:
    """compression.py:35 with the build's tie rule (stable argsort, reversed).  ``kind=None``
    is the reference's exact call (NumPy's default introsort; ties implementation-defined):
    the timed CPU baseline uses it, parity checks never do."""
    return np.argsort(np.abs(grad), kind=kind)[::-1][:k]


def compress(cfg: dict, grad, layer_wise: bool = False, rng=np.random, argsort_kind="stable"):
    """compression.py:23-77.  ``rng`` defaults to the process-global legacy ``np.random``;
    ``argsort_kind=None`` times the reference's own argsort call (bench.py cpu_baseline)."""
    func, _num_bits, frac, p = config_fields(cfg)
    if layer_wise:                                     # :24-25
        raise NotImplementedError
    if func == "full":                                 # :27-29 (returns the same object)
        return grad
    if func == "top":                                  # :31-37
        q = np.zeros_like(grad)
        k = num_kept(frac, q.shape[0])
        idx = topk_indices(grad, k, argsort_kind)
        q[idx] = grad[idx]
        return q
    if func == "rand":                                 # :39-45
        q = np.zeros_like(grad)
        k = num_kept(frac, q.shape[0])
        idx = rng.permutation(q.shape[0])[:k]
        q[idx] = grad[idx]
        return q
    if func == "dropout-biased":                       # :47-53  (float64 result)
        mask = rng.binomial(1, p, (grad.shape[0],))
        return grad * mask
    if func == "dropout-unbiased":                     # :55-60  (float64 result, / p in f64)
        mask = rng.binomial(1, p, (grad.shape[0],))
        return (grad * mask) / p
    raise NotImplementedError                          # :62-64 'qsgd', :76-77 unknown


# --------------------------------------------------------------------------------------
# Host-side RNG draws, restated separately so parity tests can feed the SAME draws to
# the GPU (consumes the legacy global stream exactly as compression.py:43/51/58 do).
# --------------------------------------------------------------------------------------
def draw_rand_indices(n: int, k: int, rng=np.random) -> np.ndarray:
    """compression.py:43 — ``np.random.permutation(N)[:k]``."""
    return rng.permutation(n)[:k]


def draw_dropout_mask(n: int, p: float, rng=np.random) -> np.ndarray:
    """compression.py:51/58 — ``np.random.binomial(1, p, (N,))`` (int64 0/1)."""
    return rng.binomial(1, p, (n,))
