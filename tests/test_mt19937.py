"""NumPy's legacy MT19937 stream and binomial(1, p) — the reference's dropout draws on the device.

compression.py:51 / :58 draw ``np.random.binomial(1, p, (N,))`` from the global legacy
RandomState.  The HIP path (openmsftl_amd/csrc/fc_mt.hip) reproduces that stream by jump-ahead;
its pin is NumPy itself (2.2.6 here and on the GPU box):

CPU: oracle/mt19937.py against ``np.random`` (masks, RNG state after the call, several p, an
odd and the post-seed start position); the library's host polynomials (fc_mt_charpoly,
fc_mt_jump_poly) against the oracle's Berlekamp-Massey / square-and-multiply and against
direct generation.  GPU: fc_mt_begin / fc_mt_binomial masks and end state against
``np.random`` at ragged and full sizes, several rows per round."""
import numpy as np
import pytest

from oracle import mt19937 as mt


@pytest.mark.parametrize("p", [0.0, 1e-12, 0.1, 0.3, 0.5, 0.5000001, 0.7, 0.9, 1.0])
@pytest.mark.parametrize("pre", [0, 1, 3, 623])
def test_oracle_binomial_equals_numpy(p, pre):
    """oracle.binomial_mask == np.random.binomial(1, p, n), and the state after it."""
    np.random.seed(7 + pre)
    if pre:
        np.random.random_sample(pre)              # odd / late start positions in the key block
    key, pos = mt.state_key_pos()
    n = 20_011
    want = np.random.binomial(1, p, (n,))
    got, (k2, p2) = mt.binomial_mask(key, pos, n, p)
    assert (got == want).all()
    st = np.random.get_state()
    assert (k2 == st[1]).all() and p2 == st[2]


def test_oracle_raw_stream_is_numpys():
    """temper(x[pos + i]) are np.random's 32-bit outputs; doubles are random_sample."""
    np.random.seed(123)
    np.random.random_sample(5)
    key, pos = mt.state_key_pos()
    want = np.random.random_sample(1000)
    assert (mt.doubles(mt.outputs(key, pos, 2000)) == want).all()


def test_oracle_jump_equals_generation():
    """x[D + t] = XOR_{c_i} x[i + t] (t >= 1) for c = z**D mod chi."""
    key, _ = mt.state_key_pos(np.random.RandomState(3).get_state())
    x = mt.raw_sequence(key, mt.NBITS + 626)
    for D in (1, 624, 40_000, 1_234_567):
        y = mt.jump_words(x, mt.jump_poly(D))
        ref = mt.raw_sequence(key, D + 626)[D:D + 625]
        assert (y[1:] == ref[1:]).all(), D


def _lib_poly(fn, *args) -> int:
    from openmsftl_amd import _lib as L
    buf = np.zeros(624, np.uint32)
    L.check(getattr(L.load(), fn)(*args, buf.ctypes.data), fn)
    return int.from_bytes(buf.tobytes(), "little")


def test_library_charpoly_equals_oracle():
    """fc_mt_charpoly (C++ Berlekamp-Massey, host) == the oracle's (Python)."""
    chi = _lib_poly("fc_mt_charpoly")
    assert chi.bit_length() - 1 == mt.NBITS and chi & 1
    assert chi == mt.charpoly()


@pytest.mark.parametrize("D", [0, 1, 19_936, 19_937, 19_938, 2_000_001, 2 * 25_557_032 - 1])
def test_library_jump_poly_equals_oracle(D):
    """fc_mt_jump_poly (carry-less multiplies + Barrett reduction) == square-and-multiply."""
    assert _lib_poly("fc_mt_jump_poly", D) == mt.jump_poly(D)


def test_library_jump_poly_jumps_far():
    """A jump the size of 64 rows of 25.5 M draws, checked by the jump itself: from x the
    polynomial's sum lands where generating 624 * 2 past a second, nearby jump lands."""
    key, _ = mt.state_key_pos(np.random.RandomState(9).get_state())
    x = mt.raw_sequence(key, mt.NBITS + 626)
    D = 64 * 2 * 25_557_032 - 1
    a = mt.jump_words(x, _lib_poly("fc_mt_jump_poly", D))              # x[D + 1 .. D + 625)
    b = mt.jump_words(x, _lib_poly("fc_mt_jump_poly", D - 1300))       # x[D - 1299 .. D - 675)
    again = mt.raw_sequence(b[1:], 1300 + 624 + 2)                     # x[D - 1299 ...] onward
    assert (again[1300:1300 + 624] == a[1:625]).all()


# ---- GPU: the device stream against np.random ------------------------------------------------
def _device_round(n, ps, seed, pre):
    import torch
    from openmsftl_amd import codec
    from openmsftl_amd.compression import bitmask_words
    np.random.seed(seed)
    if pre:
        np.random.random_sample(pre)
    key, pos, _, _ = codec.mt_state()
    want = [bitmask_words(np.random.binomial(1, p, (n,)), n, True) for p in ps]
    st = np.random.get_state()
    R = codec.MtRound(n, len(ps), key, pos, torch.device("cuda", 0))
    got = [R.binomial(r, p).cpu().numpy().view(np.uint32) for r, p in enumerate(ps)]
    k2, p2, redraw = R.end_state()
    return got, want, (k2, p2, redraw), st


@pytest.mark.gpu
@pytest.mark.parametrize("n,ps,seed,pre", [
    (1, [0.3, 0.6], 1, 0),                              # one element per row
    (31, [0.5, 0.5, 0.0, 1.0], 2, 623),                 # ragged word, p = 0 / 1, pos 624
    (100_003, [0.1, 0.7, 0.5], 3, 5),                   # several segments, odd pos
    (32_768 * 3, [0.25], 4, 2),                         # exact segment multiple
    (1_000_000, [0.1] * 5, 5, 1),                       # five rows: level-1 jumps
])
def test_device_binomial_equals_numpy(n, ps, seed, pre):
    got, want, (k2, p2, redraw), st = _device_round(n, ps, seed, pre)
    for r, (g, w) in enumerate(zip(got, want)):
        assert g.tobytes() == w.tobytes(), f"row {r}"
    assert not redraw
    assert (k2 == st[1]).all() and p2 == st[2]


@pytest.mark.gpu
def test_device_binomial_full_size_rows():
    """Two 25.5 M rows (configs[4]'s gradient length), p = 0.1 and 0.9."""
    got, want, (k2, p2, redraw), st = _device_round(25_557_032, [0.1, 0.9], 11, 1)
    for g, w in zip(got, want):
        assert g.tobytes() == w.tobytes()
    assert not redraw and (k2 == st[1]).all() and p2 == st[2]


@pytest.mark.gpu
def test_device_plan_made_for_more_rows_serves_a_shorter_round():
    """MtPlan is cached per (device, n) with a row capacity: a round of fewer rows than the
    plan holds reads the same segment polynomials (plan layout independent of capacity)."""
    import torch
    from openmsftl_amd import codec
    dev = torch.device("cuda", 0)
    codec.MtPlan.get(100_003, 40, dev)
    for rows in (3, 1):
        got, want, (k2, p2, redraw), st = _device_round(100_003, [0.2] * rows, 21 + rows, 7)
        assert all(g.tobytes() == w.tobytes() for g, w in zip(got, want))
        assert (k2 == st[1]).all() and p2 == st[2]


@pytest.mark.gpu
@pytest.mark.parametrize("codec_name", ["dropout-biased", "dropout-unbiased"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n,p", [(1, 0.5), (4099, 0.1), (300_001, 0.7), (1_000_000, 1.0)])
def test_compress_dropout_device_draws_equal_host_draws(codec_name, dtype, n, p, monkeypatch):
    """The drop-in compress() (compression.py:47-60) with np.random's draws made on the device
    returns the same float64 bytes as with NumPy's own np.random.binomial call, and leaves
    np.random in the same state."""
    from openmsftl_amd import compression
    from openmsftl_amd.compression import Compression
    g = np.random.default_rng(n).standard_normal(n).astype(dtype)
    g[::97] = -0.0
    C = Compression({"compression_function": codec_name, "dropout_p": p})
    outs, nxt = [], []
    for device_mt in (True, False):
        monkeypatch.setattr(compression, "DEVICE_MT", device_mt)
        np.random.seed(n % 1000)
        np.random.random_sample(3)
        outs.append(C.compress(g))
        nxt.append(int(np.random.randint(0, 2 ** 31 - 1)))
    assert outs[0].dtype == np.float64 and outs[0].tobytes() == outs[1].tobytes()
    assert nxt[0] == nxt[1]
