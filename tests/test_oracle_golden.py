"""Pin the CPU oracle to golden vectors produced by the REFERENCE (tests/golden/make_golden.py).

CPU only.  These tests are what makes the oracle trustworthy as the GPU checker.
"""
import hashlib

import numpy as np
import pytest

from conftest import golden, has_tie_at_boundary
from oracle import compression_oracle as co
from oracle import gar_oracle as go
from oracle import packet_oracle as po

G = golden()


def _same(a, b):
    """Equal as the reference's consumers see it: NaN==NaN, dtype equal, values equal."""
    assert a.dtype == b.dtype, (a.dtype, b.dtype)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("name", G.cases("top__"))
def test_top_matches_reference(name):
    m = G.meta(name)
    g = G.input(name)
    ref = G.arr(name, "output")
    out = co.compress({"compression_function": "top", "fraction_coordinate": m["fraction"]}, g)
    k = co.effective_k(co.num_kept(m["fraction"], g.shape[0]), g.shape[0])
    if not has_tie_at_boundary(g, k):
        # tie-free at the cut: the reference is fully determined -> bit-exact
        assert out.tobytes() == ref.tobytes()
        return
    # tie group straddles the cut: the reference's pick is implementation-defined
    # (unstable argsort); both must keep everything above the tie and the same count in it.
    keys = po.mag_key(g)
    t = np.sort(keys)[::-1][k - 1]
    sel_ref = np.zeros(g.shape[0], bool)
    sel_out = np.zeros(g.shape[0], bool)
    sel_ref[np.nonzero(ref.view(np.uint32) != 0)[0]] = True
    sel_out[np.nonzero(out.view(np.uint32) != 0)[0]] = True
    above = keys > t
    nz = keys != 0  # zeros are invisible in a dense output
    assert np.all(sel_ref[above & nz]) and np.all(sel_out[above & nz])
    assert not np.any(sel_ref[(keys < t)]) and not np.any(sel_out[(keys < t)])
    assert sel_ref[keys == t].sum() == sel_out[keys == t].sum()


def test_top_tie_rule_is_highest_index_first():
    g = np.array([1.0, -1.0, 1.0, 0.5, -1.0], dtype=np.float32)
    out = co.compress({"compression_function": "top", "fraction_coordinate": 0.4}, g)  # k=2
    assert list(np.nonzero(out)[0]) == [2, 4]


@pytest.mark.parametrize("name", G.cases("top__"))
def test_composite_rule_equals_stable_argsort(name):
    """The HIP codec's composite-key rule (packet_oracle) == the oracle's argsort rule."""
    m = G.meta(name)
    g = G.input(name)
    n = g.shape[0]
    k = co.effective_k(co.num_kept(m["fraction"], n), n)
    want = np.sort(co.topk_indices(g, co.num_kept(m["fraction"], n))).astype(np.uint32)
    got = po.selected_indices(po.mag_key(g), k)
    np.testing.assert_array_equal(got, want)


def test_full_returns_same_object():
    name = "full__gauss_1000"
    assert G.meta(name)["same_object"] is True
    g = G.input(name)
    assert co.compress({"compression_function": "full"}, g) is g


@pytest.mark.parametrize("name", G.cases("rand__"))
def test_rand_matches_reference(name):
    m = G.meta(name)
    g = G.input(name)
    np.random.seed(m["seed"])
    out = co.compress({"compression_function": "rand", "fraction_coordinate": m["fraction"]}, g)
    assert int(np.random.randint(0, 2**31 - 1)) == m["rng_next"]   # same RNG consumption
    _same(out, G.arr(name, "output"))
    assert out.tobytes() == G.arr(name, "output").tobytes()


@pytest.mark.parametrize("name", G.cases("dropout-"))
def test_dropout_matches_reference(name):
    m = G.meta(name)
    g = G.input(name)
    np.random.seed(m["seed"])
    with np.errstate(invalid="ignore"):
        out = co.compress({"compression_function": m["codec"], "dropout_p": m["p"]}, g)
    if "rng_next" in m:
        assert int(np.random.randint(0, 2**31 - 1)) == m["rng_next"]
    ref = G.arr(name, "output")
    assert out.dtype == np.float64 and ref.dtype == np.float64
    assert out.tobytes() == ref.tobytes()


@pytest.mark.parametrize("name", G.cases("fedavg__"))
def test_fedavg_matches_reference(name):
    Gm = G.arr(name, "G")
    ref = G.arr(name, "output")
    out = go.FedAvgOracle({"aggregation_scheme": "fed_avg"}).aggregate(Gm)
    assert out.tobytes() == ref.tobytes()
    w = np.full(Gm.shape[0], 1.0 / Gm.shape[0], dtype=np.float32)
    seq = go.sequential_weighted_sum(list(Gm), w)
    assert seq.tobytes() == ref.tobytes()          # left-to-right fp32 chain


def test_fedavg_weights_persist_and_assert_M():
    f = go.FedAvgOracle({})
    f.aggregate(np.ones((4, 3), np.float32))
    with pytest.raises(AssertionError):
        f.aggregate(np.ones((5, 3), np.float32))


def test_error_surface_matches_reference():
    errs = G.manifest["errors"]
    assert errs == {"bogus|False": "NotImplementedError", "qsgd|False": "NotImplementedError",
                    "top|True": "NotImplementedError"}
    for fn, lw in (("qsgd", False), ("bogus", False), ("top", True)):
        with pytest.raises(NotImplementedError):
            co.compress({"compression_function": fn}, np.ones(8, np.float32), layer_wise=lw)


def test_bankers_rounding_k():
    assert co.num_kept(0.5, 5) == 2 and co.num_kept(0.5, 7) == 4
    assert co.effective_k(-1, 10) == 9 and co.effective_k(15, 10) == 10


@pytest.mark.parametrize("key", sorted(G.manifest["large"]))
def test_large_digest_via_composite_rule(key):
    """16 M / 25.5 M top-k: the composite rule reproduces the reference's digests."""
    d = G.manifest["large"][key]
    if d["n"] > 20_000_000:
        pytest.skip("25.5 M case checked in the GPU suite to keep the CPU suite short")
    g = np.random.default_rng(d["seed"]).standard_normal(d["n"], dtype=np.float32)
    idx, val = po.topk_packet(g, d["k"])
    assert hashlib.sha256(idx.tobytes()).hexdigest() == d["sorted_idx_sha256"]
    out = po.decode_dense(d["n"], idx, val)
    assert hashlib.sha256(out.tobytes()).hexdigest() == d["output_sha256"]


def test_philox_known_answers():
    from oracle.philox import KAT, philox4x32_10
    for ctr, key, want in KAT:
        got = philox4x32_10(*[np.uint32(c) for c in ctr], *[np.uint32(k) for k in key])
        assert tuple(int(x) for x in got) == want


# ---- aggregation rows (tests/golden/make_golden_agg.py: the reference's own outputs) ------
from conftest import agg_golden  # noqa: E402

A = agg_golden()


def test_numpy_axis0_sum_order():
    """gar.py:44's np.sum(axis=0) = row-order fp32 adds starting from +0: an all-(-0) column
    sums to +0, a one-row G too; nonzero values equal the plain left-to-right chain."""
    rng = np.random.default_rng(5)
    for M in (1, 2, 7, 64):
        Gm = (rng.standard_normal((M, 999)) * 10.0 ** rng.uniform(-6, 3, (M, 1))).astype(np.float32)
        Gm[:, :50] = -0.0
        Gm[:, 50:60] = -np.float32(1e-45)
        w = np.full(M, 1.0 / M, np.float32)
        ref = np.sum(np.multiply(Gm, w[:, None]), axis=0)
        assert go.sequential_weighted_sum(list(Gm), w).tobytes() == ref.tobytes()
        assert not np.signbit(ref[:50]).any()


@pytest.mark.parametrize("name", A.cases("fedavg_signed__"))
def test_fedavg_signed_zero_matches_reference(name):
    Gm, ref = A.arr(name, "G"), A.arr(name, "output")
    w = np.full(Gm.shape[0], 1.0 / Gm.shape[0], dtype=np.float32)
    assert go.sequential_weighted_sum(list(Gm), w).tobytes() == ref.tobytes()
    assert go.FedAvgOracle({}).aggregate(Gm).tobytes() == ref.tobytes()


@pytest.mark.parametrize("name", A.cases("hier__"))
def test_hierarchical_merge_matches_reference(name):
    """aggregation.py:68-75 / 80-93: cluster means (last cluster absorbs the remainder), then
    FedAvg over the merged rows."""
    Gm, sizes = A.arr(name, "G"), A.meta(name)["cluster_size_list"]
    H = Gm
    for cs in sizes:
        H = go.merge_gradient(H, cs)
    assert H.tobytes() == A.arr(name, "merged").tobytes()
    out = go.FedAvgOracle({}).aggregate(H)
    assert out.tobytes() == A.arr(name, "output").tobytes()


def test_qsgd_oracle_packing_and_scaling():
    """oracle/qsgd_oracle.py (parity unpinned w.r.t. the reference, which raises): the W-bit
    packing round-trips, levels stay in [0, s], and values are +-norm/(s tau) * level."""
    from oracle import qsgd_oracle as qo
    rng = np.random.default_rng(3)
    for n, bits in ((1, 1), (13, 2), (1000, 3), (4099, 8), (777, 14)):
        g = rng.standard_normal(n).astype(np.float32)
        nrm = qo.norm64(g)
        words = qo.encode(g, bits, 9, 2, nrm)
        W = qo.width(bits)
        assert words.shape[0] == (n + 7) // 8 * (8 * W // 32)
        lev, sign = qo.levels_and_signs(g, bits, 9, 2, nrm)
        c = qo.unpack(words, n, bits)
        assert np.array_equal(c, (sign << np.uint32(W - 1)) | lev)
        assert lev.max() <= 2 ** bits
        v = qo.decode(words, n, bits, nrm)
        s = 2.0 ** bits
        np.testing.assert_array_equal(np.abs(v), (nrm / (s * qo.tau(n, s)) * lev).astype(np.float32))
        assert np.array_equal(np.signbit(v) & (lev > 0), np.signbit(g) & (lev > 0))


@pytest.mark.parametrize("bits", [1, 2, 8, 14])
def test_qsgd_oracle_level_never_exceeds_s(bits):
    """an element with |g_i| == ||g|| (a one-hot gradient) sits at level s for
    every dither value U (floor(s + U) = s for U < 1); a level above s must never become 0.
    All 65,536 dither values, at magnitudes whose fp32 product |g| * fl32(s / |g|) lands
    above s as well as below it."""
    from oracle import qsgd_oracle as qo
    s = 2 ** bits
    h = np.arange(65536, dtype=np.uint32)
    for x in (1.0, 3.0, 0.1, 7.3e-5, 1e30, 2.9e-38):
        x32 = np.float32(x)
        lev = qo.levels_from_dither(np.full(65536, x32, np.float32), h, bits, float(x32))
        assert (lev == s).all(), (x, np.unique(lev))
    # below the top: floor(p + U) with the sum exact
    g = np.full(65536, np.float32(0.5), np.float32)
    lev = qo.levels_from_dither(g, h, bits, 1.0)
    want = np.floor(np.float64(np.float32(0.5) * np.float32(s)) + h / 65536.0)
    assert (lev == want).all()
