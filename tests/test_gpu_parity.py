"""GPU parity: the HIP codec (through the C ABI) against the CPU oracle / reference goldens.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
Bars: index sets and top/rand values bit-exact; the dense dropout result compress() returns
byte-exact (float64, -0.0 and NaN bits included); dropout packets (bitmap + kept values) equal
as the reference's consumers see them (assert_array_equal: NaN==NaN, +0==-0) and bit-exact on
every nonzero finite coordinate; FedAVG bit-exact fp32.
"""
import hashlib

import numpy as np
import pytest

from conftest import golden, has_tie_at_boundary
from oracle import compression_oracle as co
from oracle import gar_oracle as go
from oracle import packet_oracle as po
from oracle import philox as ph

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
G = golden()


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from openmsftl_amd import _lib
    lib = _lib.load()
    assert lib.fc_abi_version() == 4


def _codec():
    from openmsftl_amd import codec
    return codec


def _L():
    from openmsftl_amd import _lib
    return _lib


def _gpu_topk(g_np, k, exact=False):
    codec = _codec()
    g = torch.from_numpy(np.ascontiguousarray(g_np, dtype=np.float32)).cuda()
    pkt = codec.encode_top(g, k, exact=exact)
    out = codec.decode(pkt).cpu().numpy()
    return pkt, out


def _check_top_packet(g_np, k, pkt, out):
    keys = po.mag_key(g_np)
    want_idx = po.selected_indices(keys, k)
    want_out = po.decode_dense(g_np.shape[0], want_idx, g_np[want_idx])
    assert out.tobytes() == want_out.tobytes()
    idx, val, h = pkt.raw_entries()
    assert h.status == 0
    assert np.all(np.diff(idx.astype(np.int64)) > 0), "packet indices must ascend"
    assert np.uint64(h.thresh) == po.threshold(keys, k)
    c = po.comps(keys)[idx]
    kept = c >= np.uint64(h.thresh)
    np.testing.assert_array_equal(idx[kept], want_idx)
    assert val.tobytes() == g_np[idx].tobytes()
    assert h.n_entries >= k and kept.sum() == k
    # L64 (header `lower`): every listed entry has comp >= L64 and L64 <= T64; the sample's
    # last workgroup is the header's only writer (a second writer once left it at 0)
    assert np.uint64(h.lower) <= np.uint64(h.thresh)
    assert len(c) == 0 or c.min() >= np.uint64(h.lower)
    if k and h.n_entries > k:                      # slack listed: the bracket's lower end is set
        assert h.lower > 0 or po.comps(keys).min() == 0


# ---- top: golden cases ----------------------------------------------------------------
@pytest.mark.parametrize("name", G.cases("top__"))
def test_top_golden(name):
    from openmsftl_amd import Compression
    m = G.meta(name)
    g = G.input(name)
    C = Compression({"compression_function": "top", "fraction_coordinate": m["fraction"]})
    out = C.compress(g.copy())
    ora = co.compress({"compression_function": "top", "fraction_coordinate": m["fraction"]}, g)
    assert out.dtype == np.float32
    assert out.tobytes() == ora.tobytes()
    k = co.effective_k(co.num_kept(m["fraction"], g.shape[0]), g.shape[0])
    if not has_tie_at_boundary(g, k):
        assert out.tobytes() == G.arr(name, "output").tobytes()   # the reference itself


# ---- top: sizes, fractions, fast vs exact ----------------------------------------------
SIZES = [1, 5, 4095, 4096, 8191, 8192, 8193, 100_003, 1 << 20, (1 << 20) + 17, 3_000_001]
FRACS = [0.1, 0.01, 0.5, 0.9, 1e-6, 0.999]


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("f", FRACS)
def test_top_sizes(n, f):
    g = np.random.default_rng(n * 7 + int(f * 1000)).standard_normal(n, dtype=np.float32)
    g *= np.float32(10.0) ** np.random.default_rng(n).uniform(-4, 1, n).astype(np.float32)
    k = co.effective_k(co.num_kept(f, n), n)
    pkt, out = _gpu_topk(g, k)
    _check_top_packet(g, k, pkt, out)


@pytest.mark.parametrize("n,f", [(100_003, 0.1), (3_000_001, 0.01), (1 << 20, 0.37)])
def test_top_exact_path_equals_fast(n, f):
    g = np.random.default_rng(5).standard_normal(n, dtype=np.float32)
    k = co.effective_k(co.num_kept(f, n), n)
    p1, o1 = _gpu_topk(g, k)
    p2, o2 = _gpu_topk(g, k, exact=True)
    assert o1.tobytes() == o2.tobytes()
    idx2, _, h2 = p2.raw_entries()
    assert h2.n_entries == k
    _check_top_packet(g, k, p2, o2)


ADVERSARIAL = {
    "constant": lambda n: np.full(n, 0.5, np.float32),
    "zeros_signed": lambda n: np.where(np.arange(n) % 3 == 0, -0.0, 0.0).astype(np.float32),
    "ascending": lambda n: np.arange(n, dtype=np.float32),
    "smallint_ties": lambda n: np.random.default_rng(1).integers(-4, 5, n).astype(np.float32),
    "nan_inf_mix": lambda n: np.where(np.random.default_rng(2).random(n) < 0.05, np.nan,
                                      np.where(np.random.default_rng(3).random(n) < 0.05,
                                               -np.inf, np.random.default_rng(4).standard_normal(n))
                                      ).astype(np.float32),
    "denormals": lambda n: (np.random.default_rng(6).standard_normal(n) * 1e-41).astype(np.float32),
    "layered_scales": lambda n: (np.random.default_rng(8).standard_normal(n)
                                 * np.repeat(10.0 ** np.arange(-6, 2), -(-n // 8))[:n]).astype(np.float32),
}


@pytest.mark.parametrize("kind", sorted(ADVERSARIAL))
@pytest.mark.parametrize("n", [70_001, 2_500_000])
@pytest.mark.parametrize("f", [0.1, 0.5])
def test_top_adversarial(kind, n, f):
    g = ADVERSARIAL[kind](n)
    k = co.effective_k(co.num_kept(f, n), n)
    pkt, out = _gpu_topk(g, k)
    _check_top_packet(g, k, pkt, out)


def test_top_bracket_miss_falls_back_to_exact():
    """Large values hidden between the sampled segments -> bracket misses -> exact path."""
    n = 4 << 20
    g = np.zeros(n, np.float32)
    nseg = max(64, min(1024, n // 64 // 1024))     # make_plan (fc_capi.hip)
    starts = ((np.arange(nseg, dtype=np.int64) * (n - 1024)) // (nseg - 1)) & ~3
    sampled = np.zeros(n, bool)
    for s in starts:
        sampled[s:s + 1024] = True
    hidden = np.nonzero(~sampled)[0]
    g[hidden[: n // 8]] = np.random.default_rng(0).standard_normal(n // 8).astype(np.float32)
    k = n // 10
    codec = _codec()
    gt = torch.from_numpy(g).cuda()
    pkt = codec.encode_top(gt, k, check=False)
    torch.cuda.synchronize()
    redo = codec.resolve([pkt])
    assert redo == 1
    out = codec.decode(pkt).cpu().numpy()
    _check_top_packet(g, k, pkt, out)


def _wave_overflow_gradient(n=4 << 20, f=0.1, seed=5):
    """A gradient whose chunk 7 holds ~100 candidates (|g| within 1e-5 of the k-th
    magnitude) in wave 3's elements alone -- past that wave's 32-entry candidate sub-slot
    while the chunk stays under its 256-entry candidate slot -- and chunk 9 holds 40 spread
    over two waves (no overflow)."""
    rng = np.random.default_rng(seed)
    g = rng.standard_normal(n, dtype=np.float32)
    k = co.effective_k(co.num_kept(f, n), n)
    T = np.partition(np.abs(g), n - k)[n - k]
    def near(m):
        v = T * (1.0 + rng.uniform(-1e-5, 1e-5, m))
        return (v * rng.choice([-1.0, 1.0], m)).astype(np.float32)
    lay = lambda base, w: (base + np.arange(4)[:, None, None] * 2048 + w * 256
                           + np.arange(4)[None, :, None] * 64 + np.arange(64)[None, None, :]).ravel()
    pos = rng.choice(lay(7 * 8192, 3), 100, replace=False)
    g[pos] = near(100)
    pos = np.concatenate([rng.choice(lay(9 * 8192, 1), 20, replace=False),
                          rng.choice(lay(9 * 8192, 6), 20, replace=False)])
    g[pos] = near(40)
    return g, k


@pytest.mark.parametrize("path", ["single", "batch", "dense"])
def test_top_wave_candidate_overflow(path):
    """Per-wave candidate sub-slots (k_compact_mag1 / k_fused_mag): a wave with more than 32
    candidates marks its chunk overflowed and the resolve re-reads the chunk's entries; the
    result is still the oracle's, on the fused single-client path (compaction-side bins), the
    batched path (resolve-side bins) and the dense path."""
    g, k = _wave_overflow_gradient()
    codec = _codec()
    if path == "single":
        pkt, out = _gpu_topk(g, k)
        _check_top_packet(g, k, pkt, out)
    elif path == "batch":
        g2 = _wave_overflow_gradient(seed=6)[0]
        grads = [torch.from_numpy(x).cuda() for x in (g, g2)]
        pk = codec.encode_top_batch(grads, k)
        for x, p in zip((g, g2), pk):
            _check_top_packet(x, k, p, codec.decode(p).cpu().numpy())
    else:
        pkt, q = _dense_top(g, k)
        _check_dense(g, k, pkt, q)


# ---- top straight to the dense q (fc_topk_encode_dense: compaction streams q + fix-up) ----
def _dense_top(g_np, k):
    codec = _codec()
    gt = torch.from_numpy(g_np).cuda()
    pkt = codec.Packet.alloc(g_np.shape[0], _L().FC_FMT_IDXVAL, gt.device, k=k)
    q = codec.compress_top_dense(gt, k, packet=pkt).cpu().numpy()
    return pkt, q


def _check_dense(g_np, k, pkt, q):
    """The dense path's product is q (its packet is scratch, FC_FMT_DENSE): q equals the
    oracle's and the header's T64 is the oracle's threshold; the scratch packet refuses to
    decode.  A bracket miss re-encoded the packet exactly (then it is a full packet)."""
    keys = po.mag_key(g_np)
    want_idx = po.selected_indices(keys, k)
    assert q.tobytes() == po.decode_dense(g_np.shape[0], want_idx, g_np[want_idx]).tobytes()
    h = pkt.header()
    assert h.status == 0
    assert np.uint64(h.thresh) == po.threshold(keys, k)
    if h.format == _L().FC_FMT_DENSE:
        with pytest.raises(ValueError):
            _codec().decode(pkt)
    else:
        _check_top_packet(g_np, k, pkt, q)


@pytest.mark.parametrize("n", [5, 8192, 8193, 100_003, (1 << 20) + 17, 3_000_001])
@pytest.mark.parametrize("f", [0.1, 0.01, 0.5, 0.999])
def test_top_dense_sizes(n, f):
    g = np.random.default_rng(n * 3 + int(f * 1000)).standard_normal(n, dtype=np.float32)
    g *= np.float32(10.0) ** np.random.default_rng(n + 1).uniform(-4, 1, n).astype(np.float32)
    k = co.effective_k(co.num_kept(f, n), n)
    pkt, q = _dense_top(g, k)
    _check_dense(g, k, pkt, q)


@pytest.mark.parametrize("kind", sorted(ADVERSARIAL))
def test_top_dense_adversarial(kind):
    n, f = 2_500_000, 0.1
    g = ADVERSARIAL[kind](n)
    k = co.effective_k(co.num_kept(f, n), n)
    pkt, q = _dense_top(g, k)
    _check_dense(g, k, pkt, q)


def test_top_dense_golden_and_bracket_miss():
    """Reference goldens through the dense path, and a bracket miss (exact re-encode +
    decode into the same output)."""
    for name in G.cases("top__"):
        m = G.meta(name)
        g = G.input(name)
        n = g.shape[0]
        k = co.effective_k(co.num_kept(m["fraction"], n), n)
        _, q = _dense_top(g.astype(np.float32), k)
        ora = co.compress({"compression_function": "top", "fraction_coordinate": m["fraction"]}, g)
        assert q.tobytes() == ora.astype(np.float32).tobytes(), name
    n = 4 << 20
    g = np.zeros(n, np.float32)
    nseg = max(64, min(1024, n // 64 // 1024))     # make_plan (fc_capi.hip)
    starts = ((np.arange(nseg, dtype=np.int64) * (n - 1024)) // (nseg - 1)) & ~3
    sampled = np.zeros(n, bool)
    for s in starts:
        sampled[s:s + 1024] = True
    hidden = np.nonzero(~sampled)[0]
    g[hidden[: n // 8]] = np.random.default_rng(0).standard_normal(n // 8).astype(np.float32)
    k = n // 10
    pkt, q = _dense_top(g, k)
    _check_dense(g, k, pkt, q)


def test_top_dense_128M_equals_packet_decode():
    """Size-independent check at the headline size: dense path == decode(encode_top)."""
    codec = _codec()
    n = 134_217_728
    gt = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
    k = co.effective_k(co.num_kept(0.1, n), n)
    q = codec.compress_top_dense(gt, k)
    ref = codec.decode(codec.encode_top(gt, k))
    assert torch.equal(q.view(torch.int32), ref.view(torch.int32))
    assert int((q != 0).sum()) == k


@pytest.mark.parametrize("key", sorted(G.manifest["large"]))
def test_top_large_digests(key):
    d = G.manifest["large"][key]
    g = np.random.default_rng(d["seed"]).standard_normal(d["n"], dtype=np.float32)
    pkt, out = _gpu_topk(g, d["k"])
    assert hashlib.sha256(out.tobytes()).hexdigest() == d["output_sha256"]
    idx, val, h = pkt.raw_entries()
    kept = po.comps(po.mag_key(g))[idx] >= np.uint64(h.thresh)
    assert hashlib.sha256(idx[kept].tobytes()).hexdigest() == d["sorted_idx_sha256"]


def test_top_128M_properties():
    """BASELINE size: 134,217,728 fp32, f = 0.1 — size-independent properties."""
    n, f = 134_217_728, 0.1
    k = co.num_kept(f, n)
    codec = _codec()
    gen = torch.Generator(device="cuda").manual_seed(1234)
    g = torch.randn(n, device="cuda", generator=gen)
    pkt = codec.encode_top(g, k)
    out = codec.decode(pkt)
    h = pkt.header()
    assert h.status == 0 and h.n_entries >= k
    nz = out != 0
    assert int(nz.sum()) == k
    assert torch.equal(out[nz], g[nz])                       # exact copies
    a = g.abs()
    assert float(a[nz].min()) >= float(a[~nz].max())         # every kept >= every dropped
    pos = torch.arange(pkt.capacity, device="cuda")
    listed = (pos % 8192) < pkt.cnt.to(torch.int64)[pos // 8192]
    # chunk-local uint16 indices (int16 storage) + the slot's chunk base = element index
    idx = (pkt.idx[listed].to(torch.int64) & 0xffff) + (pos[listed] // 8192) * 8192
    assert idx.numel() == h.n_entries
    assert bool((idx[1:] > idx[:-1]).all())                  # ascending packet (slot order)
    # slack stays small (the packet carries few unselected entries)
    assert h.n_entries - k < 0.06 * k


# ---- batched encode (fc_topk_encode_batch) ----------------------------------------------
def _packet_bytes(p):
    idx, val, h = p.raw_entries()
    return idx.tobytes(), val.tobytes(), int(h.thresh), int(h.n_entries), int(h.status)


@pytest.mark.parametrize("n,f,M", [(100_003, 0.1, 5), (3_000_001, 0.01, 3), (1 << 20, 0.37, 4),
                                   (8193, 0.5, 7), (2, 0.5, 2)])
def test_batch_encode_equals_single(n, f, M):
    codec = _codec()
    rng = np.random.default_rng(n + M)
    host = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 1)).astype(np.float32)
            for _ in range(M)]
    grads = [torch.from_numpy(x).cuda() for x in host]
    k = co.effective_k(co.num_kept(f, n), n)
    batch = codec.encode_top_batch(grads, k)
    for x, g, pb in zip(host, grads, batch):
        ps = codec.encode_top(g, k)
        assert _packet_bytes(pb) == _packet_bytes(ps)
        _check_top_packet(x, k, pb, codec.decode(pb).cpu().numpy())


@pytest.mark.parametrize("streams", [1, 2])
def test_batch_encode_in_two_parts(streams):
    """fc_topk_encode_batch_part: the sample part, then (after unrelated work on the caller's
    stream) the finish part, gives the packets of one fc_topk_encode_batch call."""
    from openmsftl_amd import _lib as L
    codec = _codec()
    n, M = 300_001, 5
    rng = np.random.default_rng(77)
    grads = [torch.from_numpy((rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 1))
                              .astype(np.float32)).cuda() for _ in range(M)]
    k = co.num_kept(0.1, n)
    want = [_packet_bytes(p) for p in codec.encode_top_batch(grads, k, streams=streams)]
    pk = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, grads[0].device, k=k) for _ in range(M)]
    codec.encode_top_batch(grads, k, packets=pk, check=False, streams=streams,
                           part=L.FC_PART_SAMPLE, fork=False, join=False)
    torch.ones(1 << 20, device="cuda").sum()                   # caller-stream work in between
    codec.encode_top_batch(grads, k, packets=pk, check=False, streams=streams,
                           part=L.FC_PART_FINISH)
    torch.cuda.synchronize()
    assert [_packet_bytes(p) for p in pk] == want
    with pytest.raises(ValueError):
        codec.encode_top_batch(grads, k, packets=pk, part=L.FC_PART_SAMPLE)   # check=True


def test_batch_encode_parts_more_groups_than_streams():
    """Three sub-batches on two streams (group 2 shares stream 0 with group 0): every
    sub-batch keeps its own encoder state between its SAMPLE and FINISH parts, so no packet
    comes back RETRY and all equal the one-call encode."""
    from openmsftl_amd import _lib as L
    codec = _codec()
    n, M = 200_003, 7
    rng = np.random.default_rng(78)
    grads = [torch.from_numpy((rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 1))
                              .astype(np.float32)).cuda() for _ in range(M)]
    k = co.num_kept(0.1, n)
    want = [_packet_bytes(p) for p in codec.encode_top_batch(grads, k, streams=1)]
    pk = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, grads[0].device, k=k) for _ in range(M)]
    for part in (L.FC_PART_SAMPLE, L.FC_PART_FINISH):
        codec.encode_top_batch(grads, k, packets=pk, check=False, streams=2, groups=[3, 2, 2],
                               part=part)
    torch.cuda.synchronize()
    assert [int(h.status) for h in codec.headers(pk)] == [0] * M
    assert [_packet_bytes(p) for p in pk] == want


def test_batch_encode_above_resolve_chunk_list():
    """n = 2^28 + 8193 (32,769 chunks): 16 resolve workgroups per client would each own more
    chunks than the k_resolve LDS size list holds (the call came back RETRY for every client
    and went down the exact path); the launch adds workgroups instead.  Straight out of the
    batch launch every status is OK and the packets equal the lone encodes'."""
    codec = _codec()
    n, M = (1 << 28) + 8193, 2
    grads = [torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(s))
             .mul_(10.0 ** -s) for s in range(M)]
    k = co.num_kept(0.1, n)
    from openmsftl_amd import _lib as L
    pk = codec.encode_top_batch(grads, k, check=False, streams=2)   # (> 2^27 and
    torch.cuda.synchronize()                                         # two streams: no timeouts)
    assert [int(h.status) for h in codec.headers(pk)] == [0] * M
    pk = codec.encode_top_batch(grads, k, packets=pk, check=False)
    torch.cuda.synchronize()
    assert [int(h.status) for h in codec.headers(pk)] == [0] * M
    for g, pb in zip(grads, pk):
        ps = codec.encode_top(g, k, check=False)
        hb, hs = codec.headers([pb, ps])
        assert int(hs.status) == 0
        assert (hb.thresh, hb.lower, hb.n_entries) == (hs.thresh, hs.lower, hs.n_entries)
        assert torch.equal(pb.cnt, ps.cnt) and torch.equal(pb.qoff, ps.qoff)
        pos = torch.arange(pb.capacity, device="cuda")       # the listed slot entries, on the GPU
        listed = (pos % L.FC_CHUNK) < pb.cnt.long()[pos // L.FC_CHUNK]
        del pos
        assert int(listed.sum()) == int(hb.n_entries)
        assert torch.equal(pb.idx[listed], ps.idx[listed])
        assert torch.equal(pb.val.view(torch.int32)[listed], ps.val.view(torch.int32)[listed])
        del ps, listed
    del pk, grads
    torch.cuda.empty_cache()


@pytest.mark.parametrize("M,n", [(65, 20_000), (70, 8_193 * 3), (130, 9_000)])
def test_batch_encode_client_interleave(M, n):
    """k_compact_mag1 interleaves the chunks of 64 clients in dispatch order: a full group, a
    partial last group (M % 64 clients) and > 2 groups give the per-client packets."""
    codec = _codec()
    rng = np.random.default_rng(M * 7 + n)
    host = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 1)).astype(np.float32)
            for _ in range(M)]
    grads = [torch.from_numpy(x).cuda() for x in host]
    k = co.effective_k(co.num_kept(0.1, n), n)
    batch = codec.encode_top_batch(grads, k, streams=1)
    torch.cuda.synchronize()
    for i in range(0, M, 7):
        ps = codec.encode_top(grads[i], k)
        assert _packet_bytes(batch[i]) == _packet_bytes(ps)
        _check_top_packet(host[i], k, batch[i], codec.decode(batch[i]).cpu().numpy())


@pytest.mark.parametrize("streams,groups", [(1, None), (2, None), (3, None), (2, [1, 3, 1]),
                                            (2, [4, 1])])
def test_batch_encode_forked_streams(streams, groups):
    """Sub-batches on forked streams (encode_top_batch(streams=...)) give the same packets as
    one launch chain and as per-client encodes; odd M splits unevenly."""
    codec = _codec()
    n, M, f = 1 << 20, 5, 0.1
    rng = np.random.default_rng(77)
    host = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 1)).astype(np.float32)
            for _ in range(M)]
    grads = [torch.from_numpy(x).cuda() for x in host]
    k = co.effective_k(co.num_kept(f, n), n)
    batch = codec.encode_top_batch(grads, k, streams=streams, groups=groups)
    torch.cuda.synchronize()
    for x, g, pb in zip(host, grads, batch):
        ps = codec.encode_top(g, k)
        assert _packet_bytes(pb) == _packet_bytes(ps)
        _check_top_packet(x, k, pb, codec.decode(pb).cpu().numpy())


@pytest.mark.timeout(120)
def test_batch_encodes_on_concurrent_streams_stay_ok():
    """Two batched encodes running concurrently on one device (the sub-batches of
    encode_top_batch(streams=2) on two forked streams, nothing orders them): no batched kernel
    waits in-kernel, so no status ever leaves OK.  Round 4's k_resolve waited for the bin and
    stalled here to the spin bound in 23 of 1,500 steps unless the encodes were serialized
    (tools/stall_probe.py); this loop of 600 steps, queued back to back with a FedAVG fold
    between them, counts the statuses on the device after each step (no host sync)."""
    assert not hasattr(_codec(), "_ordered_encode")          # no serialization to lean on
    codec = _codec()
    from openmsftl_amd import _lib as L
    n, M, f = 1 << 22, 128, 0.1
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device="cuda").manual_seed(9)
    grads = [torch.randn(n, device="cuda", generator=gen) * (10.0 ** (-4 + 3 * (i % 7) / 6))
             for i in range(M)]
    k = co.effective_k(co.num_kept(f, n), n)
    hdrs = torch.zeros((M, L.HDR_BYTES), dtype=torch.uint8, device=dev)
    pk = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, hdr=hdrs[j], k=k) for j in range(M)]
    codec.encode_top_batch(grads, k, packets=pk)
    jobs = codec.encode_jobs(grads, pk)
    w = [1.0 / M] * M
    views = codec.views_tensor(pk, w, dev)
    acc = torch.empty(n, dtype=torch.float32, device=dev)
    bad = torch.zeros((), dtype=torch.int64, device=dev)
    status = hdrs[:, 36:40]
    for _ in range(600):
        codec.encode_top_batch(grads, k, packets=pk, jobs=jobs, check=False, streams=2)
        bad += (status != 0).any(dim=1).sum()
        codec.decode_accumulate(pk, w, out=acc, views=views)
    torch.cuda.synchronize()
    assert int(bad) == 0, f"{int(bad)} client statuses not OK (stalled k_resolve -> RETRY)"
    assert codec.resolve(pk) == 0


@pytest.mark.timeout(120)
def test_fused_encodes_on_concurrent_streams_never_stall():
    """k_fused_mag (the lone packet and drop-in dense encodes, and fc_topk_encode_decode's
    encode) is a kernel whose workgroups wait in-kernel, for the bracket of their own launch.
    The library orders such launches per device itself (include/fedcodec.h, Concurrency) —
    nothing in Python does any more — so a packet encode, a dense one and an encode + decode
    (their own workspaces) issued on three streams 200 times each, with nothing else ordering
    them, never stall to the poll bound: every status is OK (counted on each stream, no host
    sync) and every result equals the single-stream calls'."""
    codec = _codec()
    assert not hasattr(codec, "_fused_encode")
    n, f = 1 << 24, 0.1
    gen = torch.Generator(device="cuda").manual_seed(17)
    g0 = torch.randn(n, device="cuda", generator=gen) * 1e-3
    g1 = torch.randn(n, device="cuda", generator=gen) * 3e-2
    k = co.effective_k(co.num_kept(f, n), n)
    g2 = torch.randn(n, device="cuda", generator=gen)
    ref0 = _packet_bytes(codec.encode_top(g0, k))
    ref1 = codec.decode(codec.encode_top(g1, k)).clone()
    ref2p = codec.encode_top(g2, k)
    ref2 = (_packet_bytes(ref2p), codec.decode(ref2p).clone())
    s0, s1, s2 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s0):
        p0 = codec.encode_top(g0, k, check=False)
    with torch.cuda.stream(s1):
        p1 = codec.Packet.alloc(n, codec.L.FC_FMT_IDXVAL, g1.device, k=k)
        out1 = torch.empty_like(g1)
    with torch.cuda.stream(s2):                 # fc_topk_encode_decode: its decode waits too
        p2, out2 = codec.encode_decode_top(g2, k, check=False)
    torch.cuda.synchronize()
    bad = [torch.zeros((), dtype=torch.int64, device="cuda") for _ in range(3)]
    torch.cuda.synchronize()
    for _ in range(200):                        # statuses counted on each stream, no host sync
        with torch.cuda.stream(s0):
            codec.encode_top(g0, k, packet=p0, check=False)
            bad[0] += (p0.hdr[36:40] != 0).any().to(torch.int64)
        with torch.cuda.stream(s1):
            codec.compress_top_dense(g1, k, out=out1, packet=p1, check=False)
            bad[1] += (p1.hdr[36:40] != 0).any().to(torch.int64)
        with torch.cuda.stream(s2):
            codec.encode_decode_top(g2, k, packet=p2, out=out2, check=False)
            bad[2] += (p2.hdr[36:40] != 0).any().to(torch.int64)
    torch.cuda.synchronize()
    assert [int(b) for b in bad] == [0, 0, 0]
    assert _packet_bytes(p0) == ref0
    assert torch.equal(out1.view(torch.int32), ref1.view(torch.int32))
    assert _packet_bytes(p2) == ref2[0]
    assert torch.equal(out2.view(torch.int32), ref2[1].view(torch.int32))


@pytest.mark.timeout(120)
def test_fused_f64_encodes_on_concurrent_streams_never_stall():
    """k_fused64 (fc_topk_dense_f64_sampled) polls in-kernel like k_fused_mag; the
    library orders it with the fp32 fused encodes.  Two float64 sampled encodes and a float32
    dense one on three streams, 100 rounds: no RETRY, results equal the ordered ones."""
    codec = _codec()
    n, f = 1 << 22, 0.1
    gen = torch.Generator(device="cuda").manual_seed(23)
    a = torch.randn(n, device="cuda", generator=gen, dtype=torch.float64) * 1e-2
    b = torch.randn(n, device="cuda", generator=gen, dtype=torch.float64) * 5.0
    c = torch.randn(n, device="cuda", generator=gen) * 1e-3
    k = co.num_kept(f, n)
    ra, rb = codec.compress_top_dense_f64(a, k).clone(), codec.compress_top_dense_f64(b, k).clone()
    rc = codec.compress_top_dense(c, k).clone()
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = []
    torch.cuda.synchronize()
    for s, x in zip(streams, (a, b)):
        with torch.cuda.stream(s):
            outs.append(torch.empty_like(x))
    with torch.cuda.stream(streams[2]):
        oc = torch.empty_like(c)
        pc = codec.Packet.alloc(n, codec.L.FC_FMT_IDXVAL, c.device, k=k)
    torch.cuda.synchronize()
    bads = []
    for s in streams:
        with torch.cuda.stream(s):
            bads.append(torch.zeros((), dtype=torch.int64, device="cuda"))
    torch.cuda.synchronize()
    for _ in range(100):
        for i, x in enumerate((a, b)):
            with torch.cuda.stream(streams[i]):
                codec.compress_top_dense_f64(x, k, out=outs[i], check=False)
                bads[i] += (codec._f64_status(outs[i]) != 0).any().to(torch.int64)
        with torch.cuda.stream(streams[2]):
            codec.compress_top_dense(c, k, out=oc, packet=pc, check=False)
            bads[2] += (pc.hdr[36:40] != 0).any().to(torch.int64)
    torch.cuda.synchronize()
    assert [int(x) for x in bads] == [0, 0, 0]
    assert torch.equal(outs[0], ra) and torch.equal(outs[1], rb)
    assert torch.equal(oc.view(torch.int32), rc.view(torch.int32))


def test_fused_encodes_ordered_across_streams():
    """The library's ordering of fused encodes: a fused encode on another stream than the
    device's previous one waits for the event recorded after that one.  Alternating a packet encode and a dense one over two
    streams 200 times, with other work queued behind each, never stalls (every status OK) and
    both results equal the single-stream encodes'."""
    codec = _codec()
    n, f = 1 << 24, 0.1
    gen = torch.Generator(device="cuda").manual_seed(18)
    g0 = torch.randn(n, device="cuda", generator=gen) * 1e-3
    g1 = torch.randn(n, device="cuda", generator=gen) * 3e-2
    k = co.effective_k(co.num_kept(f, n), n)
    ref0 = _packet_bytes(codec.encode_top(g0, k))
    ref1 = codec.decode(codec.encode_top(g1, k)).clone()
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s0):
        p0 = codec.encode_top(g0, k, check=False)
        bad0 = torch.zeros((), dtype=torch.int64, device="cuda")
        junk0 = torch.empty_like(g0)
    with torch.cuda.stream(s1):
        p1 = codec.Packet.alloc(n, codec.L.FC_FMT_IDXVAL, g1.device, k=k)
        out1 = torch.empty_like(g1)
        bad1 = torch.zeros((), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for i in range(200):
        with torch.cuda.stream(s0):
            codec.encode_top(g0, k, packet=p0, check=False)
            bad0 += (p0.hdr[36:40] != 0).any().to(torch.int64)
            if i % 3 == 0:
                codec.decode(p0, out=junk0)          # work queued behind the encode
        with torch.cuda.stream(s1):
            codec.compress_top_dense(g1, k, out=out1, packet=p1, check=False)
            bad1 += (p1.hdr[36:40] != 0).any().to(torch.int64)
    torch.cuda.synchronize()
    assert int(bad0) == 0 and int(bad1) == 0
    assert _packet_bytes(p0) == ref0
    assert torch.equal(out1.view(torch.int32), ref1.view(torch.int32))


@pytest.mark.parametrize("M,streams", [(5, 2), (7, 3), (2, 2), (1, 2)])
def test_encode_fold_batch_pipelined(M, streams):
    """encode_fold_batch (each sub-batch folded on its stream as soon as it is encoded, the
    folds chained in row order) gives the packets of encode_top_batch and, bit for bit, the
    FedAVG of gar.py:44 on the G those packets decode to (oracle)."""
    codec = _codec()
    n, f = 300_001, 0.1
    rng = np.random.default_rng(91 + M)
    host = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 1)).astype(np.float32)
            for _ in range(M)]
    grads = [torch.from_numpy(x).cuda() for x in host]
    k = co.effective_k(co.num_kept(f, n), n)
    w = np.full(M, 1.0 / M, dtype=np.float32)            # gar.py:37-40's default weights
    pk = [codec.Packet.alloc(n, codec.L.FC_FMT_IDXVAL, grads[0].device, k=k) for _ in range(M)]
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    for _ in range(2):                                   # reused buffers, second pass too
        codec.encode_fold_batch(grads, k, w, out, packets=pk, streams=streams)
        assert codec.resolve(pk) == 0
        torch.cuda.synchronize()
    ref = codec.encode_top_batch(grads, k)
    for a, b in zip(pk, ref):
        assert _packet_bytes(a) == _packet_bytes(b)
    G = go.build_dense_G([co.compress({"compression_function": "top", "fraction_coordinate": f}, x)
                          for x in host], np.float32)
    want = go.FedAvgOracle({}).aggregate(G)
    assert out.cpu().numpy().tobytes() == want.tobytes()


def test_batch_encode_philox_and_fallback():
    """Native rand-k keys per client (seed/offset per job) and one client whose sampled
    bracket misses (resolved by the per-packet exact path) inside the same batch."""
    codec = _codec()
    L = _L()
    n = 4 << 20
    k = n // 10
    seeds, offs = [11, 12, 13], [1, 2, 3]
    host = [np.random.default_rng(i).standard_normal(n, dtype=np.float32) for i in range(3)]
    grads = [torch.from_numpy(x).cuda() for x in host]
    pk = codec.encode_top_batch(grads, k, key_mode=L.FC_KEY_PHILOX, seeds=seeds, offsets=offs)
    for x, p, s, o in zip(host, pk, seeds, offs):
        keys = (ph.element_words(n, s, o) >> np.uint32(1)).astype(np.uint32)
        want = po.selected_indices(keys, k)
        assert codec.decode(p).cpu().numpy().tobytes() == po.decode_dense(n, want, x[want]).tobytes()
    # hidden large values between sampled segments (as test_top_bracket_miss_falls_back_...)
    nseg = max(64, min(1024, n // 64 // 1024))     # make_plan (fc_capi.hip)
    starts = ((np.arange(nseg, dtype=np.int64) * (n - 1024)) // (nseg - 1)) & ~3
    sampled = np.zeros(n, bool)
    for s in starts:
        sampled[s:s + 1024] = True
    bad = np.zeros(n, np.float32)
    hidden = np.nonzero(~sampled)[0]
    bad[hidden[: n // 8]] = np.random.default_rng(0).standard_normal(n // 8).astype(np.float32)
    host2 = [host[0], bad, host[2]]
    grads2 = [torch.from_numpy(x).cuda() for x in host2]
    pk2 = codec.encode_top_batch(grads2, k, check=False)
    torch.cuda.synchronize()
    assert codec.resolve(pk2) == 1
    for x, p in zip(host2, pk2):
        _check_top_packet(x, k, p, codec.decode(p).cpu().numpy())


def test_batch_encode_arguments():
    codec = _codec()
    L = _L()
    lib = L.load()
    g = torch.zeros(1000, device="cuda")
    with pytest.raises(ValueError):
        codec.encode_top_batch([g, torch.zeros(999, device="cuda")], 10)
    rc = lib.fc_topk_encode_batch(None, 1, 1000, 10, 0, 8192, None, 0, None)
    assert rc == -1 and b"jobs" in lib.fc_last_error()


# ---- rand ------------------------------------------------------------------------------
@pytest.mark.parametrize("name", G.cases("rand__"))
def test_rand_numpy_rng_golden(name):
    from openmsftl_amd import Compression
    m = G.meta(name)
    g = G.input(name)
    np.random.seed(m["seed"])
    out = Compression({"compression_function": "rand",
                       "fraction_coordinate": m["fraction"]}).compress(g)
    assert int(np.random.randint(0, 2**31 - 1)) == m["rng_next"]
    assert out.dtype == np.float32
    assert out.tobytes() == G.arr(name, "output").tobytes()


@pytest.mark.parametrize("n,f", [(1000, 0.1), (100_003, 0.5), (3_000_001, 0.01), (24_581, 0.5),
                                 (65_536, 0.9), (16_777_216, 0.1)])
def test_rand_philox_matches_oracle(n, f):
    """Native rand-k (fc_topk_encode with Philox keys): the lone encode bins its candidates in
    the compaction (round 6) — its packet, header included, equals the batched encode's (whose
    k_resolve<true> bins them) byte for byte, with no RETRY, and decodes to the oracle's choice.
    24,581 at f = 0.5 overflows every full chunk's 256-entry candidate slot (~16 sigma = ~1,250
    candidates over 4 chunks): the resolve re-reads those chunks' entries and recomputes keys."""
    codec = _codec()
    L = _L()
    g = np.random.default_rng(n).standard_normal(n, dtype=np.float32)
    k = co.num_kept(f, n)
    seed, off = 0xDEADBEEF12345, 7
    gd = torch.from_numpy(g).cuda()
    pkt = codec.encode_top(gd, k, key_mode=L.FC_KEY_PHILOX, seed=seed, offset=off)
    assert pkt.header().status == 0
    out = codec.decode(pkt).cpu().numpy()
    keys = (ph.element_words(n, seed, off) >> np.uint32(1)).astype(np.uint32)
    want = po.selected_indices(keys, k)
    assert out.tobytes() == po.decode_dense(n, want, g[want]).tobytes()
    if 0 < k < n:
        (bp,) = codec.encode_top_batch([gd], k, key_mode=L.FC_KEY_PHILOX, seeds=[seed], offsets=[off])
        assert _packet_bytes(bp) == _packet_bytes(pkt)
        assert bp.hdr.cpu().numpy().tobytes() == pkt.hdr.cpu().numpy().tobytes()


# ---- dropout ---------------------------------------------------------------------------
def _dropout_equal(out, ref):
    assert out.dtype == np.float64 == ref.dtype
    np.testing.assert_array_equal(out, ref)                 # NaN==NaN, +0==-0
    fin = np.isfinite(ref) & (ref != 0)
    assert out[fin].tobytes() == ref[fin].tobytes()


@pytest.mark.parametrize("name", G.cases("dropout-"))
def test_dropout_numpy_rng_golden(name):
    from openmsftl_amd import Compression
    m = G.meta(name)
    g = G.input(name)
    np.random.seed(m["seed"])
    out = Compression({"compression_function": m["codec"], "dropout_p": m["p"]}).compress(g)
    if "rng_next" in m:
        assert int(np.random.randint(0, 2**31 - 1)) == m["rng_next"]
    ref = G.arr(name, "output")
    _dropout_equal(out, ref)
    assert out.tobytes() == ref.tobytes()                     # -0.0 and NaN bits too


@pytest.mark.parametrize("codec_name", ["dropout-biased", "dropout-unbiased"])
@pytest.mark.parametrize("p", [0.1, 0.3, 0.0])
def test_dropout_dense_f32_byte_exact(codec_name, p):
    """compress()'s dense fp32 dropout path (fc_mask_dense_f32): g * mask (/ p) in float64,
    byte for byte as NumPy computes it (compression.py:52, :59) with -0.0 for dropped
    negative g and NaN for dropped +-inf, on both mask sources."""
    codec = _codec()
    L = _L()
    n = 1_000_003
    g = np.random.default_rng(12).standard_normal(n, dtype=np.float32)
    g[::9973] = np.inf
    g[5::9973] = -np.inf
    g[7::10007] = np.float32(-0.0)
    cid = L.FC_CODEC_DROPOUT_BIASED if codec_name == "dropout-biased" else L.FC_CODEC_DROPOUT_UNBIASED
    gd = torch.from_numpy(g).cuda()
    out = codec.mask_dense_f64(gd, cid, p=p, seed=9, offset=4).cpu().numpy()
    mask = ph.bernoulli_mask(n, p, 9, 4).astype(np.int64)
    with np.errstate(invalid="ignore", divide="ignore"):
        ref = g * mask if codec_name == "dropout-biased" else (g * mask) / p
    assert out.tobytes() == ref.tobytes()
    from openmsftl_amd.compression import bitmask_words
    hm = np.random.default_rng(3).binomial(1, 0.5, n)
    mb = torch.from_numpy(bitmask_words(hm, n, True).view(np.int32)).cuda()
    out = codec.mask_dense_f64(gd, cid, p=p, mask_bits=mb).cpu().numpy()
    with np.errstate(invalid="ignore", divide="ignore"):
        ref = g * hm if codec_name == "dropout-biased" else (g * hm) / p
    assert out.tobytes() == ref.tobytes()


@pytest.mark.parametrize("codec_name", ["dropout-biased", "dropout-unbiased"])
@pytest.mark.parametrize("p", [0.1, 0.3, 1.0, 0.0])
def test_dropout_philox_matches_oracle(codec_name, p):
    codec = _codec()
    L = _L()
    n = 1_000_003
    g = np.random.default_rng(11).standard_normal(n, dtype=np.float32)
    g[::9973] = np.inf
    seed, off = 42, 3
    cid = L.FC_CODEC_DROPOUT_BIASED if codec_name == "dropout-biased" else L.FC_CODEC_DROPOUT_UNBIASED
    pkt = codec.encode_mask(torch.from_numpy(g).cuda(), cid, p=p, seed=seed, offset=off)
    out = codec.decode(pkt, dtype=torch.float64).cpu().numpy()
    mask = ph.bernoulli_mask(n, p, seed, off).astype(np.int64)
    with np.errstate(invalid="ignore", divide="ignore"):
        ref = g * mask if codec_name == "dropout-biased" else (g * mask) / p
    _dropout_equal(out, ref)
    out32 = codec.decode(pkt).cpu().numpy()
    with np.errstate(invalid="ignore"):
        np.testing.assert_array_equal(out32, ref.astype(np.float32))


# ---- FedAVG ----------------------------------------------------------------------------
@pytest.mark.parametrize("name", G.cases("fedavg__"))
def test_fedavg_dense_golden(name):
    from openmsftl_amd import FedAvg
    Gm = G.arr(name, "G")
    out = FedAvg({"aggregation_scheme": "fed_avg"}).aggregate(Gm)
    assert out.tobytes() == G.arr(name, "output").tobytes()


@pytest.mark.parametrize("M,n,f", [(4, 4096, 0.1), (17, 100_003, 0.1), (64, 70_001, 0.01)])
def test_fedavg_packets_bit_exact(M, n, f):
    """Packets -> k_decode<ACC> == reference FedAvg on the dense G of the same rows."""
    codec = _codec()
    from openmsftl_amd import FedAvg
    rng = np.random.default_rng(M)
    grads = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-4, -1)).astype(np.float32)
             for _ in range(M)]
    k = co.num_kept(f, n)
    pkts = [codec.encode_top(torch.from_numpy(x).cuda(), k) for x in grads]
    agg = FedAvg({}).aggregate_packets(pkts).cpu().numpy()
    Gd = go.build_dense_G([co.compress({"compression_function": "top",
                                        "fraction_coordinate": f}, x) for x in grads], np.float32)
    ref = go.FedAvgOracle({}).aggregate(Gd)
    assert agg.tobytes() == ref.tobytes()


def test_fedavg_packets_without_qoff():
    """include/fedcodec.h: an encoder given qoff = NULL writes no quarter offsets; the fold
    then scans each chunk's whole slot range per quarter and is still bit-exact (ADVICE r02:
    it used to dereference the NULL pointer).  Mixed with packets that do carry qoff."""
    codec = _codec()
    M, n, f = 5, 70_001, 0.1
    rng = np.random.default_rng(505)
    grads = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-4, -1)).astype(np.float32)
             for _ in range(M)]
    k = co.num_kept(f, n)
    pkts = []
    for i, x in enumerate(grads):
        p = codec.Packet.alloc(n, 0, "cuda", k=k)
        if i % 2 == 0:
            p.qoff = None                                          # encoded with qoff = NULL
        pkts.append(codec.encode_top(torch.from_numpy(x).cuda(), k, packet=p))
    agg = codec.decode_accumulate(pkts, list(np.full(M, 1.0 / M, np.float32))).cpu().numpy()
    Gd = go.build_dense_G([co.compress({"compression_function": "top",
                                        "fraction_coordinate": f}, x) for x in grads], np.float32)
    assert agg.tobytes() == go.FedAvgOracle({}).aggregate(Gd).tobytes()


@pytest.mark.parametrize("split", [1, 5, 70])
def test_fedavg_continue_equals_one_call(split):
    """fc_decode_accumulate_continue: rows split across calls (or ranks of the chained
    reduce, distributed.py) fold to the same bits as one call; > 64 rows span launches."""
    codec = _codec()
    M, n, f = 96, 40_961, 0.05
    rng = np.random.default_rng(split)
    grads = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-4, -1)).astype(np.float32)
             for _ in range(M)]
    k = co.num_kept(f, n)
    pkts = [codec.encode_top(torch.from_numpy(x).cuda(), k) for x in grads]
    w = list(np.full(M, 1.0 / M, np.float32))
    one = codec.decode_accumulate(pkts, w).cpu().numpy()
    acc = codec.decode_accumulate(pkts[:split], w[:split])
    codec.decode_accumulate(pkts[split:], w[split:], out=acc, continue_sum=True)
    assert acc.cpu().numpy().tobytes() == one.tobytes()
    from openmsftl_amd.distributed import ShardedFedAvg, packet_fold
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    ShardedFedAvg().aggregate(packet_fold(pkts), M, out)       # world 1: plain fold
    assert out.cpu().numpy().tobytes() == one.tobytes()
    Gd = go.build_dense_G([co.compress({"compression_function": "top",
                                        "fraction_coordinate": f}, x) for x in grads], np.float32)
    assert one.tobytes() == go.FedAvgOracle({}).aggregate(Gd).tobytes()


def test_fedavg_packets_dropout_unbiased_and_weights():
    codec = _codec()
    L = _L()
    M, n, p = 9, 50_001, 0.1
    rng = np.random.default_rng(3)
    grads = [rng.standard_normal(n).astype(np.float32) for _ in range(M)]
    w = rng.uniform(-1, 1, M).astype(np.float32)
    pkts, rows = [], []
    for i, x in enumerate(grads):
        pk = codec.encode_mask(torch.from_numpy(x).cuda(), L.FC_CODEC_DROPOUT_UNBIASED, p=p,
                               seed=100 + i)
        pkts.append(pk)
        mask = ph.bernoulli_mask(n, p, 100 + i).astype(np.int64)
        rows.append(((x * mask) / p).astype(np.float32))
    agg = codec.decode_accumulate(pkts, list(w)).cpu().numpy()
    ref = go.sequential_weighted_sum(rows, w)
    np.testing.assert_array_equal(agg, ref)
    nz = ref != 0
    assert agg[nz].tobytes() == ref[nz].tobytes()


def _signed_zero_grads(M, n, rng):
    """Gradients built so that the FedAVG sum meets every sign-of-zero case: exact +-0
    entries (kept at f = 0.5 as ties), negative denormals whose weighted term underflows
    to -0, and columns where every row is -0."""
    grads = []
    for i in range(M):
        x = (rng.standard_normal(n) * 1e-3).astype(np.float32)
        sel = rng.uniform(size=n)
        x[sel < 0.45] = -0.0
        x[(sel >= 0.45) & (sel < 0.55)] = 0.0
        x[(sel >= 0.55) & (sel < 0.65)] = -np.float32(1e-45)
        # all-(-0) columns at the top indices: the tie rule keeps the highest indices of the
        # zero-key group first, so every row keeps them and their sum stays -0
        x[n - n // 16:] = -0.0
        grads.append(x)
    return grads


@pytest.mark.parametrize("wkind", ["mean", "negative", "mixed_signs", "nonfinite"])
def test_fedavg_packets_signed_zeros_and_weight_classes(wkind):
    """k_decode_sparse skips the dropped coordinates; the dense sum of gar.py:44 (NumPy's
    +0-started axis-0 add.reduce) adds fl(+0 * w) there: +-0 (neutral) or NaN (w = +-inf /
    NaN).  The packet FedAVG must equal the dense sum bit for bit (NaN positions for NaN)."""
    codec = _codec()
    M, n, f = 12, 20_011, 0.5
    rng = np.random.default_rng({"mean": 1, "negative": 2, "mixed_signs": 3, "nonfinite": 4}[wkind])
    grads = _signed_zero_grads(M, n, rng)
    if wkind == "mean":
        w = np.full(M, 1.0 / M, np.float32)
    elif wkind == "negative":
        w = -rng.uniform(0.01, 1, M).astype(np.float32)
    elif wkind == "mixed_signs":
        w = rng.uniform(-1, 1, M).astype(np.float32)
        w[2], w[5] = np.float32(0.0), np.float32(-0.0)
    else:
        w = rng.uniform(0.01, 1, M).astype(np.float32)
        w[3], w[7] = np.float32(np.inf), np.float32(np.nan)
    k = co.num_kept(f, n)
    pkts = [codec.encode_top(torch.from_numpy(x).cuda(), k) for x in grads]
    agg = codec.decode_accumulate(pkts, list(w)).cpu().numpy()
    rows = [co.compress({"compression_function": "top", "fraction_coordinate": f}, x)
            for x in grads]
    with np.errstate(invalid="ignore", over="ignore"):
        ref = go.sequential_weighted_sum([r.astype(np.float32) for r in rows], w)
    nan = np.isnan(ref)
    np.testing.assert_array_equal(np.isnan(agg), nan)
    assert agg[~nan].tobytes() == ref[~nan].tobytes()
    if wkind in ("mean", "negative"):           # np.sum's +0 start: no -0 survives
        top = slice(n - n // 16, n)
        assert (ref[top] == 0).all() and not np.signbit(agg[top]).any()
        assert not (np.signbit(agg) & (agg == 0)).any()


@pytest.mark.parametrize("M", [70, 129, 140])
def test_fedavg_packets_signed_zeros_across_launches(M):
    """> 128 packets: the sum continues across launches (acc_in), -0 bookkeeping included."""
    codec = _codec()
    n, f = 9_001, 0.5
    grads = _signed_zero_grads(M, n, np.random.default_rng(9))
    w = np.full(M, 1.0 / M, np.float32)
    k = co.num_kept(f, n)
    pkts = [codec.encode_top(torch.from_numpy(x).cuda(), k) for x in grads]
    agg = codec.decode_accumulate(pkts, list(w)).cpu().numpy()
    rows = [co.compress({"compression_function": "top", "fraction_coordinate": f}, x)
            for x in grads]
    ref = go.sequential_weighted_sum([r.astype(np.float32) for r in rows], w)
    assert agg.tobytes() == ref.tobytes()



# ---- aggregation rows: reference goldens (tests/golden/make_golden_agg.py) ---------------
def _agg():
    from conftest import agg_golden
    return agg_golden()


class _Client:
    """The attributes aggregation.py:59-66 reads from a client."""

    def __init__(self, cid, grad, cfg):
        from openmsftl_amd import Compression
        self.client_id, self.grad, self.C = cid, grad, Compression(cfg)


@pytest.mark.parametrize("name", [c for c in __import__("conftest").agg_golden().cases("fedavg_signed__")])
def test_fedavg_dense_signed_zero_golden(name):
    """k_wsum (dense FedAVG) against the reference's FedAvg on G with signed zeros."""
    from openmsftl_amd import FedAvg
    A = _agg()
    out = FedAvg({"aggregation_scheme": "fed_avg"}).aggregate(A.arr(name, "G"))
    assert out.tobytes() == A.arr(name, "output").tobytes()


@pytest.mark.parametrize("name", [c for c in __import__("conftest").agg_golden().cases("hier__")])
def test_aggregator_hierarchical_golden(name):
    """Aggregator.aggregate_grads with num_hierarchies > 0 (aggregation.py:68-75, 80-93) on the
    reference's own G ('full' rows), device merges + FedAvg == the reference's output."""
    from openmsftl_amd.aggregation import Aggregator
    A = _agg()
    Gm, sizes = A.arr(name, "G"), A.meta(name)["cluster_size_list"]
    clients = [_Client(i, Gm[i].copy(), {"compression_function": "full"}) for i in range(Gm.shape[0])]
    agg = Aggregator({"aggregation_scheme": "fed_avg", "num_hierarchies": len(sizes),
                      "cluster_size_list": sizes})
    agg.aggregate_grads(clients)
    assert agg.curr_G.cpu().numpy().tobytes() == A.arr(name, "merged").tobytes()
    assert agg.agg_grad.tobytes() == A.arr(name, "output").tobytes()


def _ref_merge_lines(m, sizes):
    """The progress lines the reference prints for its merge stages (aggregation.py:71, 88, 90)."""
    out = []
    for stage, cs in enumerate(sizes):
        num = m // cs
        b = [[i * cs, (i + 1) * cs] for i in range(num)]
        b[-1][1] = max(b[-1][1], m)
        out.append(f"{stage}-stage gradient aggregation: cluster size={cs}")
        out.append(f"#client clusters: {num}")
        out += [f"Averaging gradient from the {s}-th client to the {e}=th" for s, e in b]
        m = num
    return out


@pytest.mark.parametrize("sizes", [[], [3], [4, 2]])
def test_aggregator_top_packets_match_dense_reference(sizes, capsys):
    """The streamed packet path (host ring -> top-k encode -> packet fold / packet cluster
    means) == the dense G the reference builds from the same compressed rows, merged and
    reduced (oracle).  A budget of a few packets forces several fold groups per cluster.  The
    merge stages print the reference's progress lines."""
    from openmsftl_amd.aggregation import Aggregator
    M, n, f = 17, 40_961, 0.1
    rng = np.random.default_rng(len(sizes))
    cfg = {"compression_function": "top", "fraction_coordinate": f}
    grads = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-4, -1)).astype(np.float32)
             for _ in range(M)]
    for x in grads[:3]:
        x[:100] = -0.0                               # signed zeros in the kept set
    clients = [_Client(i, g, cfg) for i, g in enumerate(grads)]
    from openmsftl_amd.pipeline import packet_bytes
    agg = Aggregator({"aggregation_scheme": "fed_avg", "num_hierarchies": len(sizes),
                      "cluster_size_list": sizes,
                      "device_budget_bytes": 6 * 4 * n + 3 * packet_bytes(n) + (8 << 20)})
    capsys.readouterr()
    agg.aggregate_grads(clients)
    assert agg.agg_path == "stream"                # the streamed packet path ran
    assert capsys.readouterr().out.splitlines() == _ref_merge_lines(M, sizes)
    Gd = go.build_dense_G([co.compress(cfg, x) for x in grads], np.float32)
    for cs in sizes:
        Gd = go.merge_gradient(Gd, cs)
    ref = go.FedAvgOracle({}).aggregate(Gd)
    assert agg.agg_grad.tobytes() == ref.tobytes()
    with pytest.raises(Exception, match="Client List is Empty"):
        agg.aggregate_grads([])


# ---- QSGD (opt-in; parity unpinned w.r.t. the reference: pinned to oracle/qsgd_oracle.py) --
QSGD_CASES = [(1, 1), (5, 2), (4097, 2), (100_003, 1), (100_003, 4), (65_536, 8), (70_001, 14),
              ((1 << 20) + 3, 2)]


@pytest.mark.parametrize("n,bits", QSGD_CASES)
def test_qsgd_codes_and_values_match_oracle(n, bits):
    from oracle import qsgd_oracle as qo
    codec = _codec()
    rng = np.random.default_rng(n + bits)
    g = (rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 1)).astype(np.float32)
    if n > 10:
        g[:3] = [0.0, -0.0, 1e-40]
    seed, off = 1234 + bits, 7
    pkt = codec.encode_qsgd(torch.from_numpy(g).cuda(), bits, seed=seed, offset=off)
    h = pkt.header()
    assert h.codec == 5 and h.format == 2 and h.k == bits and h.status == 0
    assert h.p == pytest.approx(qo.norm64(g), rel=1e-12)        # fp64, reassociated sum
    words = pkt.codes.cpu().numpy().view(np.uint32)
    want = qo.encode(g, bits, seed, off, h.p)
    assert words[: want.shape[0]].tobytes() == want.tobytes()
    out = codec.decode_qsgd(pkt).cpu().numpy()
    assert out.tobytes() == qo.decode(want, n, bits, h.p).tobytes()


def test_qsgd_fedavg_and_statistics():
    """FedAVG over QSGD packets == the +0-started row-order sum of the decoded rows; and the
    quantiser's expectation is g / tau (the reference comment's scaling)."""
    from oracle import qsgd_oracle as qo
    codec = _codec()
    M, n, bits = 9, 50_021, 2
    rng = np.random.default_rng(11)
    grads = [rng.standard_normal(n).astype(np.float32) for _ in range(M)]
    pkts = [codec.encode_qsgd(torch.from_numpy(x).cuda(), bits, seed=i, offset=1)
            for i, x in enumerate(grads)]
    w = rng.uniform(0.01, 1, M).astype(np.float32)
    agg = codec.decode_accumulate_qsgd(pkts, list(w)).cpu().numpy()
    rows = [qo.decode(p.codes.cpu().numpy().view(np.uint32), n, bits, p.header().p) for p in pkts]
    assert agg.tobytes() == go.sequential_weighted_sum(rows, w).tobytes()
    # unbiased up to 1/tau: mean over 200 seeds of one gradient
    x = grads[0][:4096].copy()
    gx = torch.from_numpy(x).cuda()
    acc = np.zeros(4096, np.float64)
    for s in range(200):
        acc += codec.decode_qsgd(codec.encode_qsgd(gx, 4, seed=s)).cpu().numpy()
    s4 = 16.0
    t = qo.tau(4096, s4)
    err = np.abs(acc / 200 - x / t)
    bound = 4 * qo.norm64(x) / (s4 * t) / np.sqrt(200)           # ~4 sigma of one level step
    assert (err < bound).mean() > 0.999


def test_qsgd_fedavg_past_one_launch():
    """fc_qsgd_decode_accumulate folds at most kQsgdFoldM = 512 packets per launch (their scales
    in LDS) and continues the partial sum over longer folds: 700 packets (two launches) equal
    the +0-started row-order sum of the oracle-decoded rows, bit for bit."""
    from oracle import qsgd_oracle as qo
    codec = _codec()
    M, n, bits = 700, 4_099, 3
    rng = np.random.default_rng(12)
    grads = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-3, 0)).astype(np.float32) for _ in range(M)]
    pkts = [codec.encode_qsgd(torch.from_numpy(x).cuda(), bits, seed=i, offset=2)
            for i, x in enumerate(grads)]
    w = rng.uniform(0.01, 1, M).astype(np.float32)
    agg = codec.decode_accumulate_qsgd(pkts, list(w)).cpu().numpy()
    rows = [qo.decode(p.codes.cpu().numpy().view(np.uint32), n, bits, p.header().p) for p in pkts]
    assert agg.tobytes() == go.sequential_weighted_sum(rows, w).tobytes()


@pytest.mark.parametrize("bits_of", ["w4", "w8", "w16", "mixed"])
@pytest.mark.parametrize("n", [37, 65_541])
def test_qsgd_fedavg_each_code_width(bits_of, n):
    """The fold reads a launch's codes 16 B per lane when all its packets share one code width
    (4 / 8 / 16 bits: 32 / 16 / 8 elements per lane) and per quad otherwise: each equals the
    +0-started row-order sum of the oracle-decoded rows, bit for bit, on ragged n (a partial
    last lane and a partial last code word), and continue_sum folds into a partial sum."""
    from oracle import qsgd_oracle as qo
    codec = _codec()
    M = 11
    bits = {"w4": [2] * M, "w8": [5] * M, "w16": [12] * M,
            "mixed": [[2, 5, 12, 3][i % 4] for i in range(M)]}[bits_of]
    rng = np.random.default_rng(n + M)
    grads = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-3, 0)).astype(np.float32) for _ in range(M)]
    pkts = [codec.encode_qsgd(torch.from_numpy(x).cuda(), b, seed=i, offset=4)
            for i, (x, b) in enumerate(zip(grads, bits))]
    w = rng.uniform(0.01, 1, M).astype(np.float32)
    rows = [qo.decode(p.codes.cpu().numpy().view(np.uint32), n, b, p.header().p)
            for p, b in zip(pkts, bits)]
    agg = codec.decode_accumulate_qsgd(pkts, list(w)).cpu().numpy()
    assert agg.tobytes() == go.sequential_weighted_sum(rows, w).tobytes()
    part = codec.decode_accumulate_qsgd(pkts[:4], list(w[:4]))
    codec.decode_accumulate_qsgd(pkts[4:], list(w[4:]), out=part, continue_sum=True)
    assert part.cpu().numpy().tobytes() == agg.tobytes()


@pytest.mark.parametrize("n", [1, 1000])
def test_qsgd_one_hot_keeps_its_element(n):
    """a one-hot gradient at bits = 14 lost its element (level s + 1 -> 0) about
    once per 1024 encodes.  500 seeds: the codes equal the oracle's and the element always
    decodes to +-norm / tau, never 0."""
    from oracle import qsgd_oracle as qo
    codec = _codec()
    bits = 14
    g = np.zeros(n, np.float32)
    g[n // 2] = np.float32(-0.37)
    gd = torch.from_numpy(g).cuda()
    s = 2.0 ** bits
    want_v = np.float32(-(qo.norm64(g) / (s * qo.tau(n, s))) * s)
    for seed in range(500):
        pkt = codec.encode_qsgd(gd, bits, seed=seed, offset=3)
        h = pkt.header()
        words = pkt.codes.cpu().numpy().view(np.uint32)
        want = qo.encode(g, bits, seed, 3, h.p)
        assert words[: want.shape[0]].tobytes() == want.tobytes()
        assert codec.decode_qsgd(pkt).cpu().numpy()[n // 2] == want_v, seed


def test_qsgd_compression_surface():
    """'qsgd' raises NotImplementedError as in the reference unless opted in."""
    from openmsftl_amd import Compression
    from oracle import qsgd_oracle as qo
    g = np.random.default_rng(2).standard_normal(10_007).astype(np.float32)
    with pytest.raises(NotImplementedError):
        Compression({"compression_function": "qsgd"}).compress(g)
    C = Compression({"compression_function": "qsgd", "qsgd": "native", "num_bits": 2, "seed": 5})
    out = C.compress(g)
    assert out.dtype == np.float32 and out.shape == g.shape
    levels = np.unique(np.abs(out))
    assert levels.shape[0] <= 5                                   # 0..s levels, s = 4
    want = qo.compress(g, 2, 5, 1, qo.norm64(g))
    np.testing.assert_allclose(out, want, rtol=1e-6, atol=0)      # norm: fp64 reassociation


# ---- flat-layout staging (model_helper.py:11-35, client.py:44,52-54) ---------------------------
LENET_SHAPES = [(20, 1, 5, 5), (20,), (50, 20, 5, 5), (50,), (500, 800), (500,), (10, 500), (10,)]


@pytest.mark.parametrize("shapes", [LENET_SHAPES, [(1,)], [(3,)] * 700 + [(70_001,)],
                                    [(4_194_305,), (7,), (2, 3, 4)]])
def test_flat_stage_matches_model_helper(shapes):
    from openmsftl_amd.model_helper import FlatLayout
    from oracle import model_helper_oracle as mo
    rng = np.random.default_rng(len(shapes))
    old = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    new = [(o - np.float32(0.01) * rng.standard_normal(s).astype(np.float32)).astype(np.float32)
           for o, s in zip(old, shapes)]
    if new[0].size > 2:                                    # exact-zero deltas and specials
        new[0].flat[0] = old[0].flat[0]
        old[0].flat[1], new[0].flat[1] = np.float32(-0.0), np.float32(0.0)
        new[0].flat[2] = np.inf
    params = [torch.from_numpy(o.copy()).cuda() for o in old]
    lay = FlatLayout(params)
    flat = lay.flatten()
    cur = mo.flatten_params(old)
    assert flat.cpu().numpy().tobytes() == cur.tobytes()
    for p, x in zip(params, new):                           # "train": overwrite in place
        p.copy_(torch.from_numpy(x))
    grad = lay.client_delta(flat)
    want_grad, want_cur = mo.client_step_delta(cur, new)
    assert grad.cpu().numpy().tobytes() == want_grad.tobytes()
    assert flat.cpu().numpy().tobytes() == want_cur.tobytes()
    agg = torch.from_numpy(rng.standard_normal(lay.n).astype(np.float32)).cuda()
    lay.scatter(agg)
    back = mo.dist_weights_to_model(agg.cpu().numpy(), shapes)
    for p, b in zip(params, back):
        assert p.cpu().numpy().tobytes() == b.tobytes()


def test_flat_stage_arguments():
    from openmsftl_amd.model_helper import FlatLayout
    with pytest.raises(TypeError):
        FlatLayout([torch.zeros(3, dtype=torch.float64, device="cuda")])
    with pytest.raises(ValueError):
        FlatLayout([])


@pytest.mark.timeout(120)
def test_batched_compaction_past_the_grid_y_limit():
    """k_compact_mag1 runs on a 3-D grid (client in the interleave group, chunk, group) while a
    client has at most 65,535 chunks (the grid's y limit) and on the linear, divided grid past
    it.  One gradient of 2^29 + 12,345 elements (65,537 chunks) through the batched encode
    (linear grid) and through the lone fused encode (k_fused_mag, which maps chunks itself): the
    two packets are byte-equal (same plan, same bracket), and the decoded result keeps exactly k
    coordinates, none smaller in magnitude than any dropped one."""
    codec = _codec()
    n, f = (1 << 29) + 12_345, 0.01
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(23))
    k = co.effective_k(co.num_kept(f, n), n)
    lone = codec.encode_top(g, k)
    [batch] = codec.encode_top_batch([g], k)
    torch.cuda.synchronize()
    assert _packet_bytes(batch) == _packet_bytes(lone)
    q = codec.decode(batch)
    kept = q != 0
    assert int(kept.sum()) == k
    assert float(g.abs()[kept].min()) >= float(g.abs()[~kept].max())


@pytest.mark.timeout(120)
def test_graphed_calls_equal_eager_calls():
    """codec.GraphedCalls: the lone packet encode + decode, fc_topk_encode_decode, a native
    rand-k encode, the drop-in dense encode and a batched encode + fold, captured into one HIP
    graph and replayed three times, give the eager calls' bytes (the fused kernels' bracket tags
    and every self-cleaning counter live on the device, so replays line up with eager calls)."""
    codec = _codec()
    from openmsftl_amd import _lib as L
    n, M, f = 3_000_017, 6, 0.1
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device="cuda").manual_seed(29)
    grads = [torch.randn(n, device="cuda", generator=gen) * (10.0 ** -(1 + i % 3)) for i in range(M)]
    k = co.effective_k(co.num_kept(f, n), n)
    ref_pkt = _packet_bytes(codec.encode_top(grads[0], k))
    ref_dense = codec.compress_top_dense(grads[1], k).clone()
    w = [1.0 / M] * M
    ref_pk = codec.encode_top_batch(grads, k)
    ref_acc = codec.decode_accumulate(ref_pk, w).clone()
    pkt = codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    dpkt = codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k)
    dense = torch.empty(n, dtype=torch.float32, device=dev)
    pk = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k) for _ in range(M)]
    jobs = codec.encode_jobs(grads, pk)
    views = codec.views_tensor(pk, w, dev)
    acc = torch.empty(n, dtype=torch.float32, device=dev)

    ref_ed = codec.encode_decode_top(grads[2], k)
    ref_ed = (_packet_bytes(ref_ed[0]), ref_ed[1].clone())
    ref_rk = _packet_bytes(codec.encode_top(grads[3], k, key_mode=L.FC_KEY_PHILOX, seed=3, offset=9))
    epkt = codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k)
    eout = torch.empty(n, dtype=torch.float32, device=dev)
    rpkt = codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k)

    def calls():
        codec.encode_top(grads[0], k, packet=pkt, check=False)
        codec.decode(pkt, out=out)
        codec.encode_decode_top(grads[2], k, packet=epkt, out=eout, check=False)
        codec.encode_top(grads[3], k, key_mode=L.FC_KEY_PHILOX, seed=3, offset=9, packet=rpkt, check=False)
        codec.compress_top_dense(grads[1], k, out=dense, packet=dpkt, check=False)
        codec.encode_top_batch(grads, k, packets=pk, jobs=jobs, check=False)
        codec.decode_accumulate(pk, w, out=acc, views=views)

    gc = codec.GraphedCalls(calls)
    for _ in range(3):
        out.zero_(); dense.zero_(); acc.zero_(); eout.zero_()
        gc.replay()
        torch.cuda.synchronize()
        assert codec.resolve([pkt]) == 0 and codec.resolve(pk) == 0
        assert codec.resolve([epkt]) == 0 and codec.resolve([rpkt]) == 0
        assert _packet_bytes(epkt) == ref_ed[0] and torch.equal(eout.view(torch.int32), ref_ed[1].view(torch.int32))
        assert _packet_bytes(rpkt) == ref_rk
        assert dpkt.header().status == 0
        assert _packet_bytes(pkt) == ref_pkt
        assert torch.equal(dense.view(torch.int32), ref_dense.view(torch.int32))
        assert torch.equal(acc.view(torch.int32), ref_acc.view(torch.int32))
        assert torch.equal(out.view(torch.int32), codec.decode(codec.encode_top(grads[0], k)).view(torch.int32))


@pytest.mark.parametrize("n,f,seed", [(1_000_003, 0.1, 1), (16_777_216, 0.1, 2), (16_777_216, 0.01, 3),
                                      (25_557_032, 0.01, 4), (300_001, 0.5, 5), (8_192 * 40 + 17, 0.3, 6)])
def test_encode_decode_top_equals_encode_then_decode(n, f, seed):
    """fc_topk_encode_decode (the resolve's gather and finish inside the decode launch): the
    packet — entries, counts, quarter offsets and the header with T64, n_entries, status — is
    fc_topk_encode's (+ k_resolve) byte for byte, and out equals fc_decode_dense of it and the
    oracle's compress('top') (compression.py:31-37)."""
    codec = _codec()
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 1)).astype(np.float32)
    x[rng.integers(0, n, 50)] = 0.0
    g = torch.from_numpy(x).cuda()
    k = co.effective_k(co.num_kept(f, n), n)
    ref = codec.encode_top(g, k)
    want = codec.decode(ref).cpu().numpy()
    for _ in range(3):                                      # reused workspace: self-cleaning
        p, out = codec.encode_decode_top(g, k)
        assert _packet_bytes(p) == _packet_bytes(ref)
        assert p.hdr.cpu().numpy().tobytes() == ref.hdr.cpu().numpy().tobytes()
        assert torch.equal(p.qoff, ref.qoff) and torch.equal(p.cnt, ref.cnt)
        assert out.cpu().numpy().tobytes() == want.tobytes()
    assert want.tobytes() == co.compress({"compression_function": "top", "fraction_coordinate": f},
                                         x).tobytes()


def test_encode_decode_top_ties_and_rank0():
    """Heavy ties at the threshold (many equal magnitudes in bin beta) and a k that the
    definite set fills exactly (rank 0: every candidate is slack)."""
    codec = _codec()
    n = 2_000_000
    rng = np.random.default_rng(9)
    x = rng.standard_normal(n).astype(np.float32)
    x[:300_000] = np.float32(0.5)                           # a tied plateau
    g = torch.from_numpy(x).cuda()
    for k in (co.num_kept(0.1, n), int((np.abs(x) > 0.5).sum()), int((np.abs(x) > 0.5).sum()) + 1000):
        ref = codec.encode_top(g, k)
        want = codec.decode(ref).cpu().numpy()
        p, out = codec.encode_decode_top(g, k)
        assert p.hdr.cpu().numpy().tobytes() == ref.hdr.cpu().numpy().tobytes(), k
        assert out.cpu().numpy().tobytes() == want.tobytes(), k
