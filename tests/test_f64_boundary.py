"""float64 gradients / weights and the drop-in boundary.

Goldens: tests/golden/make_golden_f64.py ran the REFERENCE on float64 inputs
(attack_models.py:105-106 -> aggregation.py:61) and on float64 GAR weights (DGA,
aggregation.py:181-198).  CPU tests pin the oracle to them and check the integration recipe
(tools/check_integration.py) against /root/reference when it is present; GPU tests run the
product (Compression, Aggregator, FedAvg, the patched aggregate_grads) through the C ABI.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN_DIR, ROOT
from oracle import compression_oracle as co
from oracle import gar_oracle as go


class F64Golden:
    def __init__(self):
        with open(os.path.join(GOLDEN_DIR, "manifest_f64.json")) as fh:
            self.manifest = json.load(fh)
        self.arrays = np.load(os.path.join(GOLDEN_DIR, "golden_f64.npz"))

    def cases(self, prefix=""):
        return sorted(k for k in self.manifest["cases"] if k.startswith(prefix))

    def meta(self, name):
        return self.manifest["cases"][name]

    def input(self, name):
        return self.arrays["input|" + self.meta(name)["input"]]

    def arr(self, name, key):
        return self.arrays[f"{name}|{key}"]


F = F64Golden()


def tie_at_cut64(g: np.ndarray, k: int) -> bool:
    """True when the k-th largest |g| (NaN above +inf, as argsort orders it) is tied with the
    (k+1)-th: the reference's unstable argsort then picks implementation-defined members."""
    n = g.shape[0]
    if k <= 0 or k >= n:
        return False
    u = np.ascontiguousarray(g, dtype=np.float64).view(np.uint64) & np.uint64(0x7FFFFFFFFFFFFFFF)
    u = np.where(u > np.uint64(0x7FF0000000000000), np.uint64(0x7FF0000000000001), u)
    keys = np.sort(u)[::-1]
    return bool(keys[k - 1] == keys[k])


class _Client:
    """The attributes aggregate_grads reads (aggregation.py:61-63, 76)."""

    def __init__(self, cid, grad, C):
        self.client_id, self.grad, self.C = cid, grad, C


# ---- CPU: the oracle against the reference's float64 outputs --------------------------------
@pytest.mark.parametrize("name", F.cases("top|"))
def test_oracle_top_f64(name):
    m, g = F.meta(name), F.input(name)
    out = co.compress({"compression_function": "top", "fraction_coordinate": m["fraction"]}, g.copy())
    ref = F.arr(name, "output")
    assert out.dtype == ref.dtype == np.float64
    k = co.effective_k(co.num_kept(m["fraction"], g.shape[0]), g.shape[0])
    if not tie_at_cut64(g, k):
        assert out.tobytes() == ref.tobytes()


@pytest.mark.parametrize("name", F.cases("rand|") + F.cases("dropout-"))
def test_oracle_rng_codecs_f64(name):
    m, g = F.meta(name), F.input(name)
    np.random.seed(m["seed"])
    cfg = {"compression_function": m["codec"], "fraction_coordinate": m.get("fraction", 0.5),
           "dropout_p": m.get("p", 0.5)}
    with np.errstate(invalid="ignore"):
        out = co.compress(cfg, g)
    assert int(np.random.randint(0, 2**31 - 1)) == m["rng_next"]
    assert out.dtype == np.float64
    assert out.tobytes() == F.arr(name, "output").tobytes()        # -0.0 included


def _oracle_aggregate(m, grads, weights):
    """aggregation.py:54-78 restated with the oracle (rows in order, merges, gar.py:44)."""
    np.random.seed(m["seed"])
    cfg = {"compression_function": m["codec"], "fraction_coordinate": 0.1, "dropout_p": 0.3}
    Gm = go.build_dense_G([co.compress(cfg, g) for g in grads], grads.dtype)
    for cs in m["agg_cfg"].get("cluster_size_list", []):
        Gm = go.merge_gradient(Gm, cs)
    f = go.FedAvgOracle({})
    if weights.size:
        f.gradient_weights = weights
    with np.errstate(invalid="ignore"):
        return f.aggregate(Gm)


@pytest.mark.parametrize("name", F.cases("agg|"))
def test_oracle_aggregate_f64(name):
    m = F.meta(name)
    out = _oracle_aggregate(m, F.arr(name, "grads"), F.arr(name, "weights"))
    ref = F.arr(name, "output")
    assert out.dtype == ref.dtype and out.tobytes() == ref.tobytes()


# ---- CPU: the boundary ---------------------------------------------------------------------
def test_full_returns_the_callers_object():
    """compression.py:27-29: 'full' returns the input itself (no copy, no GPU needed)."""
    import torch
    from openmsftl_amd.compression import Compression
    C = Compression({"compression_function": "full"})
    g = np.arange(7, dtype=np.float32)
    assert C.compress(g) is g
    t = torch.arange(5, dtype=torch.float32)
    assert C.compress(t) is t
    g64 = np.zeros(3)
    assert C.compress(g64) is g64


@pytest.mark.skipif(not os.path.isdir("/root/reference/ftl"),
                    reason="the reference tree exists only in the build container")
def test_integration_recipe_against_reference():
    """INTEGRATION.md §1-§2 applied to OpenMSFTL itself: device GAR bound where __get_gar looks
    (aggregation.py:15,47-48), aggregate_grads swapped, no GPU touched."""
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_integration.py")],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    assert json.loads(line)["ok"] is True


# ---- GPU: the product ----------------------------------------------------------------------
def _gpu_compression(cfg):
    from openmsftl_amd.compression import Compression
    return Compression(cfg)


@pytest.mark.gpu
@pytest.mark.parametrize("name", F.cases("top|"))
def test_gpu_top_f64(name):
    m, g = F.meta(name), F.input(name)
    out = _gpu_compression({"compression_function": "top", "fraction_coordinate": m["fraction"]}).compress(g)
    assert out.dtype == np.float64 and out.shape == g.shape
    want = co.compress({"compression_function": "top", "fraction_coordinate": m["fraction"]}, g.copy())
    assert out.tobytes() == want.tobytes()                         # the oracle's tie rule
    k = co.effective_k(co.num_kept(m["fraction"], g.shape[0]), g.shape[0])
    if not tie_at_cut64(g, k):
        assert out.tobytes() == F.arr(name, "output").tobytes()    # the reference itself


@pytest.mark.gpu
@pytest.mark.parametrize("name", F.cases("rand|") + F.cases("dropout-"))
def test_gpu_rng_codecs_f64(name):
    m, g = F.meta(name), F.input(name)
    np.random.seed(m["seed"])
    cfg = {"compression_function": m["codec"], "fraction_coordinate": m.get("fraction", 0.5),
           "dropout_p": m.get("p", 0.5)}
    out = _gpu_compression(cfg).compress(g)
    assert int(np.random.randint(0, 2**31 - 1)) == m["rng_next"]   # same RNG consumption
    assert out.dtype == np.float64
    assert out.tobytes() == F.arr(name, "output").tobytes()        # -0.0 / NaN included


@pytest.mark.gpu
@pytest.mark.parametrize("n,f", [(1, 0.5), (2049, 0.37), (1 << 20, 0.1), (3_000_001, 0.01)])
def test_gpu_top_f64_sizes_and_ties(n, f):
    rng = np.random.default_rng(n)
    g = rng.standard_normal(n)
    g[rng.random(n) < 0.3] = 0.5                                   # a large tie group
    g[rng.random(n) < 0.01] = -0.0
    out = _gpu_compression({"compression_function": "top", "fraction_coordinate": f}).compress(g)
    want = co.compress({"compression_function": "top", "fraction_coordinate": f}, g)
    assert out.tobytes() == want.tobytes()


@pytest.mark.gpu
def test_gpu_philox_rand_f64_selects_the_fp32_set():
    """Native rand-k keys depend on the index only: the float64 path keeps the same set."""
    n, f = 100_003, 0.1
    g = np.random.default_rng(1).standard_normal(n) + 3.0          # no zeros
    cfg = {"compression_function": "rand", "fraction_coordinate": f, "rng": "philox", "seed": 77}
    q64 = _gpu_compression(cfg).compress(g)
    q32 = _gpu_compression(cfg).compress(g.astype(np.float32))
    assert q64.dtype == np.float64
    assert np.array_equal(q64 != 0, q32 != 0)
    assert np.count_nonzero(q64) == co.num_kept(f, n)
    np.testing.assert_array_equal(q64[q64 != 0], g[q64 != 0])


@pytest.mark.gpu
@pytest.mark.parametrize("name", F.cases("agg|"))
def test_gpu_aggregator_f64(name):
    from openmsftl_amd.aggregation import Aggregator
    from openmsftl_amd.compression import Compression
    m = F.meta(name)
    grads, w = F.arr(name, "grads"), F.arr(name, "weights")
    np.random.seed(m["seed"])
    cfg = {"compression_function": m["codec"], "fraction_coordinate": 0.1, "dropout_p": 0.3}
    clients = [_Client(i, grads[i].copy(), Compression(cfg)) for i in range(grads.shape[0])]
    A = Aggregator(m["agg_cfg"])
    if w.size:
        A.gar.gradient_weights = w
    A.aggregate_grads(clients)
    ref = F.arr(name, "output")
    assert A.agg_grad.dtype == ref.dtype
    assert A.agg_grad.tobytes() == ref.tobytes()


@pytest.mark.gpu
def test_gpu_patched_aggregate_grads_with_reference_style_gar():
    """integration.install() binds aggregation.aggregate_grads onto the REFERENCE Aggregator,
    whose GAR may lack aggregate_packets (fed_spectral_avg, or FedAvg bound before install):
    it must then receive the host G the reference builds.  The reference is absent on the GPU
    box, so a class with the reference's attributes stands in, and the oracle's FedAvg (a
    restatement of gar.py:32-56) plays the reference GAR."""
    from openmsftl_amd import aggregation
    from openmsftl_amd.compression import Compression
    from conftest import golden
    G = golden()
    name = "fedavg__M4__n4096__top"
    Gm, order = G.arr(name, "G"), G.arr(name, "order")

    class RefStyleAggregator:                                     # aggregation.py:26-41
        aggregate_grads = aggregation.aggregate_grads

        def __init__(self):
            self.gar = go.FedAvgOracle({"aggregation_scheme": "fed_avg"})
            self.curr_G = None
            self.agg_grad = None
            self.analyze_pc = False
            self.num_hierarchies = 0
            self.cluster_size_list = []

    # the golden G rows are already compressed: 'full' clients reproduce them as G's rows
    clients = [_Client(int(order[i]), Gm[i].copy(), Compression({"compression_function": "full"}))
               for i in range(Gm.shape[0])]
    A = RefStyleAggregator()
    A.aggregate_grads(clients)
    assert isinstance(A.curr_G, np.ndarray) and A.curr_G.tobytes() == Gm.tobytes()
    assert A.agg_grad.tobytes() == G.arr(name, "output").tobytes()
    # top clients on the same gradients: packets cannot feed a host GAR -> dense host G
    rng = np.random.default_rng(0)
    grads = [rng.standard_normal(4096).astype(np.float32) for _ in range(4)]
    cfg = {"compression_function": "top", "fraction_coordinate": 0.1}
    A2 = RefStyleAggregator()
    A2.aggregate_grads([_Client(i, g, Compression(cfg)) for i, g in enumerate(grads)])
    want = go.FedAvgOracle({}).aggregate(go.build_dense_G([co.compress(cfg, g) for g in grads],
                                                          np.float32))
    assert A2.agg_grad.tobytes() == want.tobytes()


@pytest.mark.gpu
def test_gpu_fedavg_weight_dtypes():
    """gar.py:44 promotes G * w: float32 G with float64 weights -> float64 result (and
    aggregate_packets refuses float64 weights rather than silently rounding them)."""
    import torch
    from openmsftl_amd import codec
    from openmsftl_amd.gar import FedAvg
    rng = np.random.default_rng(3)
    Gm = rng.standard_normal((6, 1001)).astype(np.float32)
    w64 = rng.random(6)
    f = FedAvg({})
    f.gradient_weights = w64
    got = f.aggregate(Gm)
    ref = go.FedAvgOracle({})
    ref.gradient_weights = w64
    want = ref.aggregate(Gm)
    assert got.dtype == np.float64 and got.tobytes() == want.tobytes()
    pk = [codec.encode_top(torch.from_numpy(r).cuda(), 100) for r in Gm]
    with pytest.raises(TypeError):
        f.aggregate_packets(pk)


# ---- the sampled fp64 path (fc_topk_dense_f64_sampled) against the exact radix select ------
def _f64_inputs(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "gauss":
        return rng.standard_normal(n) * 10.0 ** rng.uniform(-4, -1)
    if kind == "layers":                       # per-"layer" scales 1e-6 .. 1e2
        g = rng.standard_normal(n)
        cuts = np.sort(rng.choice(n, 7, replace=False))
        for j, (a, b) in enumerate(zip(np.r_[0, cuts], np.r_[cuts, n])):
            g[a:b] *= 10.0 ** (j - 6)
        return g
    if kind == "lowbits":                      # many values share their high 32 key bits
        return 1.0 + rng.integers(0, 1 << 20, n) * 2.0 ** -52 * rng.choice([-1.0, 1.0], n)
    if kind == "special":
        g = rng.standard_normal(n)
        g[rng.integers(0, n, 50)] = np.inf
        g[rng.integers(0, n, 50)] = -np.inf
        g[rng.integers(0, n, 50)] = np.nan
        g[rng.random(n) < 0.05] = -0.0
        return g
    raise ValueError(kind)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["gauss", "layers", "lowbits", "special"])
@pytest.mark.parametrize("n,f", [((1 << 20) + 3, 0.1), (3_000_001, 0.01), (16_777_216 + 5, 0.1)])
def test_gpu_sampled_top_f64_equals_exact(kind, n, f):
    """Sampled bracket + one streaming pass + exact candidate select gives the exact radix
    select's bytes; on Gaussian-like gradients without a retry."""
    import torch
    from openmsftl_amd import codec
    g = torch.from_numpy(_f64_inputs(kind, n, n % 1000)).cuda()
    k = co.num_kept(f, n)
    want = codec.compress_top_dense_f64(g, k, exact=True)
    got = codec.compress_top_dense_f64(g, k, check=False)
    redo = codec.resolve_f64(got)
    assert got.cpu().numpy().tobytes() == want.cpu().numpy().tobytes()
    if kind in ("gauss", "layers"):
        assert redo == 0, "sampled bracket missed on a Gaussian-like gradient"


@pytest.mark.gpu
def test_gpu_sampled_top_f64_vs_oracle_and_reuse():
    """3 M Gaussian, f = 0.1: the oracle's bytes, twice on one workspace (self-cleaning)."""
    import torch
    from openmsftl_amd import codec
    n, f = 3_000_017, 0.1
    g = _f64_inputs("gauss", n, 9)
    want = co.compress({"compression_function": "top", "fraction_coordinate": f}, g.copy())
    gd = torch.from_numpy(g).cuda()
    for _ in range(2):
        got = codec.compress_top_dense_f64(gd, co.num_kept(f, n))
        assert got.cpu().numpy().tobytes() == want.tobytes()
