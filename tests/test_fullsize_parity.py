"""Full-size parity of the workloads the benchmarks time (GPU).

The oracle's SHA-256 digests (tests/golden/make_digests_full.py, build container) of:
  * configs[2]: 128 clients x 16,777,216, top f = 0.1, batched encode (fc_topk_encode_batch,
    two forked streams) — every client's dense q (compression.py:31-37) and the FedAVG
    aggregate of the 128 packets (aggregation.py:61-63 -> gar.py:44);
  * configs[3] shard shape: 8 clients x 134,217,728 through encode_top_batch(streams=2) and
    the 8-packet fold, as bench.py runs its 128-client shard;
  * configs[4]: 70 clients x 25,557,032, top f = 0.01, through openmsftl_amd.pipeline.HostFedAvg
    (H2D -> encode -> fold in groups of 64 -> D2H: the continued fold is crossed), as
    tools/e2e_bench.py runs it.
plus the single-client fused paths (fc_topk_encode_dense / fc_topk_encode) on client 0 of
configs[2] (= configs[1], one 16 M gradient) and of configs[3] (the single 128 M gradient).
Inputs are regenerated here bit-identically (torch's CPU generator; the input digests of the
first clients are checked first, so a generator difference is reported as such).
"""
import hashlib
import importlib.util
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR

pytestmark = pytest.mark.gpu

D = json.load(open(os.path.join(GOLDEN_DIR, "digests_full.json")))
_spec = importlib.util.spec_from_file_location("make_digests_full",
                                               os.path.join(GOLDEN_DIR, "make_digests_full.py"))
MD = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MD)


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _device_grads(name, count, device):
    import torch
    out = []
    for c in range(count):
        g = MD.fullsize_grad(name, c)
        want = D[name]["input_sha256"].get(str(c))
        if want is not None:
            assert sha(g) == want, f"{name}: input generator differs for client {c}"
        out.append(torch.from_numpy(g).to(device))
    return out


def _check_batch(name, streams=2):
    import torch
    from openmsftl_amd import codec
    from openmsftl_amd.distributed import fedavg_weights
    d = D[name]
    M, n, k = d["clients"], d["n"], d["k"]
    dev = torch.device("cuda", 0)
    grads = _device_grads(name, M, dev)
    pkts = codec.encode_top_batch(grads, k, streams=streams)     # check=True: resolves retries
    del grads
    bad = []
    q = torch.empty(n, dtype=torch.float32, device=dev)
    for c, p in enumerate(pkts):
        codec.decode(p, out=q)
        if sha(q.cpu().numpy()) != d["q_sha256"][str(c)]:
            bad.append(c)
    assert not bad, f"{name}: dense q differs from the oracle for clients {bad[:10]}"
    w = fedavg_weights(M)
    agg = codec.decode_accumulate(pkts, [float(x) for x in w])
    assert sha(agg.cpu().numpy()) == d["aggregate_sha256"], f"{name}: FedAVG aggregate differs"


@pytest.mark.timeout(300)
def test_configs2_128x16M_batched_encode_and_fold():
    _check_batch("configs2")


@pytest.mark.timeout(300)
def test_configs3_shard_shape_8x128M_batched_encode_and_fold():
    _check_batch("configs3")


@pytest.fixture(scope="module")
def configs4_host():
    """configs[4]'s 70 x 25.5 M client gradients as host NumPy arrays (7.2 GB, made once)."""
    d = D["configs4"]
    host = []
    for c in range(d["clients"]):
        g = MD.fullsize_grad("configs4", c)
        want = d["input_sha256"].get(str(c))
        if want is not None:
            assert sha(g) == want, f"configs4: input generator differs for client {c}"
        host.append(g)
    return host


@pytest.mark.timeout(300)
def test_configs4_host_ring_70x25M(configs4_host):
    import torch
    from openmsftl_amd.pipeline import HostFedAvg
    d = D["configs4"]
    M, n, k = d["clients"], d["n"], d["k"]
    host = [torch.from_numpy(g).pin_memory() for g in configs4_host]
    pipe = HostFedAvg(n, k, group=d["group"], ring=4)
    out = pipe.run(host, M)
    assert sha(out.numpy()) == d["aggregate_sha256"], "configs4: ring aggregate differs"
    # a second pass over the same pipeline (reused packets and workspaces) gives the same bytes
    assert sha(pipe.run(host, M).numpy()) == d["aggregate_sha256"]


class _Client:
    """The reference Client's fields aggregation.py:54-78 reads (client_id, grad, C)."""

    def __init__(self, cid, grad, C):
        self.client_id, self.grad, self.C = cid, grad, C


@pytest.mark.timeout(300)
@pytest.mark.parametrize("pin", ["stage", "register"])
def test_configs4_device_aggregator_70x25M(configs4_host, pin):
    """The integrated path driver.py runs: openmsftl_amd.aggregation.Aggregator
    .aggregate_grads over 70 fake clients whose ``grad`` is a pageable NumPy array
    (client.py:53), top f = 0.01 (aggregation.py:54-78 -> gar.py:44), NumPy in, NumPy
    ``agg_grad`` out.  Streamed through the bounded host ring (pinned staging, or the arrays
    page-locked in place) in fold groups of 64: equal to the oracle's aggregate digest.
    Prints the NumPy-to-NumPy rate."""
    import time

    import torch
    from openmsftl_amd import Compression
    from openmsftl_amd.aggregation import Aggregator
    d = D["configs4"]
    C = Compression({"compression_function": "top", "fraction_coordinate": d["fraction"]})
    clients = [_Client(i, g, C) for i, g in enumerate(configs4_host)]
    agg = Aggregator({"aggregation_scheme": "fed_avg"})
    agg._host_pipelines = {}
    agg.aggregate_grads(clients)                       # allocates the ring + packets
    agg._host_pipelines[next(iter(agg._host_pipelines))].pin = pin
    assert agg.agg_path == "stream"
    assert sha(agg.agg_grad) == d["aggregate_sha256"], "configs4: Aggregator aggregate differs"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agg.aggregate_grads(clients)                       # weights persisted (gar.py:41-42)
    dt = time.perf_counter() - t0
    assert sha(agg.agg_grad) == d["aggregate_sha256"]
    gbps = 4.0 * d["n"] * d["clients"] / dt / 1e9
    print(f"\n[configs4 Aggregator numpy->numpy pin={pin}] {dt:.3f} s = {gbps:.2f} GB/s "
          f"of client gradients")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("codec_name,clients", [("full", 70), ("dropout-unbiased", 32),
                                                ("dropout-biased", 16), ("rand", 6)])
def test_configs4_device_aggregator_other_codecs(configs4_host, codec_name, clients):
    """The Aggregator's streamed path for the other codecs at the configs[4] size (25.5 M):
    'full' (the reference's configured codec, client_config.json:48) over all 70 clients,
    'dropout-*' p = 0.1 (np.random.binomial's own MT19937 draws made on the device,
    openmsftl_amd/csrc/fc_mt.hip) and 'rand' f = 0.01 (host permutation masks drawn from
    np.random in row order) over the first clients, with the default device budget; agg_grad
    byte-equal to the oracle's row-order fold of the oracle's rows (compression.py:39-60,
    gar.py:44) and the RNG where the reference leaves it.  Prints the NumPy-to-NumPy rate
    (DESIGN.md §5)."""
    import time

    from oracle import compression_oracle as co
    from oracle import gar_oracle as go
    from openmsftl_amd import Compression
    from openmsftl_amd.aggregation import Aggregator
    cfg = {"compression_function": codec_name, "dropout_p": 0.1, "fraction_coordinate": 0.01}
    grads = configs4_host[:clients]
    w = np.full(clients, 1.0 / clients, np.float32)
    np.random.seed(4)
    want = go.sequential_weighted_sum((np.asarray(co.compress(cfg, g), np.float32) for g in grads), w)
    nxt = int(np.random.randint(0, 2 ** 31 - 1))
    agg = Aggregator({"aggregation_scheme": "fed_avg"})
    C = Compression(cfg)
    for rep in range(2):
        np.random.seed(4)
        t0 = time.perf_counter()
        agg.aggregate_grads([_Client(i, g, C) for i, g in enumerate(grads)])
        dt = time.perf_counter() - t0
        assert agg.agg_path == "stream"
        assert agg.agg_draws == {"full": None, "rand": "host"}.get(codec_name, "device-mt")
        assert int(np.random.randint(0, 2 ** 31 - 1)) == nxt
        assert agg.agg_grad.tobytes() == want.tobytes(), f"{codec_name}: aggregate differs"
    gbps = 4.0 * D["configs4"]["n"] * clients / dt / 1e9
    print(f"\n[configs4 Aggregator numpy->numpy {codec_name} x {clients}] {dt:.3f} s = "
          f"{gbps:.2f} GB/s of client gradients")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", ["configs2", "configs3"])
def test_single_client_fused_paths_fullsize(name):
    """The single-client paths at full size against the same oracle digests: BASELINE
    configs[1] (one 16 M gradient = client 0 of configs2) and the north star's single 128 M
    gradient (client 0 of configs3), through the drop-in dense path (k_fused_mag<true> +
    k_resolve's in-kernel fix-up) and the packet path (k_fused_mag<false> + k_resolve, then the
    dense decode)."""
    import torch
    from openmsftl_amd import codec
    d = D[name]
    n, k = d["n"], d["k"]
    (g,) = _device_grads(name, 1, torch.device("cuda", 0))
    q = codec.compress_top_dense(g, k)
    assert sha(q.cpu().numpy()) == d["q_sha256"]["0"], f"{name}: fused dense q differs"
    del q
    p = codec.encode_top(g, k)
    assert sha(codec.decode(p).cpu().numpy()) == d["q_sha256"]["0"], f"{name}: packet path differs"
