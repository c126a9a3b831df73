"""The host-resident FedAVG round on more than one GPU (GPU): BASELINE configs[4]'s
H2D -> encode -> fold -> cross-GPU combine -> D2H path.

* ``DeviceRing`` (one process, one pipeline per GPU, the drop-in ``Aggregator``'s fan-out)
  and ``RankRing`` (one rank per GPU): fold groups dealt round-robin, the running aggregate
  passed on in group order — bit-exact against the oracle's one-process FedAVG
  (compression.py:31-37 -> aggregation.py:61-63 -> gar.py:44).  Two pipelines / two gloo
  ranks share cuda:0, standing in for two GPUs.
* ``tools/e2e_bench.py --gpus 2`` (the configs[4] runner itself, two gloo ranks) over the
  committed configs[4] inputs (70 x 25,557,032, top f = 0.01): ring and chain modes give the
  oracle's aggregate digest; reduce mode gives fl32(P0 + P1) of the two shards' partial sums
  (the single fp32 addition a 2-rank sum-reduce performs; each partial sum is bit-exact).
The oracle here is the checker only (packet_oracle / gar_oracle, numpy)."""
import hashlib
import importlib.util
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN_DIR
from oracle import gar_oracle as go
from oracle import packet_oracle as po

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 300_007                                   # ragged: the last chunk is partial
FRAC = 0.1


def _k():
    from openmsftl_amd.compression import kept_count
    return kept_count(FRAC, N)


def _grads(M, seed):
    rng = np.random.default_rng(seed)
    return [(rng.standard_normal(N) * 10.0 ** rng.uniform(-4, -1)).astype(np.float32)
            for _ in range(M)]


def _want(grads):
    k = _k()
    rows = []
    for g in grads:
        idx, val = po.topk_packet(g, k)
        rows.append(po.decode_dense(N, idx, val))
    return go.FedAvgOracle({}).aggregate(np.stack(rows))


def _pipes(count, group):
    from openmsftl_amd.pipeline import HostFedAvg
    dev = torch.device("cuda", 0)
    return [HostFedAvg(N, _k(), group=group, ring=2, device=dev, sets=2) for _ in range(count)]


@pytest.mark.timeout(120)
@pytest.mark.parametrize("pipes,group,pinned", [(2, 3, False), (3, 2, True), (2, 64, True)])
def test_device_ring_bit_exact(pipes, group, pinned):
    """13 clients, groups of 2-3 dealt over 2-3 pipelines (the aggregate hops 4-6 times);
    group 64 = one group, one pipeline idle.  Run twice: reused pipelines, same bytes."""
    from openmsftl_amd.pipeline import DeviceRing
    grads = _grads(13, seed=pipes * 10 + group)
    want = _want(grads)
    host = [torch.from_numpy(g).pin_memory() for g in grads] if pinned else grads
    ring = DeviceRing(_pipes(pipes, group))
    for _ in range(2):
        got = ring.run(host, len(grads)).numpy()
        assert got.tobytes() == want.tobytes()


@pytest.mark.timeout(120)
def test_device_ring_forced_retry_is_exact():
    """A client whose sampled bracket 'missed' (status poked to RETRY after its encode) is
    re-encoded exactly from its host copy before its group is folded."""
    from openmsftl_amd import _lib as L
    from openmsftl_amd.pipeline import DeviceRing
    grads = _grads(7, seed=5)
    want = _want(grads)
    pipes = _pipes(2, 2)
    orig = pipes[1].encode_group

    def poked(get, rows, ps=0, plan=None):
        orig(get, rows, ps, plan)
        # after the status copy was queued: overwrite the pinned status of the group's first
        # client once the encode is done (check_group waits on the same event first)
        pipes[1].encoded[ps].synchronize()
        pipes[1].status_host[ps][0].copy_(torch.tensor([L.FC_STATUS_RETRY_EXACT, 0, 0, 0],
                                                       dtype=torch.uint8))
    pipes[1].encode_group = poked
    ring = DeviceRing(pipes)
    got = ring.run(grads, len(grads)).numpy()
    assert got.tobytes() == want.tobytes()
    assert ring.exact_fallbacks >= 1


@pytest.mark.timeout(120)
def test_rank_ring_one_process():
    """RankRing without a process group is the one-GPU fold (world 1)."""
    from openmsftl_amd.pipeline import RankRing
    grads = _grads(9, seed=3)
    want = _want(grads)
    rr = RankRing(_pipes(1, 4)[0])
    got = rr.run(grads, len(grads))
    assert got.cpu().numpy().tobytes() == want.tobytes()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_ring_worker(rank, world, port, M, group, seed, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from openmsftl_amd.pipeline import HostFedAvg, RankRing
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        grads = _grads(M, seed)
        calls = []

        def get(i):
            calls.append(i)
            return grads[i]
        rr = RankRing(HostFedAvg(N, _k(), group=group, ring=2, device=dev, sets=2), dst=0)
        out = rr.run(get, M)
        torch.cuda.synchronize()
        if rank == 0:
            q.put(("agg", out.cpu().numpy().copy()))
        q.put(("rows", rank, sorted(set(calls))))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(150)
@pytest.mark.parametrize("M,group", [(13, 3), (13, 4), (2, 4)])
def test_rank_ring_two_gloo_ranks(M, group):
    """Two ranks, groups dealt round-robin: (13, 3) ends on rank 0 = dst; (13, 4) ends on
    rank 1, which sends the result to rank 0; (2, 4) leaves rank 1 without a group.  Each
    rank streams only its own groups' rows."""
    import torch.multiprocessing as mp
    from openmsftl_amd.pipeline import group_bounds
    grads = _grads(M, seed=M * 100 + group)
    want = _want(grads)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_ring_worker, args=(r, 2, port, M, group, M * 100 + group, q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(3):
            item = q.get(timeout=100)
            res[item[0] if item[0] == "agg" else (item[0], item[1])] = item[-1]
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert res["agg"].tobytes() == want.tobytes()
    for r in range(2):
        mine = sorted(i for t, g in enumerate(group_bounds(M, group)) if t % 2 == r for i in g)
        assert res[("rows", r)] == mine


def _rank_ring_plan_worker(rank, world, port, M, group, codec_name, q):
    """RankRing with a row plan whose masks are drawn on the host: each rank draws every row's
    mask in order (its own taken, the others dropped), so both ranks leave np.random where the
    reference's one-process loop does."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from openmsftl_amd.aggregation import row_plan
        from openmsftl_amd.compression import Compression
        from openmsftl_amd.pipeline import HostFedAvg, RankRing
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        grads = _grads(M, seed=11)

        class Client:
            def __init__(self, g):
                self.grad, self.C = g, Compression({"compression_function": codec_name,
                                                    "dropout_p": 0.3, "fraction_coordinate": 0.1})
        np.random.seed(5)
        plan = row_plan([Client(g) for g in grads], N)
        rr = RankRing(HostFedAvg(N, group=group, ring=2, device=dev, sets=2), dst=0)
        out = rr.run(grads, M, plan=plan)
        plan.close()
        torch.cuda.synchronize()
        q.put(("next", rank, int(np.random.randint(0, 2 ** 31 - 1))))
        if rank == 0:
            q.put(("agg", out.cpu().numpy().copy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(150)
@pytest.mark.parametrize("codec_name", ["dropout-unbiased", "rand"])
def test_rank_ring_two_gloo_ranks_host_draws(codec_name):
    """The ring across two ranks with host-drawn masks ('dropout-unbiased' / 'rand' in parity
    mode): the aggregate equals the one-process reference round (oracle) byte for byte and
    every rank's RNG ends where the reference's does."""
    import torch.multiprocessing as mp
    from oracle import compression_oracle as co
    M, group = 7, 2
    grads = _grads(M, seed=11)
    cfg = {"compression_function": codec_name, "dropout_p": 0.3, "fraction_coordinate": 0.1}
    np.random.seed(5)
    rows = [np.asarray(co.compress(cfg, g), np.float32) for g in grads]
    nxt = int(np.random.randint(0, 2 ** 31 - 1))
    want = go.FedAvgOracle({}).aggregate(np.stack(rows))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_ring_plan_worker, args=(r, 2, port, M, group, codec_name, q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(3):
            item = q.get(timeout=100)
            res[item[0] if item[0] == "agg" else (item[0], item[1])] = item[-1]
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert res[("next", 0)] == nxt and res[("next", 1)] == nxt
    assert res["agg"].tobytes() == want.tobytes()


@pytest.mark.timeout(120)
def test_aggregator_fans_out_over_devices():
    """The drop-in Aggregator with aggregation_config["devices"] = [0, 0]: a DeviceRing of two
    pipelines (two stand-ins for two GPUs), agg_grad byte-equal to the oracle's FedAVG; and a
    fold-group budget small enough that the 11 clients cross several groups and hops."""
    from openmsftl_amd import Compression
    from openmsftl_amd.aggregation import Aggregator
    from openmsftl_amd.pipeline import DeviceRing, packet_bytes

    class Client:
        def __init__(self, cid, grad, C):
            self.client_id, self.grad, self.C = cid, grad, C
    grads = _grads(11, seed=21)
    want = _want(grads)
    C = Compression({"compression_function": "top", "fraction_coordinate": FRAC})
    budget = (4 + 2) * 4 * N + (1 << 22) + 2 * 3 * packet_bytes(N)     # 3 packets per set
    agg = Aggregator({"aggregation_scheme": "fed_avg", "devices": [0, 0],
                      "device_budget_bytes": budget})
    agg.aggregate_grads([Client(i, g, C) for i, g in enumerate(grads)])
    assert agg.agg_path == "stream"
    (pipe,) = agg._host_pipelines.values()
    assert isinstance(pipe, DeviceRing) and len(pipe.pipes) == 2 and pipe.group < 11
    assert agg.agg_grad.tobytes() == want.tobytes()


# ---- configs[4] at full size through the multi-rank runner -------------------------------
D4 = json.load(open(os.path.join(GOLDEN_DIR, "digests_full.json")))["configs4"]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _runner(tmp_path, mode, group=16):
    agg = tmp_path / f"agg_{mode}.npy"
    cmd = [sys.executable, os.path.join(ROOT, "tools", "e2e_bench.py"), "--gpus", "2",
           "--backend", "gloo", "--source", "configs4", "--mode", mode, "--group", str(group),
           "--warmup", "0", "--reps", "1", "--dump-agg", str(agg)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    proc = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert proc.returncode == 0, proc.stderr[-4000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, proc.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["clients"] == D4["clients"] and line["mode"] == mode
    print(f"\n[configs4 e2e 2 gloo ranks, {mode}] {line['value']} GB/s "
          f"(one GPU shared; rehearsal, not a measurement)")
    return np.load(agg)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["ring", "chain"])
def test_configs4_runner_two_ranks_bit_exact(tmp_path, mode):
    got = _runner(tmp_path, mode)
    assert sha(got) == D4["aggregate_sha256"], f"configs4 {mode}: aggregate differs"


@pytest.mark.timeout(300)
def test_configs4_runner_two_ranks_reduce(tmp_path):
    """Reduce mode: rank r folds rows shard_range(70, 2, r) from +0 (bit-exact partial sums,
    recomputed here through HostFedAvg on the same inputs); the 2-rank sum-reduce adds them
    once in fp32."""
    from openmsftl_amd.distributed import fedavg_weights, shard_range
    from openmsftl_amd.pipeline import HostFedAvg
    spec = importlib.util.spec_from_file_location("make_digests_full",
                                                  os.path.join(GOLDEN_DIR, "make_digests_full.py"))
    MD = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(MD)
    got = _runner(tmp_path, "reduce")
    M, n, k = D4["clients"], D4["n"], D4["k"]
    w = fedavg_weights(M)
    pipe = HostFedAvg(n, k, group=16)
    parts = []
    for r in range(2):
        rows = shard_range(M, 2, r)
        host = [torch.from_numpy(MD.fullsize_grad("configs4", i)).pin_memory() for i in rows]
        parts.append(pipe.run(host, len(rows), w[rows.start:rows.stop]).numpy().copy())
        del host
    want = np.add(parts[0], parts[1], dtype=np.float32)
    assert got.tobytes() == want.tobytes()
