"""N>1 FedAVG with the HIP codec on the data path (GPU): two gloo ranks share cuda:0.

Each rank encodes its shard of the clients with the HIP top-k encoder, folds its packets
(``packet_fold`` -> fc_decode_accumulate) and combines through ShardedFedAvg
(openmsftl_amd/distributed.py); gloo stages the device partial sums through host memory.
  * chain: bit-exact against the oracle's one-process FedAVG of the clients' dense q
    (compression.py:31-37 -> aggregation.py:61-63 -> gar.py:44);
  * reduce: within the reassociation bound stated in distributed.py.
The oracle here is the checker only (packet_oracle / gar_oracle, numpy)."""
import os
import socket

import numpy as np
import pytest

from oracle import gar_oracle as go
from oracle import packet_oracle as po

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N = 300_007                                   # ragged: the last 8192-element chunk is partial
FRAC = 0.1


def _grads(M, seed):
    rng = np.random.default_rng(seed)
    return [(rng.standard_normal(N) * 10.0 ** rng.uniform(-4, -1)).astype(np.float32)
            for _ in range(M)]


def _k():
    from openmsftl_amd.compression import kept_count
    return kept_count(FRAC, N)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, M, mode, seed, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from openmsftl_amd import codec
        from openmsftl_amd.distributed import ShardedFedAvg, packet_fold, shard_range
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        grads = _grads(M, seed)
        rows = shard_range(M, world, rank)
        pkts = [codec.encode_top(torch.from_numpy(grads[i]).to(dev), _k()) for i in rows]
        out = torch.empty(N, dtype=torch.float32, device=dev)
        ShardedFedAvg(mode=mode, dst=0).aggregate(packet_fold(pkts), M, out)
        torch.cuda.synchronize()
        if rank == 0:
            q.put(out.cpu().numpy().copy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, M, mode, seed):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, M, mode, seed, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    return res


def _oracle_rows(M, seed):
    k = _k()
    rows = []
    for g in _grads(M, seed):
        idx, val = po.topk_packet(g, k)
        rows.append(po.decode_dense(N, idx, val))
    return rows


@pytest.mark.timeout(150)
@pytest.mark.parametrize("M", [6, 1])         # M=1: rank 1's shard is empty
def test_two_ranks_chain_bit_exact(M):
    rows = _oracle_rows(M, seed=M)
    want = go.FedAvgOracle({}).aggregate(np.stack(rows))
    got = _run(2, M, "chain", seed=M)
    assert got.tobytes() == want.tobytes()


@pytest.mark.timeout(150)
def test_two_ranks_reduce_within_bound():
    M, W = 7, 2
    rows = _oracle_rows(M, seed=11)
    w = np.full(M, 1.0 / M, np.float32)
    want = go.sequential_weighted_sum(rows, w)
    got = _run(W, M, "reduce", seed=11)
    mag = np.sum(np.abs(np.stack(rows) * w[:, None]), axis=0, dtype=np.float64)
    tol = (M + W) * 2.0 ** -24 * mag                     # distributed.py's stated bound
    assert np.all(np.abs(got.astype(np.float64) - want) <= tol)
    assert not np.array_equal(got, np.zeros_like(got))
