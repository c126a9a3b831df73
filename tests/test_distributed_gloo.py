"""N>1 path of the FedAVG reduce on CPU (gloo, world_size 2 and 3): client sharding, the
reassociating sum-reduce and the bit-exact chained fold (openmsftl_amd/distributed.py).

The local fold here is the oracle's sequential fp32 sum (the arithmetic of gar.py:44); on
the GPU the same orchestration runs k_decode<ACC> (tests/test_gpu_parity.py covers that
fold bit-exactly, and bench.py drives it over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gar_oracle as go
from openmsftl_amd.distributed import ShardedFedAvg, fedavg_weights, shard_range


def _rows(M, n, seed=0):
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(M):
        r = (rng.standard_normal(n) * 10.0 ** rng.uniform(-4, -1)).astype(np.float32)
        r[rng.random(n) < 0.9] = 0.0                      # top-k-like sparsity (f = 0.1)
        rows.append(r)
    return rows


def _oracle_fold(all_rows):
    def fold(rows, w, out, continue_sum):
        acc = out.numpy()
        for j, i in enumerate(rows):
            c = np.multiply(all_rows[i], w[j])
            if j == 0 and not continue_sum:
                acc[:] = np.add(np.zeros_like(c), c)      # np.sum's +0 start (gar.py:44)
            else:
                acc[:] = np.add(acc, c)
        return out
    return fold


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, M, n, mode, dst, seed, q, async_op=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = _rows(M, n, seed)
        out = torch.empty(n, dtype=torch.float32)
        fa = ShardedFedAvg(mode=mode, dst=dst)
        if async_op:                                      # bench.py's overlapped reduce
            work = fa.aggregate(_oracle_fold(rows), M, out, async_op=True)
            work.wait()
        else:
            fa.aggregate(_oracle_fold(rows), M, out)
        if rank == dst:
            q.put(out.numpy().copy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, M, n, mode, dst=0, seed=0, async_op=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, M, n, mode, dst, seed, q, async_op))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_shard_range_partitions_rows_in_order():
    for M in (0, 1, 7, 128, 1024):
        for W in (1, 2, 3, 8):
            got = [i for r in range(W) for i in shard_range(M, W, r)]
            assert got == list(range(M))
            sizes = [len(shard_range(M, W, r)) for r in range(W)]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def test_weights_match_reference_default():
    w = fedavg_weights(10)
    assert w.dtype == np.float32 and w.tobytes() == np.full(10, 1.0 / 10, np.float32).tobytes()
    with pytest.raises(Exception):
        fedavg_weights(0)


@pytest.mark.parametrize("world,M", [(2, 8), (3, 7), (2, 1)])
def test_chain_is_bit_exact(world, M):
    n = 4099
    rows = _rows(M, n)
    ref = go.sequential_weighted_sum(rows, fedavg_weights(M))
    got = _run(world, M, n, "chain", dst=0)
    assert got.tobytes() == ref.tobytes()
    G = np.stack(rows)
    assert got.tobytes() == go.FedAvgOracle({}).aggregate(G).tobytes()   # gar.py:44 itself


@pytest.mark.parametrize("world,M,async_op", [(2, 8, False), (3, 10, False), (2, 8, True)])
def test_reduce_within_reassociation_bound(world, M, async_op):
    n = 4099
    rows = _rows(M, n, seed=1)
    w = fedavg_weights(M)
    ref = go.sequential_weighted_sum(rows, w)
    got = _run(world, M, n, "reduce", seed=1, async_op=async_op)
    mag = np.sum(np.abs(np.stack(rows) * w[:, None]), axis=0, dtype=np.float64)
    tol = (M + world) * 2.0 ** -24 * mag                 # stated in distributed.py
    assert np.all(np.abs(got.astype(np.float64) - ref) <= tol)


def test_chain_to_other_dst():
    M, n = 5, 1000
    rows = _rows(M, n, seed=2)
    ref = go.sequential_weighted_sum(rows, fedavg_weights(M))
    assert _run(2, M, n, "chain", dst=0, seed=2).tobytes() == ref.tobytes()
    assert _run(3, M, n, "chain", dst=1, seed=2).tobytes() == ref.tobytes()
