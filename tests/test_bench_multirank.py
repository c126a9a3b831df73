"""bench.py --gpus N is a real N-rank run (GPU): the launcher starts one process per rank
before touching the GPU, every rank issues exactly one reduce per step (a retry forced on ONE
rank re-encodes and re-folds locally before that reduce), and the aggregate matches the
oracle's FedAVG (gar.py:44 over server.py:74's sampled clients) within distributed.py's
stated reassociation bound.  Two gloo ranks share the one GPU of the box."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import gar_oracle as go
from oracle import packet_oracle as po

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M, N, W, F = 4, 1_048_576, 2, 0.1


def _run_bench(tmp_path, extra=()):
    agg = tmp_path / "agg.npy"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(W), "--backend", "gloo",
           "--clients", str(M), "--n", str(N), "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-single", "--roofline-steps", "0",
           "--dump-agg", str(agg), *extra]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    proc = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert proc.returncode == 0, proc.stderr[-4000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, proc.stdout[-2000:]          # ONE JSON line, from rank 0 only
    return json.loads(lines[0]), np.load(agg)


def _oracle_rows():
    import bench
    from openmsftl_amd.compression import kept_count
    k = kept_count(F, N)
    rows = []
    for r in range(W):
        for g in bench.make_grads(M, N, r, torch.device("cuda", 0), torch):
            idx, val = po.topk_packet(g.cpu().numpy(), k)
            rows.append(po.decode_dense(N, idx, val))
    return rows


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_rank_bench_forced_retry_on_one_rank(tmp_path):
    line, got = _run_bench(tmp_path, ("--force-retry-rank", "1"))
    assert line["n_gpus"] == W
    assert line["config"]["parallelism"] == f"dp{W}"
    assert line["extra"]["exact_fallbacks"] == 1          # rank 1's poked packet, once
    assert line["value"] > 0
    rows = _oracle_rows()
    w = np.full(M * W, 1.0 / (M * W), np.float32)
    want = go.sequential_weighted_sum(rows, w)
    mag = np.sum(np.abs(np.stack(rows) * w[:, None]), axis=0, dtype=np.float64)
    tol = (M * W + W) * 2.0 ** -24 * mag                  # distributed.py's stated bound
    assert np.all(np.abs(got.astype(np.float64) - want) <= tol)
    assert np.count_nonzero(got) > 0


def test_world_mismatch_is_refused(tmp_path):
    """--gpus must equal the launched world size (no silent one-rank run)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                           "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=120)
    assert proc.returncode != 0
    assert "WORLD_SIZE" in proc.stderr


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_rccl_world1_bench_issues_its_reduce(tmp_path):
    """The RCCL code path on a one-GPU box: bench.py --gpus 1 --backend
    nccl --force-pg initialises a one-rank nccl group (device_id=), and every step issues its
    one async reduce (the work handle waited on two steps later, stream-ordered against the
    next encodes).  The aggregate equals the world-1 fold bit for bit (a one-rank sum-reduce
    adds nothing) = the oracle's FedAVG of the rank's clients."""
    agg = tmp_path / "agg.npy"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--backend", "nccl",
           "--force-pg", "--clients", str(M), "--n", str(N), "--steps", "4", "--warmup", "1",
           "--no-cpu-baseline", "--no-single", "--no-matrix", "--roofline-steps", "0",
           "--dump-agg", str(agg)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    proc = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert proc.returncode == 0, proc.stderr[-4000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    line = json.loads(lines[-1])
    assert line["n_gpus"] == 1
    assert line["extra"]["process_group"] == {"backend": "nccl", "world": 1,
                                              "collective_per_step": "reduce (async)"}
    got = np.load(agg)
    import bench
    from openmsftl_amd.compression import kept_count
    k = kept_count(F, N)
    rows = []
    for g in bench.make_grads(M, N, 0, torch.device("cuda", 0), torch):
        idx, val = po.topk_packet(g.cpu().numpy(), k)
        rows.append(po.decode_dense(N, idx, val))
    want = go.sequential_weighted_sum(rows, np.full(M, 1.0 / M, np.float32))
    assert got.tobytes() == want.tobytes()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_rccl_world1_e2e_reduce(tmp_path):
    """tools/e2e_bench.py --gpus 1 --backend nccl --mode reduce --force-pg: the configs[4]
    runner's reduce mode through a one-rank nccl group (the collective issued on the fold's
    device buffer), on the committed configs[4] inputs: the aggregate digest equals the
    oracle's (70 x 25.5 M, top f = 0.01)."""
    import hashlib
    from conftest import GOLDEN_DIR
    d4 = json.load(open(os.path.join(GOLDEN_DIR, "digests_full.json")))["configs4"]
    agg = tmp_path / "agg.npy"
    cmd = [sys.executable, os.path.join(ROOT, "tools", "e2e_bench.py"), "--gpus", "1",
           "--backend", "nccl", "--mode", "reduce", "--force-pg", "--source", "configs4",
           "--group", "16", "--warmup", "0", "--reps", "1", "--dump-agg", str(agg)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    proc = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert proc.returncode == 0, proc.stderr[-4000:]
    line = json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["process_group"] is True and line["backend"] == "nccl" and line["mode"] == "reduce"
    got = np.load(agg)
    assert hashlib.sha256(got.tobytes()).hexdigest() == d4["aggregate_sha256"]
