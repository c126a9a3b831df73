#!/usr/bin/env python3
"""Headline benchmark: device-resident gradient encode+decode GB/s (BASELINE.json `metric`).

Workload (BASELINE.json configs[3], per-GPU shard): every GPU holds M = 128 synthetic client
gradients of N = 134,217,728 fp32 (s_c * N(0,1), s_c log-uniform in [1e-4, 1e-1], generated
on device).  One step = for every client a top-k (f = 0.1) encode into a device packet
(compression.py:31-37), then the FedAVG decode-accumulate of all M packets (aggregation.py:61-63
+ gar.py:44, bit-exact fp32), then — with N > 1 GPUs — one RCCL fp32 reduce of the partial
aggregate to rank 0.  Weak scaling: per-GPU work is fixed.

    python bench.py [--gpus 1] [--steps 10] [--warmup 2]
    torchrun --nproc-per-node N ... bench.py --gpus N       (one process per GPU, RCCL)

Prints ONE JSON line on rank 0.  `value` = gradient bytes (4 N per client, all ranks) per
second of step time; `roofline` = the encode pass k_compact_mag1 (the dominant kernel), algorithmic
bytes 4N + 8k per client (ABI-3 packets write 6 B per entry) over its HIP-event-timed average launch duration, `traffic` from the
committed calibrated PMC summary; `cpu_baseline` = the reference's exact NumPy calls
(compression.py:31-37, default argsort) on one 128 M gradient, with every BASELINE.md §3 row
in `extra.cpu_baseline_matrix`.  A self-check outside the timed region re-encodes two clients
alone and compares them bit for bit with the batch.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# SURVEY.md §8(d) prices a packet entry at 8 B (uint32 idx + fp32 val) in the algorithmic bytes
# that roofline.achieved must use; ABI-3 packets actually carry 6 B (uint16 chunk-local index),
# which the PMC `traffic` field shows (below the algorithmic bytes, not above)
ENTRY_BYTES = 8.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)   # ~5.3 s timed: visible to a 5-s GPU-busy sampler
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clients", type=int, default=128, help="clients per GPU")
    ap.add_argument("--n", type=int, default=134_217_728, help="gradient length (fp32)")
    ap.add_argument("--fraction", type=float, default=0.1)
    ap.add_argument("--streams", type=int, default=1,
                    help="forked streams the batched encode is split over (the sub-batches' "
                         "encodes still run one after the other; 1 = one launch chain)")
    ap.add_argument("--roofline-steps", type=int, default=5,
                    help="extra encode passes with one stream, timed per launch for `roofline`")
    ap.add_argument("--lib", default=None, help="A/B only: load this libfedcodec.so build")
    ap.add_argument("--tag", default=None, help="A/B only: a label echoed in the JSON line")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (RCCL over xGMI: the measurement) or gloo (rehearsal only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single", action="store_true", help="skip the single-gradient probe")
    ap.add_argument("--no-matrix", action="store_true",
                    help="skip the SURVEY §8(d) codec matrix (extra.codec_matrix)")
    ap.add_argument("--pipeline", action="store_true",
                    help="fold each encode chain's packets on its stream as soon as they are "
                         "encoded (codec.encode_fold_batch; measured no faster, A/B only)")
    ap.add_argument("--no-batch", action="store_true",
                    help="encode client by client (fc_topk_encode) instead of batched")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r06_pmc_k_compact_mag1.json"),
                    help="PMC summary (profiles/) used for roofline.traffic")
    ap.add_argument("--force-retry-rank", type=int, default=-1,
                    help="test only: on this rank, mark client 0's packet RETRY in the last "
                         "timed step (exercises the rank-uniform exact re-encode)")
    ap.add_argument("--dump-agg", default=None,
                    help="test only: rank 0 saves the last step's aggregate (.npy) here")
    ap.add_argument("--force-pg", action="store_true",
                    help="initialise the process group and issue the step's collective even at "
                         "one rank (tests the RCCL code path on a one-GPU box)")
    return ap.parse_args()


def init_pg(dist, backend, world, rank, device, force=False) -> bool:
    """The process group of this run: the launcher's env:// rendezvous for world > 1; with
    ``force`` at world 1 a one-rank group on a free local port.  Returns whether one exists."""
    if world <= 1 and not force:
        return False
    kw = {"device_id": device} if backend == "nccl" else {}
    if world <= 1 and "MASTER_ADDR" not in os.environ:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                world_size=1, **kw)
    else:
        dist.init_process_group(backend, **kw)
    return True


def spawn_ranks(argv, nproc, script=None):
    """`bench.py --gpus N` without a launcher: start N ranks (one process per GPU, the env
    torch.distributed.run would set: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*) as CHILD
    processes running ``script`` (default this file), before this process touches the GPU, and
    return the worst exit code (never exec: the parent stays alive and GPU-free).  A rank that
    fails ends the others."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script or __file__)]
                                      + list(argv), env=env))
    log(f"[launcher] {nproc} ranks, pids {[p.pid for p in procs]}, port {port}")
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:                      # a failed rank would hang the others
                    q.terminate()
        time.sleep(0.05)
    return rc


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_grads(M, n, rank, device, torch):
    """Client c's gradient: s_c * N(0,1) from torch.Generator(device).manual_seed(1000 + c).
    The M gradients are the rows of one (M, N') slab (N' = N rounded up to 4 floats, so every
    row starts 16-B aligned), the layout of the reference's G (gar.py:44): as M separate
    allocations the 128 x 16 M batched encode ran 3-5 % slower (1.77-1.80 ms against 1.72;
    128 M rows: 1 %), profiles/r05_stagger_probe.jsonl."""
    import numpy as np
    srng = np.random.default_rng(7)
    scales = 10.0 ** srng.uniform(-4, -1, size=(rank + 1) * M)[rank * M:]
    stride = (n + 3) // 4 * 4
    slab = torch.empty((M, stride), device=device, dtype=torch.float32)
    grads = []
    for i in range(M):
        gen = torch.Generator(device=device).manual_seed(1000 + rank * M + i)
        g = slab[i, :n]
        torch.randn(n, device=device, generator=gen, dtype=torch.float32, out=g)
        g.mul_(float(scales[i]))
        grads.append(g)
    return grads


def _timed(fn):
    t0 = time.perf_counter()
    out = fn()
    return out, time.perf_counter() - t0


def cpu_baseline(n, fraction):
    """The reference's own top-k call on one client gradient: oracle/compression_oracle.py with
    ``argsort_kind=None``, i.e. exactly compression.py:31-37 (np.zeros_like, round(f*N),
    np.argsort(np.abs(g)) with NumPy's DEFAULT kind, [::-1][:k], scatter), single-threaded."""
    import numpy as np
    from oracle import compression_oracle as co
    g = np.random.default_rng(0).standard_normal(n, dtype=np.float32)
    g *= np.float32(1e-2)
    cfg = {"compression_function": "top", "fraction_coordinate": fraction}
    q, dt = _timed(lambda: co.compress(cfg, g, argsort_kind=None))
    assert q.shape == g.shape
    return {"value": round(4.0 * n / dt / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "cpu_model": _cpu_model(),
            "sample": f"1 client x {n:,} fp32, top f={fraction}: the reference's exact NumPy "
                      f"calls (compression.py:31-37, default-kind argsort; "
                      f"oracle/compression_oracle.py argsort_kind=None), single-threaded; "
                      f"{dt:.2f} s on {os.cpu_count()} visible host cores (1 used)"}


def _cpu_model() -> str:
    """The host CPU's model name (record it beside the CPU baseline)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_matrix(n16=16_777_216, n25=25_557_032):
    """every codec of compression.py:23-77 and gar.py:44's FedAvg, the
    reference's exact NumPy calls (oracle, default argsort kind, legacy np.random), one core,
    on a bounded sample (one 16 M / 25.5 M client, 4 x 16 M for FedAvg), plus the per-config
    CPU time extrapolated linearly in clients."""
    import numpy as np
    from oracle import compression_oracle as co
    from oracle import gar_oracle as go
    g = np.random.default_rng(1).standard_normal(n16, dtype=np.float32) * np.float32(1e-2)
    rows = {}

    def row(name, cfg, grad, seed=0):
        np.random.seed(seed)
        _, dt = _timed(lambda: co.compress(cfg, grad, argsort_kind=None))
        rows[name] = {"ms": round(1e3 * dt, 1), "GBps": round(4.0 * grad.shape[0] / dt / 1e9, 4),
                      "n": int(grad.shape[0])}
        return dt

    t_top16 = row("top_f0.1_16M", {"compression_function": "top", "fraction_coordinate": 0.1}, g)
    row("top_f0.01_16M", {"compression_function": "top", "fraction_coordinate": 0.01}, g)
    row("rand_f0.1_16M", {"compression_function": "rand", "fraction_coordinate": 0.1}, g)
    row("dropout-biased_p0.1_16M", {"compression_function": "dropout-biased", "dropout_p": 0.1}, g)
    row("dropout-unbiased_p0.1_16M", {"compression_function": "dropout-unbiased", "dropout_p": 0.1}, g)
    rows["full_16M"] = {"ms": 0.0, "GBps": None, "n": n16,
                        "note": "compression.py:27-29 returns the caller's array (no work)"}
    g25 = np.random.default_rng(2).standard_normal(n25, dtype=np.float32) * np.float32(1e-2)
    t_top25 = row("top_f0.01_25.5M", {"compression_function": "top", "fraction_coordinate": 0.01}, g25)
    del g25
    # BASELINE configs[0]: one 4-client round on LeNet-sized gradients (431,080), top f = 0.1
    # (client_config.json:50), compress per client + FedAvg (aggregation.py:61-63, gar.py:44)
    gl = [np.random.default_rng(10 + i).standard_normal(431_080, dtype=np.float32) * np.float32(1e-3)
          for i in range(4)]
    cfg0 = {"compression_function": "top", "fraction_coordinate": 0.1}
    _, t0 = _timed(lambda: go.FedAvgOracle({}).aggregate(
        go.build_dense_G([co.compress(cfg0, x, argsort_kind=None) for x in gl], np.float32)))
    rows["configs0_4x431080_top0.1_round"] = {"ms": round(1e3 * t0, 1),
                                              "GBps": round(4 * 4.0 * 431_080 / t0 / 1e9, 4)}
    G = np.stack([g * np.float32(0.5 ** i) for i in range(4)])
    _, t_avg4 = _timed(lambda: go.FedAvgOracle({}).aggregate(G))
    rows["fedavg_4x16M"] = {"ms": round(1e3 * t_avg4, 1), "GBps_of_G": round(G.nbytes / t_avg4 / 1e9, 4)}
    per_row = t_avg4 / 4                            # FedAvg cost per 16 M row
    extrap = {
        "configs1_1x16M_top0.1_s": round(t_top16, 2),
        "configs2_128x16M_top0.1_fedavg_s": round(128 * (t_top16 + per_row), 1),
        "configs3_per_gpu_128x128M_top0.1_fedavg_s": None,      # filled from the headline client
        "configs4_per_gpu_512x25.5M_top0.01_fedavg_s": round(512 * (t_top25 + per_row * n25 / n16), 1),
        "method": "clients x (one timed client + one row of the timed 4 x 16 M FedAvg, scaled by N)",
    }
    return {"rows": rows, "extrapolated": extrap, "per_row_fedavg_16M_s": per_row,
            "cores": 1, "kind": "port (the reference's NumPy calls; default argsort kind)"}


def _packet_equal(torch, p, q):
    """Byte equality of two packets on the device: every listed entry (idx, val), the slot
    counts, quarter offsets and header fields thresh / lower / n_entries / status."""
    if not (torch.equal(p.cnt, q.cnt) and torch.equal(p.qoff, q.qoff)):
        return False
    hp, hq = p.hdr.view(torch.int64)[:3], q.hdr.view(torch.int64)[:3]   # thresh, lower, n|k
    if not (torch.equal(hp, hq) and torch.equal(p.hdr[36:40], q.hdr[36:40])):  # + status
        return False
    pos = torch.arange(p.capacity, device=p.val.device)
    listed = (pos % 8192) < p.cnt.to(torch.int64)[pos // 8192]
    return bool(torch.equal(p.idx[listed], q.idx[listed])
                and torch.equal(p.val.view(torch.int32)[listed], q.val.view(torch.int32)[listed]))


def self_check(torch, codec, grads, pkts, k, redone=()):
    """Outside the timed region: clients 0 and 1 re-encoded ALONE (fc_topk_encode) give the
    batched packets byte for byte, and the same dense result (compression.py:31-37).  A packet
    the last step re-encoded exactly (``redone``) lists no bracket slack, so only its dense
    result is compared."""
    ok = True
    for i in (0, 1):
        if i >= len(pkts):
            break
        single = codec.encode_top(grads[i], k)
        if i not in redone:
            ok = ok and _packet_equal(torch, single, pkts[i])
        a = codec.decode(single).view(torch.int32)
        b = codec.decode(pkts[i]).view(torch.int32)
        ok = ok and bool(torch.equal(a, b))
        del single, a, b
    if not ok:
        raise SystemExit("self-check failed: batched encode differs from a single-client encode")
    return ("ok: clients 0, 1 re-encoded singly: packets byte-equal to the batch's (entries, "
            "counts, quarter offsets, header) and dense results bit-identical")


def load_pmc(path):
    """HBM bytes per client of k_compact_mag1 from the committed rocprofv3 PMC summary
    (tools/pmc_round.sh: FETCH_SIZE / WRITE_SIZE at 128 clients per launch, calibrated on known
    byte counts of the same access shapes)."""
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d["hbm_bytes_per_launch"] / d.get("clients_per_launch", 1), os.path.relpath(path, ROOT)
    except (OSError, ValueError, KeyError):
        return None, None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(sys.argv[1:], args.gpus))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    if args.backend == "gloo":
        # rehearsal of the multi-rank path on fewer GPUs than ranks (ranks share devices; the
        # partial sums are staged through host memory, distributed.py); never the measurement
        local %= max(1, torch.cuda.device_count())
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    pg = init_pg(dist, args.backend, world, rank, device, args.force_pg)

    from openmsftl_amd import _lib as L
    if args.lib:
        L.load(os.path.abspath(args.lib))
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    from openmsftl_amd.distributed import ShardedFedAvg, fedavg_weights, packet_fold, shard_range

    M, n, f = args.clients, args.n, args.fraction
    k = kept_count(f, n)
    t_gen = time.perf_counter()
    grads = make_grads(M, n, rank, device, torch)
    torch.cuda.synchronize()
    log(f"[rank {rank}] generated {M} x {n:,} fp32 in {time.perf_counter() - t_gen:.1f} s")

    lib = L.load()
    hdrs = torch.empty((M, L.HDR_BYTES), dtype=torch.uint8, device=device)
    pkts = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, device, hdr=hdrs[i], k=k)
            for i in range(M)]
    # global FedAVG weights fl32(1/#clients) (gar.py:37-40); this rank owns rows
    # shard_range(M * world, world, rank) of G (distributed.py)
    w_all = fedavg_weights(M * world)
    rows = shard_range(M * world, world, rank)
    assert len(rows) == M
    views = codec.views_tensor(pkts, [float(x) for x in w_all[rows.start:rows.stop]], device)
    fold = packet_fold(pkts, views)
    jobs = codec.encode_jobs(grads, pkts)
    per_launch = 1 if args.no_batch else M          # clients per k_compact launch
    fedavg = ShardedFedAvg(mode="reduce", dst=0, always_collective=args.force_pg)
    # two aggregate buffers: step i's RCCL reduce (async, on RCCL's stream) runs under step
    # i+1's encodes; step i+2 waits for it before folding into the same buffer again
    accs = [torch.empty(n, dtype=torch.float32, device=device) for _ in range(2)]
    works = [None, None]
    nstep = [0]
    redo_total = [0]

    # packet statuses land in pinned host memory before the fold is queued: the host waits for
    # the encodes only, and queues the next step while the fold runs (a blocking read after
    # the fold left the GPU idle ~0.2 ms per step while Python launched the next one)
    status_host = torch.empty((M, 4), dtype=torch.uint8, pin_memory=True)
    encoded = torch.cuda.Event()

    pipelined = args.pipeline and not args.no_batch
    w_local = [float(x) for x in w_all[rows.start:rows.stop]]
    folded = lambda rows_, w_, out_, cont_: None    # noqa: E731 (this rank folded already)
    poke = [False]                                  # --force-retry-rank: mark the next step
    last_redo = set()                               # clients re-encoded exactly, last step

    def step():
        b = nstep[0] & 1
        nstep[0] += 1
        if works[b] is not None:
            works[b].wait()                         # stream-side wait for step i-2's reduce
        if pipelined:
            # each encode chain's packets are folded (k_fold_q) on its stream as soon as they
            # are encoded, the second fold continuing the first's partial sum in row order;
            # the statuses are copied once every chain is encoded (`ready`)
            ready = codec.encode_fold_batch(grads, k, w_local, accs[b], packets=pkts, jobs=jobs,
                                            views=views, streams=args.streams,
                                            status=(hdrs[:, 36:40], status_host))
        else:
            if args.no_batch:
                for i in range(M):
                    codec.encode_top(grads[i], k, packet=pkts[i], check=False)
            else:                                   # 4 launches for all M clients
                codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs, check=False,
                                       streams=args.streams)
            if poke[0]:                             # test only: a bracket "miss" on this rank
                hdrs[0, 36:40].copy_(torch.tensor([L.FC_STATUS_RETRY_EXACT, 0, 0, 0],
                                                  dtype=torch.uint8))
                poke[0] = False
            status_host.copy_(hdrs[:, 36:40], non_blocking=True)   # fc_packet_hdr.status
            encoded.record()
            ready = encoded
            # this rank's fold is queued before the host waits for the statuses: the host
            # queues the rest of the step while the fold runs
            fold(rows, w_local, accs[b], False)
        ready.synchronize()
        bad = status_host.view(torch.int32).view(-1)
        last_redo.clear()
        if bool((bad != 0).any()):                  # sampled bracket missed on THIS rank:
            last_redo.update(int(i) for i in torch.nonzero(bad).view(-1))
            redo_total[0] += codec.resolve(pkts)    # exact re-encode (stream-ordered after
            fold(rows, w_local, accs[b], False)     # the first fold) and fold again from +0
        # the ONE cross-rank collective of the step, issued after every local re-encode: each
        # rank issues exactly one reduce per step whatever its statuses were (rank-uniform)
        works[b] = fedavg.aggregate(folded, M * world, accs[b], weights=w_all, async_op=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with L.KernelTimer(L.FC_TIME_COMPACT | L.FC_TIME_DECODE | L.FC_TIME_ENGINE
                       | L.FC_TIME_SAMPLE) as kt:
        for s in range(args.steps):
            poke[0] = rank == args.force_retry_rank and s == args.steps - 1
            step()
        torch.cuda.synchronize()
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if pg:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=device if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = 1e3 * elapsed / args.steps
    for wk in works:                                # the last reduces land before any read
        if wk is not None:
            wk.wait()
    torch.cuda.synchronize()
    if args.dump_agg and rank == 0:
        import numpy as np
        np.save(args.dump_agg, accs[(nstep[0] - 1) & 1].cpu().numpy())
    if pg:                                          # exact re-encodes over all ranks
        t = torch.tensor([redo_total[0]], dtype=torch.int64,
                         device=device if args.backend == "nccl" else "cpu")
        dist.all_reduce(t)
        redo_total[0] = int(t.item())
    # the packets of the last timed step against single-client encodes, before anything reuses them
    checked = self_check(torch, codec, grads, pkts, k, last_redo)
    grad_bytes = 4.0 * n * M * world
    value = grad_bytes / (elapsed / args.steps) / 1e9

    # roofline of the dominant kernel (k_compact: the single streaming pass over g), HIP events
    # on the launch stream over the timed steps (one launch chain: per_launch clients per
    # k_compact_mag1 launch).  With --streams > 1 (sub-batches; a fold may run beside the next
    # sub-batch's compaction) the per-launch figure comes from extra one-chain passes instead.
    # In a rocprofv3 trace these are the k_compact_mag1 dispatches with grid.y == per_launch
    # (tools/rocpd_summary.py stats splits dispatches by grid).
    kt_roof = kt
    if args.roofline_steps > 0 and not args.no_batch and args.streams > 1:
        torch.cuda.synchronize()
        with L.KernelTimer(L.FC_TIME_COMPACT) as kt_roof:
            for _ in range(args.roofline_steps):
                codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs, check=False,
                                       streams=1)
            torch.cuda.synchronize()
    t_compact_us = kt_roof.avg_us("compact")
    # the encode pass reads 4N and writes the k entries, priced 8 B each
    alg_bytes = per_launch * (4.0 * n + ENTRY_BYTES * k)
    achieved = alg_bytes / (t_compact_us * 1e-6) / 1e9
    pmc, pmc_src = load_pmc(args.pmc)
    roofline = {"kernel": "fc::k_compact_mag1 (top-k encode pass, %d client(s) per launch)"
                          % per_launch, "bound": "hbm",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": int(pmc * per_launch) if pmc else None,
                "traffic_source": pmc_src,
                "alg_bytes_per_launch": int(alg_bytes), "avg_launch_us": round(t_compact_us, 2),
                "launches": kt_roof.launches.get("compact", 0),
                "measured": "one-stream encode passes after the timed steps"
                            if kt_roof is not kt else "timed steps"}
    breakdown = {c: {"avg_us": round(kt.avg_us(c), 2), "launches": kt.launches[c],
                     "ms_per_step": round(kt.ms[c] / args.steps, 3)}
                 for c in L.TIME_CLASSES if kt.launches.get(c)}
    breakdown["note"] = ("timed steps; %d sub-batches per step, encoded one after the other"
                         % args.streams if args.streams > 1 and not args.no_batch else "timed steps")

    # whole step against the HBM roofline (SURVEY §8(d) batched FedAvg with fused
    # decode-accumulate: M (4N + 16k) + 4N algorithmic bytes per GPU and step)
    step_alg = M * (4.0 * n + 2 * ENTRY_BYTES * k) + 4.0 * n
    step_gbps = step_alg * world / (elapsed / args.steps) / 1e9
    extra = {"per_step_kernel_time": breakdown, "exact_fallbacks": redo_total[0],
             "step_roofline": {"alg_bytes_per_gpu": int(step_alg),
                               "achieved_GBps": round(step_gbps, 1),
                               "frac": round(step_gbps / world / HBM_PEAK_GBPS, 4)}}
    extra["self_check"] = checked
    if args.tag is not None:
        extra["tag"] = args.tag
    extra["process_group"] = ({"backend": args.backend, "world": world,
                               "collective_per_step": "reduce (async)"} if pg else None)
    if rank == 0 and not args.no_single:
        extra["single_gradient"] = single_gradient(torch, codec, grads[0], k, n, graph=not pg)
        extra["qsgd_single_gradient"] = qsgd_single(torch, codec, grads[0], n)

    # the other named single-GPU sizes (BASELINE configs[1], configs[2]) as extras, after the
    # headline workload's buffers are released
    del grads, pkts, jobs, views, fold, hdrs
    torch.cuda.empty_cache()
    if world == 1 and rank == 0 and not args.no_single:
        extra["configs_1_2"] = small_configs(torch, codec, L, device, f, graph=not pg)
    if world == 1 and rank == 0 and not args.no_matrix:
        extra["codec_matrix"] = codec_matrix(torch, codec, L, device)

    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(n, f)
        mat = cpu_matrix()
        t_client = 4.0 * n / (cpu["value"] * 1e9)
        mat["extrapolated"]["configs3_per_gpu_128x128M_top0.1_fedavg_s"] = round(
            M * (t_client + mat.pop("per_row_fedavg_16M_s") * n / 16_777_216), 1)
        extra["cpu_baseline_matrix"] = mat

    if rank == 0:
        line = {
            "metric": "device-resident grad encode+decode GB/s at 1/2/4/8 MI355X; % HBM roofline",
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (device torch.randn, per-client log-uniform scale)",
            "config": {"workload": "BASELINE configs[3] per-GPU shard: clients x 134,217,728-fp32 "
                                   "gradients, top-k f=0.1 encode -> FedAVG decode-accumulate"
                                   + (" -> RCCL reduce" if world > 1 else ""),
                       "clients_per_gpu": M, "n": n, "codec": "top", "fraction": f, "k": k,
                       "parallelism": f"dp{world}",
                       **({"rehearsal": "gloo, ranks sharing GPUs"} if args.backend == "gloo" else {})},
            "roofline": roofline, "cpu_baseline": cpu, "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if pg:
        dist.destroy_process_group()


def single_gradient(torch, codec, g, k, n, iters=None, graph=True):
    """North-star probe: encode+decode of ONE 128 M gradient (packet -> dense), HBM fraction
    of the algorithmic 8N + 16k bytes.  Host wall clock over ``iters``
    back-to-back calls: 20 at 128 M, 200 below 64 M elements, so that the first launch's host
    latency and the final synchronise (~30-50 us once per loop) stay below 1 % of the loop.
    The round trip is fc_topk_encode_decode (the packet of fc_topk_encode, then its dense
    decode, the resolve's gather and finish done inside the decode launch); ``two_calls`` is
    the same packet and q from fc_topk_encode (+ k_resolve) and fc_decode_dense."""
    if iters is None:
        iters = 20 if n >= (1 << 26) else 200
    out = torch.empty_like(g)
    pkt = codec.encode_top(g, k)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        dt_ = (time.perf_counter() - t0) / iters
        codec.resolve([pkt])
        return dt_

    roundtrip = lambda: codec.encode_decode_top(g, k, packet=pkt, out=out, check=False)   # noqa: E731
    two_calls = lambda: (codec.encode_top(g, k, packet=pkt, check=False),                 # noqa: E731
                         codec.decode(pkt, out=out))
    dense = lambda: codec.compress_top_dense(g, k, out=out, packet=pkt, check=False)     # noqa: E731
    dt = timed(roundtrip)
    dt_2 = timed(two_calls)
    # the same result through fc_topk_encode_dense (compaction streams q, fix-up of the slack)
    dt_d = timed(dense)
    moved = dense_moved_bytes(n, pkt)
    codec.resolve([pkt])
    alg = 8.0 * n + 2 * ENTRY_BYTES * k
    frac = lambda t: round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)                               # noqa: E731
    res = {"n": n, "k": k, "us_per_encode_decode": round(dt * 1e6, 1),
           "grad_GBps": round(4.0 * n / dt / 1e9, 1),
           "alg_GBps": round(alg / dt / 1e9, 1),
           "hbm_frac": frac(dt),
           "path": "fc_topk_encode_decode (k_fused_mag<false> -> k_beta -> k_decode_res)",
           "two_calls": {"us": round(dt_2 * 1e6, 1), "hbm_frac": frac(dt_2),
                         "path": "fc_topk_encode (k_fused_mag<false> -> k_resolve) + fc_decode_dense"},
           "fused_dense": {"us": round(dt_d * 1e6, 1),
                           "alg_GBps": round(alg / dt_d / 1e9, 1),
                           "hbm_frac": frac(dt_d),
                           "moved_bytes": int(moved),
                           "hbm_frac_moved": round(moved / dt_d / 1e9 / HBM_PEAK_GBPS, 4)}}
    if not graph:                      # (N > 1: no graph capture beside a live process group)
        return res
    # the same calls, `iters` of them captured in one HIP graph (codec.GraphedCalls) and
    # replayed: no host work per call, cheaper kernel boundaries; same kernels, same buffers
    dt_g = _graph_us(torch, codec, roundtrip, iters) * 1e-6
    codec.resolve([pkt])
    dt_dg = _graph_us(torch, codec, dense, iters) * 1e-6
    codec.resolve([pkt])
    res["graph"] = {"us_per_encode_decode": round(dt_g * 1e6, 1), "hbm_frac": frac(dt_g)}
    res["fused_dense"]["graph"] = {"us": round(dt_dg * 1e6, 1), "hbm_frac": frac(dt_dg),
                                   "hbm_frac_moved": round(moved / dt_dg / 1e9 / HBM_PEAK_GBPS, 4)}
    return res


def _graph_us(torch, codec, fn, iters=20, reps=3):
    """Per-call µs of `iters` calls of fn captured in one HIP graph, best of `reps` replays."""
    gc = codec.GraphedCalls(lambda: [fn() for _ in range(iters)])
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gc.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters * 1e6
        best = dt if best is None else min(best, dt)
    del gc
    return best


def dense_moved_bytes(n, pkt):
    """Bytes the drop-in dense top-k (fc_topk_encode_dense) actually moves, as opposed to
    SURVEY §8(d)'s task bytes 8N + 16k (an encode AND a packet decode): it reads g (4N), writes
    q (4N) and writes + re-reads the bracket's candidates (8 B each, the header's n_cand); the
    sample (<= 8 MB) is left out."""
    return 8.0 * n + 16.0 * pkt.header().n_cand


def small_configs(torch, codec, L, device, f, n=16_777_216, M=128, steps=100, graph=True,
                  slab_packets=False, streams=1, pipeline=False):
    """BASELINE configs[1] (one 16 M gradient: encode + dense decode) and configs[2] (128
    clients x 16 M: batched encode + on-device FedAVG fold), device-resident, same codec."""
    from openmsftl_amd.compression import kept_count
    k = kept_count(f, n)
    grads = make_grads(M, n, 0, device, torch)
    one = single_gradient(torch, codec, grads[0], k, n, graph=graph)
    # slab_packets: the packets as rows of per-field slabs (codec.Packet.alloc_batch); its
    # compaction is 2-3 % faster at 16 M, but the whole configs[2] step is not
    # (profiles/r06_c2_slab_packets_ab.jsonl: 2.223-2.233 vs 2.220-2.230 ms), so off by default
    pkts = codec.Packet.alloc_batch(n, M, L.FC_FMT_IDXVAL, device, k=k) if slab_packets else \
        [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, device, k=k) for _ in range(M)]
    w = [1.0 / M] * M
    jobs = codec.encode_jobs(grads, pkts)
    views = codec.views_tensor(pkts, w, device)
    acc = torch.empty(n, dtype=torch.float32, device=device)

    def step():
        if pipeline:                    # each sub-batch folded on its stream once encoded
            codec.encode_fold_batch(grads, k, w, acc, packets=pkts, jobs=jobs, views=views,
                                    streams=streams)
            return
        codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs, check=False, streams=streams)
        codec.decode_accumulate(pkts, w, out=acc, views=views)

    for _ in range(10):                 # 2.4 ms steps: warm enough that clocks have settled
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    redo = codec.resolve(pkts)
    alg = M * (4.0 * n + 2 * ENTRY_BYTES * k) + 4.0 * n
    return {"config1_single_16M": one,
            "config2_128x16M": {"clients": M, "n": n, "k": k, "ms_per_step": round(dt * 1e3, 3),
                                "grad_GBps": round(4.0 * n * M / dt / 1e9, 1),
                                "alg_GBps": round(alg / dt / 1e9, 1),
                                "hbm_frac": round(alg / dt / 1e9 / HBM_PEAK_GBPS, 4),
                                "exact_fallbacks": redo, "streams": streams, "pipeline": pipeline}}


def _time_us(torch, fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def _row(us, alg, **kw):
    return {"us": round(us, 1), "alg_bytes": int(alg), "alg_GBps": round(alg / us / 1e3, 1),
            "hbm_frac": round(alg / us / 1e3 / HBM_PEAK_GBPS, 4), **kw}


def codec_matrix(torch, codec, L, device, n16=16_777_216, n25=25_557_032):
    """SURVEY.md §8(d)'s other codec settings, device-resident, encode + decode of one gradient
    (the `roofline` algorithmic bytes of §8(d): top/rand packets 8N + 16k; dropout bitmap
    packets 2 (4N + N/8 + 4 nnz); the dense drop-in results read 4N and write the dense q;
    'full' FedAVG M 4N + 4N).  Host RNG draws (np.random, parity mode) happen before timing:
    only their device work (mask -> packet -> dense) is timed."""
    import numpy as np
    from openmsftl_amd.compression import bitmask_words, kept_count
    rows = {}
    gen = torch.Generator(device=device)
    g16 = torch.randn(n16, device=device, generator=gen.manual_seed(5)).mul_(1e-2)
    out16 = torch.empty_like(g16)
    # top f = 0.01 (configs[4]'s codec) at 16 M and 25.5 M: packet encode + decode, and the
    # drop-in dense path (k_fused_mag<true> + k_resolve)
    for name, n in (("top_f0.01_16M", n16), ("top_f0.01_25.5M", n25)):
        g = g16 if n == n16 else torch.randn(n, device=device, generator=gen.manual_seed(6)).mul_(1e-2)
        out = out16 if n == n16 else torch.empty_like(g)
        k = kept_count(0.01, n)
        pkt = codec.encode_top(g, k)
        us = _time_us(torch, lambda: codec.encode_decode_top(g, k, packet=pkt, out=out, check=False))
        assert codec.resolve([pkt]) == 0
        usd = _time_us(torch, lambda: codec.compress_top_dense(g, k, out=out, packet=pkt, check=False))
        moved = dense_moved_bytes(n, pkt)
        assert codec.resolve([pkt]) == 0
        alg = 8.0 * n + 16.0 * k
        rows[name] = _row(us, alg, n=n, k=k, path="fc_topk_encode_decode (packet + dense decode)",
                          dense=_row(usd, alg, path="fc_topk_encode_dense", moved_bytes=int(moved),
                                     hbm_frac_moved=round(moved / usd / 1e3 / HBM_PEAK_GBPS, 4)))
    # rand f = 0.1 at 16 M: native Philox keys (fc_topk_encode PHILOX) and parity mode (the
    # host permutation as a bit mask -> fc_mask_encode idx/val -> decode)
    k = kept_count(0.1, n16)
    pkt = codec.encode_top(g16, k, key_mode=L.FC_KEY_PHILOX, seed=3, offset=1)
    us = _time_us(torch, lambda: (codec.encode_top(g16, k, key_mode=L.FC_KEY_PHILOX, seed=3, offset=1,
                                                   packet=pkt, check=False),
                                  codec.decode(pkt, out=out16)))
    assert codec.resolve([pkt]) == 0
    rows["rand_f0.1_16M_philox"] = _row(us, 8.0 * n16 + 16.0 * k, n=n16, k=k,
                                        path="fc_topk_encode(PHILOX) + fc_decode_dense")
    idx = np.random.default_rng(1).permutation(n16)[:k]
    mask = torch.from_numpy(bitmask_words(idx, n16, False).view(np.int32)).to(device)
    pm = codec.encode_mask(g16, L.FC_CODEC_RAND, mask_bits=mask, fmt=L.FC_FMT_IDXVAL)
    us = _time_us(torch, lambda: (codec.encode_mask(g16, L.FC_CODEC_RAND, mask_bits=mask,
                                                    fmt=L.FC_FMT_IDXVAL, packet=pm),
                                  codec.decode(pm, out=out16)))
    rows["rand_f0.1_16M_hostmask"] = _row(us, 8.0 * n16 + 16.0 * k + n16 / 8.0, n=n16, k=k,
                                          path="fc_mask_encode(RAND, idx/val) + fc_decode_dense; "
                                               "alg + N/8 mask bytes")
    # dropout p = 0.1 (client_config.json:49), both codecs, both mask sources: bitmap packet
    # encode + dense decode, and the drop-in dense float64 q (fc_mask_dense_f32)
    hm = np.random.default_rng(2).binomial(1, 0.1, n16)
    mb = torch.from_numpy(bitmask_words(hm, n16, True).view(np.int32)).to(device)
    out64 = torch.empty(n16, dtype=torch.float64, device=device)
    for cname, cid in (("dropout-biased", L.FC_CODEC_DROPOUT_BIASED),
                       ("dropout-unbiased", L.FC_CODEC_DROPOUT_UNBIASED)):
        for src, kw in (("philox", {"seed": 4, "offset": 2}), ("hostmask", {"mask_bits": mb})):
            pb = codec.encode_mask(g16, cid, p=0.1, **kw)
            us = _time_us(torch, lambda: (codec.encode_mask(g16, cid, p=0.1, packet=pb, **kw),
                                          codec.decode(pb, out=out16)))
            nnz = int(pb.cnt.sum().item())
            alg = 2.0 * (4.0 * n16 + n16 / 8.0 + 4.0 * nnz)
            usd = _time_us(torch, lambda: codec.mask_dense_f64(g16, cid, p=0.1, out=out64, **kw))
            algd = 4.0 * n16 + 8.0 * n16 + (n16 / 8.0 if src == "hostmask" else 0.0)
            rows[f"{cname}_p0.1_16M_{src}"] = _row(
                us, alg, n=n16, nnz=nnz, path="fc_mask_encode(bitmap) + fc_decode_dense",
                dense_f64=_row(usd, algd, path="fc_mask_dense_f32 (drop-in float64 q)"))
    # 'full' (compression.py:27-29 returns g itself): FedAVG of 128 x 16 M dense rows (k_wsum)
    M = 128
    G = torch.randn((M, n16), device=device, generator=gen.manual_seed(7))
    w = torch.full((M,), 1.0 / M, dtype=torch.float32)
    acc = torch.empty(n16, dtype=torch.float32, device=device)
    rows_l = list(G.unbind(0))
    us = _time_us(torch, lambda: codec.weighted_sum_dense(rows_l, w, out=acc), iters=10)
    rows["full_fedavg_128x16M"] = _row(us, M * 4.0 * n16 + 4.0 * n16, clients=M, n=n16,
                                       path="fc_weighted_sum_dense (k_wsum)")
    del G, rows_l
    # float64 gradient, top f = 0.1 at 16 M (RandomGaussian noise_scale 0 hands float64 over)
    g64 = g16.double()
    o64 = torch.empty_like(g64)
    k = kept_count(0.1, n16)
    us = _time_us(torch, lambda: codec.compress_top_dense_f64(g64, k, out=o64, check=False),
                  iters=10)
    redo = codec.resolve_f64(o64)
    use = _time_us(torch, lambda: codec.compress_top_dense_f64(g64, k, out=o64, exact=True),
                   iters=5)
    rows["top_f0.1_16M_fp64"] = _row(us, 16.0 * n16, n=n16, k=k, exact_fallbacks=redo,
                                     path="fc_topk_dense_f64_sampled (sampled bracket on the "
                                          "high 31 key bits, one streaming pass, exact select "
                                          "among the candidates); alg = read 8N + write 8N",
                                     exact_engine=_row(use, 16.0 * n16,
                                                       path="fc_topk_dense_f64 (exact radix "
                                                            "select, <= 8 passes of 8N)"))
    torch.cuda.empty_cache()
    return rows


def qsgd_single(torch, codec, g, n, bits=2, iters=20):
    """The opt-in QSGD codec (compression.py:62-74) on one 128 M gradient: encode (norm pass +
    quantise pass, 8N read + N W/8 written) then dense decode (N W/8 read + 4N written)."""
    pkt = codec.encode_qsgd(g, bits)
    out = torch.empty_like(g)
    for _ in range(3):
        codec.encode_qsgd(g, bits, packet=pkt)
        codec.decode_qsgd(pkt, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        codec.encode_qsgd(g, bits, packet=pkt)
        codec.decode_qsgd(pkt, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    wbytes = 4.0 if bits <= 2 else 8.0 if bits <= 6 else 16.0
    alg = 8.0 * n + n * wbytes / 8.0 + n * wbytes / 8.0 + 4.0 * n
    return {"n": n, "bits": bits, "us_per_encode_decode": round(dt * 1e6, 1),
            "alg_GBps": round(alg / dt / 1e9, 1), "hbm_frac": round(alg / dt / 1e9 / HBM_PEAK_GBPS, 4)}


if __name__ == "__main__":
    main()
