"""Host-resident FedAVG from pageable NumPy gradients (the drop-in Aggregator's input): GB/s of
client gradients through HostFedAvg for several staging set-ups (copy threads, staging buffers).
    python tools/agg_probe.py [--clients 32] [--n 25557032] [--threads 4,8,16] [--stages 2,3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--n", type=int, default=25_557_032)
    ap.add_argument("--f", type=float, default=0.01)
    ap.add_argument("--threads", default="4,8,16")
    ap.add_argument("--stages", default="2,3")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import numpy as np
    import torch
    from openmsftl_amd.compression import kept_count
    from openmsftl_amd.pipeline import HostFedAvg
    n, M = args.n, args.clients
    k = kept_count(args.f, n)
    rng = np.random.default_rng(0)
    host = [(rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** rng.uniform(-4, -1)))
            for _ in range(M)]
    gb = 4.0 * n * M / 1e9
    res = {}
    ref = None
    for st in [int(x) for x in args.stages.split(",")]:
        for th in [int(x) for x in args.threads.split(",")]:
            pipe = HostFedAvg(n, k, group=64, stage=st, copy_threads=th)
            best = None
            for _ in range(args.reps + 1):
                t0 = time.perf_counter()
                out = pipe.run(host, M)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            got = out.numpy().tobytes()
            if ref is None:
                ref = got
            assert got == ref, "staging set-ups must give the same aggregate"
            res[f"stage{st}_threads{th}_GBps"] = round(gb / best, 2)
            del pipe
            torch.cuda.empty_cache()
    print(json.dumps({"clients": M, "n": n, "k": k, **res}), flush=True)


if __name__ == "__main__":
    main()
