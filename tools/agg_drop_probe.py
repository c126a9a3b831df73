"""The drop-in Aggregator NumPy -> NumPy (driver.py's path): GB/s of client gradients for
'top' and 'full' at the configs[4] row size, best / median of --reps timed calls after one
warm call (which allocates the ring and the packets).
    python tools/agg_drop_probe.py [--clients 70] [--n 25557032] [--reps 4] [--codecs top,full]"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--pkg" in sys.argv:                  # another build's package (A/B of the host pipeline)
    sys.path.insert(0, os.path.abspath(sys.argv[sys.argv.index("--pkg") + 1]))


class _Client:
    def __init__(self, i, g, C):
        self.client_id, self.grad, self.C = i, g, C


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=70)
    ap.add_argument("--n", type=int, default=25_557_032)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--codecs", default="top,full")
    ap.add_argument("--tag", default="")
    ap.add_argument("--lib", default=None)
    ap.add_argument("--pkg", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch
    from openmsftl_amd import _lib as L
    if args.lib:
        L.load(os.path.abspath(args.lib))
    from openmsftl_amd import Compression
    from openmsftl_amd.aggregation import Aggregator
    rng = np.random.default_rng(0)
    host = [(rng.standard_normal(args.n, dtype=np.float32) * np.float32(10.0 ** rng.uniform(-4, -1)))
            for _ in range(args.clients)]
    gb = 4.0 * args.n * args.clients / 1e9
    res = {"tag": args.tag, "clients": args.clients, "n": args.n}
    for name in args.codecs.split(","):
        C = Compression({"compression_function": name, "fraction_coordinate": 0.01})
        clients = [_Client(i, g, C) for i, g in enumerate(host)]
        agg = Aggregator({"aggregation_scheme": "fed_avg"})
        agg.aggregate_grads(clients)
        ts = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            agg.aggregate_grads(clients)
            ts.append(time.perf_counter() - t0)
        res[name] = {"best_GBps": round(gb / min(ts), 2), "median_GBps": round(gb / statistics.median(ts), 2),
                     "path": agg.agg_path}
        del agg
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
