"""Kernel-boundary cost of the lone encodes: per-call time of back-to-back stream launches
against the same calls captured in one HIP graph (torch.cuda.CUDAGraph) and replayed.
    python tools/graph_probe.py [--n 16777216] [--calls 20] [--reps 5]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16_777_216)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tag", default="")
    ap.add_argument("--no-order-events", action="store_true",
                    help="A/B only: replace codec._fused_encode's per-call event with nothing")
    args = ap.parse_args()
    import contextlib
    import torch
    from openmsftl_amd import codec
    if args.no_order_events:
        codec._fused_encode = contextlib.contextmanager(lambda dev: (yield))
    from openmsftl_amd.compression import kept_count
    n, k = args.n, kept_count(0.1, args.n)
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 1e-2
    out = torch.empty_like(g)
    pkt = codec.encode_top(g, k)
    res = {"tag": args.tag, "n": n}

    def eager_dense():
        codec.compress_top_dense(g, k, out=out, packet=pkt, check=False)

    def eager_rt():
        codec.encode_top(g, k, packet=pkt, check=False)
        codec.decode(pkt, out=out)

    s = torch.cuda.Stream()
    for name, fn in (("dense", eager_dense), ("packet_rt", eager_rt)):
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record()
                for _ in range(args.calls):
                    fn()
                e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / args.calls * 1e3
            best = us if best is None else min(best, us)
        res[name + "_eager_us"] = round(best, 2)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s):
                for _ in range(args.calls):
                    fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record()
                graph.replay()
                e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / args.calls * 1e3
            best = us if best is None else min(best, us)
        res[name + "_graph_us"] = round(best, 2)
        del graph
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
