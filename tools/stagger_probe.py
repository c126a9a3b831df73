"""Does the HBM placement of the client gradients change the batched encode's bandwidth?
Client c's gradient is a view at c * (n + pad) floats into one buffer (pad = 0: rows packed at
a power-of-two stride), against M separate allocations (bench.make_grads before round 5's slab).
    python tools/stagger_probe.py [--n 16777216] [--clients 128] [--pads 0,64,1024,2112]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16_777_216)
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--pads", default="0,64,1024,2112")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import torch
    from openmsftl_amd import codec
    from openmsftl_amd import _lib as L
    from openmsftl_amd.compression import kept_count
    import bench
    dev = torch.device("cuda", 0)
    M, n = args.clients, args.n
    k = kept_count(0.1, n)
    src = [g.clone() for g in bench.make_grads(M, n, 0, dev, torch)]   # M separate allocations
    torch.cuda.empty_cache()
    pkts = None
    res = {"tag": args.tag, "n": n, "clients": M}

    def run(grads, name):
        nonlocal pkts
        if pkts is None:
            pkts = codec.encode_top_batch(grads, k)
        jobs = codec.encode_jobs(grads, pkts)
        for _ in range(3):
            codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs, check=False)
        torch.cuda.synchronize()
        with L.KernelTimer() as kt:
            for _ in range(args.iters):
                codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs, check=False)
            torch.cuda.synchronize()
        us = kt.avg_us("compact")
        res[name] = {"compact_us": round(us, 1),
                     "frac": round(M * (4.0 * n + 8.0 * k) / us / 8e6, 4)}

    run(src, "separate")
    for pad in [int(p) for p in args.pads.split(",")]:
        stride = n + pad
        buf = torch.empty(M * stride, dtype=torch.float32, device=dev)
        grads = []
        for c in range(M):
            v = buf[c * stride: c * stride + n]
            v.copy_(src[c])
            grads.append(v)
        run(grads, f"pad{pad}")
        del grads, buf
        torch.cuda.empty_cache()
    run(src, "separate_again")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
