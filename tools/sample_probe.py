"""Per-kernel HIP-event timing of the encode's small launches (k_sample1, k_resolve) on one
gradient, for A/B of diagnostic builds (FC_SAMPLE_ABLATE / FC_RESOLVE_ABLATE variants).

    python tools/sample_probe.py [--lib tools/variants/lib_X.so] [--n 134217728] [--dense]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--n", type=int, default=134_217_728)
    ap.add_argument("--f", type=float, default=0.1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dense", action="store_true")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    if args.lib:
        L.load(os.path.abspath(args.lib))
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    n, k = args.n, kept_count(args.f, args.n)
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    out = torch.empty_like(g)
    pkt = codec.encode_top(g, k)
    for _ in range(3):
        if args.dense:
            codec.compress_top_dense(g, k, out=out, packet=pkt, check=False)
        else:
            codec.encode_top(g, k, packet=pkt, check=False)
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for _ in range(args.iters):
        if args.dense:
            codec.compress_top_dense(g, k, out=out, packet=pkt, check=False)
        else:
            codec.encode_top(g, k, packet=pkt, check=False)
    torch.cuda.synchronize()
    wall_us = (time.perf_counter() - t0) / args.iters * 1e6
    with L.KernelTimer() as kt:
        for _ in range(args.iters):
            if args.dense:
                codec.compress_top_dense(g, k, out=out, packet=pkt, check=False)
            else:
                codec.encode_top(g, k, packet=pkt, check=False)
        torch.cuda.synchronize()
    res = {c: round(kt.avg_us(c), 2) for c in L.TIME_CLASSES if kt.launches.get(c)}
    res["wall_us_per_call"] = round(wall_us, 1)
    print(json.dumps({"tag": args.tag, "n": n, "dense": args.dense, "avg_us": res}), flush=True)


if __name__ == "__main__":
    main()
