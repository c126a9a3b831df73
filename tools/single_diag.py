"""Single-gradient step diagnosis: host enqueue time vs GPU (event) time per iteration for the
packet round trip (encode_top + decode) and the drop-in dense path (compress_top_dense), at
128 M and 16 M: is bench.single_gradient host-bound on a box?
    python tools/single_diag.py [--iters 50] [--reps 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--n", type=int, default=0, help="one length only (default 128 M and 16 M)")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    if args.lib:
        L.load(os.path.abspath(args.lib))
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    summary = {}
    for n in ((args.n,) if args.n else (134_217_728, 16_777_216)):
        g = torch.randn(n, device=dev, generator=gen.manual_seed(1)).mul_(1e-2)
        k = kept_count(0.1, n)
        out = torch.empty_like(g)
        pkt = codec.encode_top(g, k)
        fns = {"packet": lambda: (codec.encode_top(g, k, packet=pkt, check=False),
                                  codec.decode(pkt, out=out)),
               "encode_only": lambda: codec.encode_top(g, k, packet=pkt, check=False),
               "dense": lambda: codec.compress_top_dense(g, k, out=out, packet=pkt, check=False)}
        for rep in range(args.reps):
            for name, fn in fns.items():
                for _ in range(5):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record()
                for _ in range(args.iters):
                    fn()
                t1 = time.perf_counter()
                e1.record()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                ev = round(e0.elapsed_time(e1) / args.iters * 1e3, 1)
                summary.setdefault(f"{name}_{n >> 20}M_us", []).append(ev)
                print(json.dumps({"n": n, "path": name, "rep": rep,
                                  "host_enqueue_us": round((t1 - t0) / args.iters * 1e6, 1),
                                  "wall_us": round((t2 - t0) / args.iters * 1e6, 1),
                                  "event_us": round(e0.elapsed_time(e1) / args.iters * 1e3, 1)}),
                      flush=True)
        del g, out, pkt
    print(json.dumps({"tag": args.tag, **{k: min(v) for k, v in summary.items()}}), flush=True)


if __name__ == "__main__":
    main()
