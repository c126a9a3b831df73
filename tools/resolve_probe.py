"""Encode-latency probe for A/B builds (tools/ab.py): the paths whose resolve / sample kernels
changed between builds, each timed with HIP events over `--iters` back-to-back calls (best of
`--reps`), plus the resolve-, compaction- and decode-class kernel times (fc_timing) per call.

    python tools/resolve_probe.py [--lib PATH] [--tag T] [--iters 50] [--reps 3]

Paths: configs[2] step (128 x 16 M batched encode + fold), one 16 M and one 128 M gradient
through the drop-in dense encode and the packet encode (+ dense decode), 64 x 128 M batched
encode, fp64 sampled top-k at 16 M.  One JSON line with every figure (us / ms)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tag", default="")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="comma list of path names")
    args = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    if args.lib:
        L.load(os.path.abspath(args.lib))
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    import bench
    dev = torch.device("cuda", 0)
    res = {"tag": args.tag}
    only = set(args.only.split(",")) if args.only else None

    def timed(name, fn, iters=args.iters):
        if only is not None and name not in only:
            return
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        best, best_res, best_k = None, None, None
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with L.KernelTimer(L.FC_TIME_ENGINE | L.FC_TIME_COMPACT | L.FC_TIME_DECODE) as kt:
                e0.record()
                for _ in range(iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / iters * 1e3
            if best is None or us < best:
                best = us
                best_res = kt.ms.get("engine", 0.0) / iters * 1e3
                best_k = {c: kt.ms.get(c, 0.0) / iters * 1e3 for c in ("compact", "decode")}
        res[name + "_us"] = round(best, 2)
        res[name + "_resolve_us"] = round(best_res, 2)
        for c, v in best_k.items():
            if v:
                res[f"{name}_{c}_us"] = round(v, 2)

    gen = torch.Generator(device=dev)
    for n in (16_777_216, 134_217_728):
        g = torch.randn(n, device=dev, generator=gen.manual_seed(1)).mul_(1e-2)
        k = kept_count(0.1, n)
        out = torch.empty_like(g)
        pkt = codec.encode_top(g, k)
        tag = f"{n >> 20}M"
        timed(f"dense_{tag}", lambda: codec.compress_top_dense(g, k, out=out, packet=pkt, check=False))
        timed(f"packet_enc_{tag}", lambda: codec.encode_top(g, k, packet=pkt, check=False))
        timed(f"packet_rt_{tag}", lambda: (codec.encode_top(g, k, packet=pkt, check=False),
                                           codec.decode(pkt, out=out)))
        del g, out, pkt
    torch.cuda.empty_cache()
    # configs[2]: 128 x 16 M batched encode + fold (the bench's step)
    n, M = 16_777_216, 128
    k = kept_count(0.1, n)
    grads = bench.make_grads(M, n, 0, dev, torch)
    pkts = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k) for _ in range(M)]
    w = [1.0 / M] * M
    jobs = codec.encode_jobs(grads, pkts)
    views = codec.views_tensor(pkts, w, dev)
    acc = torch.empty(n, dtype=torch.float32, device=dev)

    def c2():
        codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs, check=False)
        codec.decode_accumulate(pkts, w, out=acc, views=views)
    timed("configs2_step", c2, iters=20)
    bad = sum(h.status != 0 for h in codec.headers(pkts))
    res["configs2_nonok"] = int(bad)
    del grads, pkts, jobs, views, acc
    torch.cuda.empty_cache()
    # 64 x 128 M batched encode (half the headline launch)
    if only is None or "batch64x128M" in only:
        n, M = 134_217_728, 64
        k = kept_count(0.1, n)
        grads = bench.make_grads(M, n, 0, dev, torch)
        pkts = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k) for _ in range(M)]
        jobs = codec.encode_jobs(grads, pkts)
        timed("batch64x128M", lambda: codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs,
                                                            check=False), iters=5)
        del grads, pkts, jobs
        torch.cuda.empty_cache()
    # fp64 sampled top-k, 16 M
    n = 16_777_216
    g64 = torch.randn(n, device=dev, dtype=torch.float64, generator=gen.manual_seed(3))
    o64 = torch.empty_like(g64)
    k = kept_count(0.1, n)
    timed("f64_16M", lambda: codec.compress_top_dense_f64(g64, k, out=o64, check=False))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
