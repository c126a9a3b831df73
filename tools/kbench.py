"""Kernel-level timing of one codec configuration (HIP events per kernel class).

    python tools/kbench.py [--lib path/to/libfedcodec.so] [--n 134217728] [--f 0.1]

Used to A/B build variants of libfedcodec.so in one process each (same device, same data).
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
    ap.add_argument("--tag", default="")
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--dec", type=int, default=0, help="FedAVG fold of this many DISTINCT packets")
    args = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    if args.lib:
        L.load(os.path.abspath(args.lib))
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    n, k = args.n, kept_count(args.f, args.n)
    if args.dec:                       # k_decode_sparse<true> over distinct packets (no cache reuse)
        M = args.dec
        gs = [torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(s))
              for s in range(M)]
        pk = codec.encode_top_batch(gs, k, streams=1)
        codec.resolve(pk)
        del gs
        w = [1.0 / M] * M
        views = codec.views_tensor(pk, w, torch.device("cuda"))
        acc = torch.empty(n, device="cuda")
        codec.decode_accumulate(pk, w, out=acc, views=views)
        torch.cuda.synchronize()
        with L.KernelTimer() as kt:
            for _ in range(args.iters):
                codec.decode_accumulate(pk, w, out=acc, views=views)
            torch.cuda.synchronize()
        us = kt.ms["decode"] * 1e3 / (args.iters * M)
        ent = sum(int(p.n_entries) for p in pk) / M if hasattr(pk[0], "n_entries") else k
        print(json.dumps({"tag": args.tag, "n": n, "k": k, "dec_packets": M,
                          "dec_us_per_pkt": round(us, 2),
                          "dec_GBps_8k": round(8.0 * k / (us * 1e-6) / 1e9, 1),
                          "acc_sum": float(acc.double().sum())}), flush=True)
        return
    if args.batch:                     # batched k_compact: clients per launch = --batch
        gs = [torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(s))
              for s in range(args.batch)]
        pk = codec.encode_top_batch(gs, k, streams=1)
        jobs = codec.encode_jobs(gs, pk)
        torch.cuda.synchronize()
        with L.KernelTimer() as kt:
            for _ in range(args.iters):
                codec.encode_top_batch(gs, k, packets=pk, jobs=jobs, check=False, streams=1)
            torch.cuda.synchronize()
        codec.resolve(pk)
        hs = codec.headers(pk)
        cnt = torch.stack([p.cnt for p in pk]).double()
        res = {c: round(kt.avg_us(c), 2) for c in L.TIME_CLASSES if kt.launches.get(c)}
        res["entries_over_k"] = round(sum(h.n_entries for h in hs) / (len(hs) * k), 4)
        res["entries_per_chunk_sd"] = round(float(cnt.std(dim=1).mean()), 1)
        res["compact_GBps_alg"] = round(args.batch * (4.0 * n + 8.0 * k)
                                        / (res["compact"] * 1e-6) / 1e9, 1)
        print(json.dumps({"tag": args.tag, "n": n, "k": k, "batch": args.batch, "avg_us": res}),
              flush=True)
        return
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    pkt = codec.encode_top(g, k)
    out = torch.empty_like(g)
    for _ in range(3):
        codec.encode_top(g, k, packet=pkt, check=False)
        codec.decode(pkt, out=out)
    torch.cuda.synchronize()
    with L.KernelTimer() as kt:
        for _ in range(args.iters):
            codec.encode_top(g, k, packet=pkt, check=False)
            codec.decode(pkt, out=out)
        torch.cuda.synchronize()
    codec.resolve([pkt])
    res = {c: round(kt.avg_us(c), 2) for c in L.TIME_CLASSES if kt.launches.get(c)}
    res["compact_GBps_alg"] = round((4.0 * n + 8.0 * k) / (res["compact"] * 1e-6) / 1e9, 1)
    # FedAVG decode-accumulate of M packets (the same packet M times): per-packet cost
    M = args.m
    pk = [pkt] * M
    views = codec.views_tensor(pk, [1.0 / M] * M, g.device)
    acc = torch.empty_like(g)
    codec.decode_accumulate(pk, [1.0 / M] * M, out=acc, views=views)
    torch.cuda.synchronize()
    with L.KernelTimer() as kt2:
        for _ in range(3):
            codec.decode_accumulate(pk, [1.0 / M] * M, out=acc, views=views)
        torch.cuda.synchronize()
    res["decacc_us_per_pkt"] = round(kt2.ms["decode"] * 1e3 / (3 * M), 2)
    print(json.dumps({"tag": args.tag, "n": n, "k": k, "avg_us": res}), flush=True)


if __name__ == "__main__":
    main()
