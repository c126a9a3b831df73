"""Per-kernel-class HIP-event timing of one codec setting on one gradient (A/B probe for
tools/ab.py): rand-k with native Philox keys, mask encodes (host permutation / host Bernoulli
mask / native Philox Bernoulli; idx/val or bitmap packets) and their dense decode.

    python tools/codec_probe.py --mode philox|rand_mask|drop_mask|drop_bern [--n 16777216]
        [--f 0.1] [--p 0.1] [--fmt idxval|bitmap] [--lib PATH] [--tag T]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="philox")
    ap.add_argument("--n", type=int, default=16_777_216)
    ap.add_argument("--f", type=float, default=0.1)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--fmt", default="bitmap")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import numpy as np
    import torch
    from openmsftl_amd import _lib as L
    if args.lib:
        L.load(os.path.abspath(args.lib))
    from openmsftl_amd import codec
    from openmsftl_amd.compression import bitmask_words, kept_count
    n = args.n
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    out = torch.empty_like(g)
    k = kept_count(args.f, n)
    fmt = L.FC_FMT_BITMAP if args.fmt == "bitmap" else L.FC_FMT_IDXVAL
    if args.mode == "philox":
        pkt = codec.encode_top(g, k, key_mode=L.FC_KEY_PHILOX, seed=3, offset=1)
        enc = lambda: codec.encode_top(g, k, key_mode=L.FC_KEY_PHILOX, seed=3, offset=1,  # noqa: E731
                                       packet=pkt, check=False)
        alg_enc, alg_dec = 4.0 * n + 8.0 * k, 8.0 * k + 4.0 * n
    else:
        if args.mode == "rand_mask":
            cid = L.FC_CODEC_RAND
            mb = bitmask_words(np.random.default_rng(1).permutation(n)[:k], n, False)
            fmt = L.FC_FMT_IDXVAL
        else:
            cid = L.FC_CODEC_DROPOUT_BIASED
            mb = bitmask_words(np.random.default_rng(2).binomial(1, args.p, n), n, True)
        kw = {"mask_bits": torch.from_numpy(mb.view(np.int32)).cuda()} \
            if args.mode != "drop_bern" else {"seed": 4, "offset": 2}
        pkt = codec.encode_mask(g, cid, p=args.p, fmt=fmt, **kw)
        enc = lambda: codec.encode_mask(g, cid, p=args.p, fmt=fmt, packet=pkt, **kw)  # noqa: E731
        nnz = int(pkt.cnt.sum().item())
        mbytes = n / 8.0 if args.mode != "drop_bern" else 0.0
        ent = 8.0 if fmt == L.FC_FMT_IDXVAL else 4.0
        alg_enc = 4.0 * n + mbytes + ent * nnz + (n / 8.0 if fmt == L.FC_FMT_BITMAP else 0.0)
        alg_dec = 4.0 * n + ent * nnz + (n / 8.0 if fmt == L.FC_FMT_BITMAP else 0.0)
    for _ in range(3):
        enc()
        codec.decode(pkt, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        enc()
        codec.decode(pkt, out=out)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.iters * 1e6
    with L.KernelTimer() as kt:
        for _ in range(args.iters):
            enc()
            codec.decode(pkt, out=out)
        torch.cuda.synchronize()
    if args.mode == "philox":
        assert codec.resolve([pkt]) == 0
    res = {c: round(kt.avg_us(c), 2) for c in L.TIME_CLASSES if kt.launches.get(c)}
    enc_us = sum(v for c, v in res.items() if c != "decode")
    print(json.dumps({"tag": args.tag, "mode": args.mode, "fmt": args.fmt, "n": n,
                      "avg_us": res, "wall_us": round(wall, 1),
                      "enc_frac": round(alg_enc / (enc_us * 1e-6) / 8e12, 4),
                      "dec_frac": round(alg_dec / (res["decode"] * 1e-6) / 8e12, 4),
                      "frac": round((alg_enc + alg_dec) / (wall * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
