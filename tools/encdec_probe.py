"""Lone-gradient round trip for A/B builds: fc_topk_encode_decode (packet encode + dense decode)
and fc_topk_encode_dense (the drop-in q), HIP-event timed per call.

    python tools/encdec_probe.py --n 134217728 [--lib tools/variants/lib_X.so] [--tag X]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=134_217_728)
    ap.add_argument("--f", type=float, default=0.1)
    ap.add_argument("--iters", type=int, default=0)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    if a.lib:
        L.load(os.path.join(ROOT, a.lib))
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    n, k = a.n, kept_count(a.f, a.n)
    iters = a.iters or (20 if n > (64 << 20) else 200)
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    out = torch.empty_like(g)
    pkt = codec.encode_top(g, k)
    res = {"n": n, "tag": a.tag}

    def t(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) * 1e3 / iters, 2)
    res["encdec_us"] = t(lambda: codec.encode_decode_top(g, k, packet=pkt, out=out, check=False))
    res["retry"] = codec.resolve([pkt])
    res["dense_us"] = t(lambda: codec.compress_top_dense(g, k, out=out, packet=pkt, check=False))
    res["encode_us"] = t(lambda: codec.encode_top(g, k, packet=pkt, check=False))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
