"""Per-call spread of the lone 128 M round trip: fc_topk_encode_decode, fc_topk_encode and
fc_decode_dense timed call by call with HIP events (min / median / max and a coarse histogram),
to see whether a slow process is slow on every call or on a few.

    python tools/rt_spread.py [--n 134217728] [--calls 60] [--lib ...] [--tag ...]
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
    ap.add_argument("--calls", type=int, default=60)
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
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    out = torch.empty_like(g)
    pkt = codec.encode_top(g, k)

    def spread(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.calls)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        us = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev)
        return {"min": round(us[0], 1), "p50": round(us[len(us) // 2], 1), "p90": round(us[int(len(us) * 0.9)], 1),
                "max": round(us[-1], 1), "all": [round(u, 1) for u in us]}

    res = {"n": n, "tag": a.tag,
           "encdec": spread(lambda: codec.encode_decode_top(g, k, packet=pkt, out=out, check=False)),
           "encode": spread(lambda: codec.encode_top(g, k, packet=pkt, check=False)),
           "decode": spread(lambda: codec.decode(pkt, out=out))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
