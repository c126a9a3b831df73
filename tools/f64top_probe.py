"""float64 top-k (fc_topk_dense_f64_sampled, k_fused64 -> k_resolve64) on one gradient, HIP-event
timed per call, for A/B builds (``--lib``/``--tag``).

    python tools/f64top_probe.py --n 16777216 [--lib tools/variants/lib_X.so] [--tag X]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16_777_216)
    ap.add_argument("--f", type=float, default=0.1)
    ap.add_argument("--iters", type=int, default=100)
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
    g = torch.randn(n, device="cuda", dtype=torch.float64,
                    generator=torch.Generator(device="cuda").manual_seed(3))
    out = torch.empty_like(g)
    fn = lambda: codec.compress_top_dense_f64(g, k, out=out, check=False)   # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    print(json.dumps({"n": n, "tag": a.tag, "f64_top_us": round(us, 2),
                      "retry": codec.resolve_f64(out)}), flush=True)


if __name__ == "__main__":
    main()
