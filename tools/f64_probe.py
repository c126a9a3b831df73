"""float64 top-k on one gradient (fc_topk_dense_f64_sampled): HIP-event averages per launch
class (k_fused64 = COMPACT: the sample and the streaming pass in one launch; k_resolve64 = ENGINE), wall
time per call, and the exact engine for comparison.

    python tools/f64_probe.py [--lib tools/variants/lib_X.so] [--n 16777216] [--f 0.1]
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
    ap.add_argument("--lib", default=None)
    ap.add_argument("--n", type=int, default=16_777_216)
    ap.add_argument("--f", type=float, default=0.1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    if a.lib:
        L.load(os.path.abspath(a.lib))
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    k = kept_count(a.f, a.n)
    g = torch.randn(a.n, device="cuda", dtype=torch.float64,
                    generator=torch.Generator(device="cuda").manual_seed(5)).mul_(1e-2)
    out = torch.empty_like(g)
    run = lambda: codec.compress_top_dense_f64(g, k, out=out, check=False)   # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        run()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.iters * 1e6
    redo = codec.resolve_f64(out)
    with L.KernelTimer() as kt:
        for _ in range(a.iters):
            run()
        torch.cuda.synchronize()
    res = {c: round(kt.avg_us(c), 2) for c in L.TIME_CLASSES if kt.launches.get(c)}
    print(json.dumps({"tag": a.tag, "n": a.n, "k": k, "avg_us": res, "wall_us": round(wall, 1),
                      "retry": redo, "hbm_frac": round(16.0 * a.n / wall / 8e6, 4)}), flush=True)


if __name__ == "__main__":
    main()
