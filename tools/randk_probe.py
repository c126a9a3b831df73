"""Native rand-k (Philox keys) at 16 M: encode + dense decode, for rocprofv3 kernel stats and
A/B builds (``--lib``/``--tag``).

    rocprofv3 --kernel-trace --stats -d gpurun_out/x -o r -- python3 tools/randk_probe.py
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
    ap.add_argument("--iters", type=int, default=200)
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
    pkt = codec.encode_top(g, k, key_mode=L.FC_KEY_PHILOX, seed=5, offset=1)

    def rt():
        codec.encode_top(g, k, key_mode=L.FC_KEY_PHILOX, seed=5, offset=1, packet=pkt, check=False)
        codec.decode(pkt, out=out)
    for _ in range(3):
        rt()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        rt()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    print(json.dumps({"tag": a.tag, "n": n, "k": k, "randk_roundtrip_us": round(us, 2),
                      "hbm_frac": round((8.0 * n + 16.0 * k) / us / 8e6, 4),
                      "retry": codec.resolve([pkt])}), flush=True)


if __name__ == "__main__":
    main()
