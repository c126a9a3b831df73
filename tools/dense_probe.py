"""Single 128 M gradient through fc_topk_encode_dense (fused top-k -> dense), for rocprofv3.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dense -o dense -- python3 tools/dense_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(n=134_217_728, f=0.1, iters=20):
    import torch
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    k = kept_count(f, n)
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    out = torch.empty_like(g)
    pkt = codec.encode_top(g, k)
    for _ in range(3):
        codec.compress_top_dense(g, k, out=out, packet=pkt, check=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        codec.compress_top_dense(g, k, out=out, packet=pkt, check=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    redo = codec.resolve([pkt])
    print(json.dumps({"n": n, "k": k, "us": round(dt * 1e6, 1), "retry": redo,
                      "alg_frac": round((8.0 * n + 16.0 * k) / dt / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
