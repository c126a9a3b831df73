"""One 128 M gradient through the lone-client fused encode, for rocprofv3 PMC passes:
``--mode packet`` = fc_topk_encode (k_fused_mag<false> + k_resolve), ``--mode dense`` =
fc_topk_encode_dense (k_fused_mag<true> + k_resolve), ``--mode batch1`` = the batched encode of
the one gradient (k_pilot + k_sample1 + k_compact_mag1 + k_resolve x2), ``--mode encdec`` =
fc_topk_encode_decode (k_fused_mag<false> + k_beta + k_decode_res).

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/x -o p -- python3 tools/fused_probe.py --mode packet
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
    ap.add_argument("--mode", default="packet", choices=("packet", "dense", "batch1", "encdec"))
    ap.add_argument("--n", type=int, default=134_217_728)
    ap.add_argument("--f", type=float, default=0.1)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    n, k = a.n, kept_count(a.f, a.n)
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    out = torch.empty_like(g)
    pkt = codec.encode_top(g, k)
    bpk = [codec.Packet.alloc(n, 0, g.device, k=k)]
    jobs = codec.encode_jobs([g], bpk)
    run = {"packet": lambda: codec.encode_top(g, k, packet=pkt, check=False),
           "dense": lambda: codec.compress_top_dense(g, k, out=out, packet=pkt, check=False),
           "batch1": lambda: codec.encode_top_batch([g], k, packets=bpk, jobs=jobs, check=False),
           "encdec": lambda: codec.encode_decode_top(g, k, packet=pkt, out=out, check=False)}[a.mode]
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(json.dumps({"mode": a.mode, "n": n, "k": k, "us": round(dt * 1e6, 1),
                      "retry": codec.resolve([pkt])}), flush=True)


if __name__ == "__main__":
    main()
