"""Lone-gradient encode paths at 128 M (and 16 M), for rocprofv3 kernel stats:
the fused packet encode (k_fused_mag<false> + k_resolve), the batched path with one client
(k_pilot/k_sample1 + k_compact_mag1 + k_resolve x2), each followed by the dense decode.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lone -o lone -- python3 tools/lone_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters):
    import torch
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    import torch
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    for n, iters in ((134_217_728, 20), (16_777_216, 200)):
        k = kept_count(0.1, n)
        g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
        out = torch.empty_like(g)
        pkt = codec.encode_top(g, k)
        bpk = [codec.Packet.alloc(n, 0, g.device, k=k)]
        jobs = codec.encode_jobs([g], bpk)
        res = {"n": n}
        res["fused_encode"] = timeit(lambda: codec.encode_top(g, k, packet=pkt, check=False), iters)
        res["fused_roundtrip"] = timeit(lambda: codec.decode(codec.encode_top(g, k, packet=pkt, check=False), out=out), iters)
        res["batch1_encode"] = timeit(lambda: codec.encode_top_batch([g], k, packets=bpk, jobs=jobs, check=False), iters)
        res["batch1_roundtrip"] = timeit(lambda: codec.decode(codec.encode_top_batch([g], k, packets=bpk, jobs=jobs, check=False)[0], out=out), iters)
        res["encdec"] = timeit(lambda: codec.encode_decode_top(g, k, packet=pkt, out=out, check=False), iters)
        res["decode"] = timeit(lambda: codec.decode(pkt, out=out), iters)
        print(json.dumps({a: (round(b, 1) if isinstance(b, float) else b) for a, b in res.items()}), flush=True)
        del g, out, pkt, bpk
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
