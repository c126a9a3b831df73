"""Sub-batch splits of the batched top-k encode over two forked streams (encode + fold step).

    python tools/split_probe.py [--clients 128]

Prints ms per step for each split and checks the aggregate is bit-equal to the one-stream one.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SPLITS = {"one": (1, None), "2x64": (2, [64, 64]), "8-56-56-8": (2, [8, 56, 56, 8]),
          "16-48-48-16": (2, [16, 48, 48, 16]), "4x32": (2, [32, 32, 32, 32]),
          "4x32_4streams": (4, [32, 32, 32, 32]), "3 streams": (3, None),
          "8x16_4streams": (4, [16] * 8)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--n", type=int, default=134_217_728)
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    dev = torch.device("cuda", 0)
    M, n = a.clients, a.n
    k = kept_count(0.1, n)
    grads = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(i))
             .mul_(10.0 ** (-1 - 3 * i / M)) for i in range(M)]
    pkts = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k) for _ in range(M)]
    w = [1.0 / M] * M
    jobs = codec.encode_jobs(grads, pkts)
    views = codec.views_tensor(pkts, w, dev)
    acc = torch.empty(n, dtype=torch.float32, device=dev)
    res, ref = {}, None
    for rep in range(2):
        for name, (nst, groups) in SPLITS.items():
            def step():
                codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs, check=False,
                                       streams=nst, groups=groups)
                codec.decode_accumulate(pkts, w, out=acc, views=views)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.iters * 1e3
            res[name] = min(res.get(name, 1e9), round(ms, 3))
            if ref is None:
                ref = acc.clone()
            elif not torch.equal(acc.view(torch.int32), ref.view(torch.int32)):
                res[name + "_MISMATCH"] = True
    res["retry"] = sum(1 for p in pkts if p.header().status != 0)
    print(json.dumps({"clients": M, "ms": res}), flush=True)


if __name__ == "__main__":
    main()
