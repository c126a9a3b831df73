"""Concurrent batched encodes (encode_top_batch(streams=2), the sub-batches free to overlap):
count client statuses that are not OK over many steps.  Round 4's k_resolve waited in-kernel
and stalled here (23 of 1,500 steps RETRY unless the encodes were serialized); since round 5
no batched kernel waits, and no serialization exists to switch off.
    python tools/stall_probe.py [--steps 300] [--n 4194304]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--m", type=int, default=128)
    args = ap.parse_args()
    import numpy as np
    import torch
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    n, M = args.n, args.m
    k = kept_count(0.1, n)
    import bench
    from openmsftl_amd import _lib as L
    dev = torch.device("cuda", 0)
    grads = bench.make_grads(M, n, 0, dev, torch)
    hdrs = torch.zeros((M, L.HDR_BYTES), dtype=torch.uint8, device=dev)
    pk = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, hdr=hdrs[j], k=k) for j in range(M)]
    codec.encode_top_batch(grads, k, packets=pk)
    jobs = codec.encode_jobs(grads, pk)
    w = [1.0 / M] * M
    views = codec.views_tensor(pk, w, dev)
    acc = torch.empty(n, dtype=torch.float32, device=dev)
    bad = torch.zeros((), dtype=torch.int64, device=dev)
    bad_steps = torch.zeros((), dtype=torch.int64, device=dev)
    status = hdrs[:, 36:40]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):            # no host sync: steps queue back to back (bench-like)
        codec.encode_top_batch(grads, k, packets=pk, jobs=jobs, check=False, streams=2)
        nb = (status != 0).any(dim=1).sum()
        bad += nb
        bad_steps += (nb > 0).long()
        codec.decode_accumulate(pk, w, out=acc, views=views)
    torch.cuda.synchronize()
    bad, bad_steps = int(bad), int(bad_steps)
    dt = (time.perf_counter() - t0) / args.steps
    print(json.dumps({"n": n, "clients": M, "steps": args.steps,
                      "steps_with_retry": bad_steps, "retry_statuses": bad,
                      "ms_per_step": round(dt * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
