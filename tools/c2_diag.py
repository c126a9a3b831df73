"""configs[2] step-time diagnosis: host enqueue time vs GPU time per step: batched encode
+ decode_accumulate or the pipelined encode_fold_batch, on 1 or 2 streams, repeated in one process (is a slow run host-bound or GPU-bound?).
    python tools/c2_diag.py [--reps 3] [--steps 100] [--modes top2,top1,fold2,fold1]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--modes", default="top2,top1,fold2,fold1")
    args = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    import bench
    dev = torch.device("cuda", 0)
    n, M = 16_777_216, 128
    k = kept_count(0.1, n)
    grads = bench.make_grads(M, n, 0, dev, torch)
    pkts = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k) for _ in range(M)]
    w = [1.0 / M] * M
    jobs = codec.encode_jobs(grads, pkts)
    views = codec.views_tensor(pkts, w, dev)
    acc = torch.empty(n, dtype=torch.float32, device=dev)
    for rep in range(args.reps):
        for ms in args.modes.split(","):
            mode, streams = ms[:-1], int(ms[-1])
            def step():
                if mode == "fold":
                    codec.encode_fold_batch(grads, k, w, acc, packets=pkts, jobs=jobs,
                                            views=views, streams=streams)
                    return
                codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs, check=False,
                                       streams=streams)
                codec.decode_accumulate(pkts, w, out=acc, views=views)
            for _ in range(10):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            for _ in range(args.steps):
                step()
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(json.dumps({"rep": rep, "mode": mode, "streams": streams,
                              "host_enqueue_us": round((t1 - t0) / args.steps * 1e6, 1),
                              "wall_ms": round((t2 - t0) / args.steps * 1e3, 3),
                              "event_ms": round(e0.elapsed_time(e1) / args.steps, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
