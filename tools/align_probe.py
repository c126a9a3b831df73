"""Lone encodes with the packet's entry arrays (packet path) or the dense result q (dense path)
placed at an offset of X bytes from their allocation's start (the allocator aligns both, like
the gradient, to 2 MiB): does the relative alignment of the streams g -> val/idx (or g -> q)
cost HBM channel conflicts?
    python tools/align_probe.py [--n 134217728] [--offsets 0,4096,8192,65536,1052672]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=134_217_728)
    ap.add_argument("--offsets", default="0,4096,8192,65536,1052672")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    dev = torch.device("cuda", 0)
    n = args.n
    k = kept_count(0.1, n)
    g = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).mul_(1e-2)
    offs = [int(x) for x in args.offsets.split(",")]
    base = codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k)
    cap = base.capacity
    res = {}

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.iters * 1e3

    for rep in range(args.reps):
        for off in offs:
            vbuf = torch.empty(cap + off // 4, dtype=torch.float32, device=dev)
            ibuf = torch.empty(cap + off // 2, dtype=torch.int16, device=dev)
            pkt = codec.Packet(n=n, fmt=L.FC_FMT_IDXVAL, k=k, val=vbuf[off // 4:off // 4 + cap],
                               cnt=base.cnt, hdr=base.hdr, idx=ibuf[off // 2:off // 2 + cap],
                               bitmap=None, qoff=base.qoff)
            qbuf = torch.empty(n + off // 4, dtype=torch.float32, device=dev)
            q = qbuf[off // 4:off // 4 + n]
            tp = timed(lambda: codec.encode_top(g, k, packet=pkt, check=False))
            td = timed(lambda: codec.compress_top_dense(g, k, out=q, packet=base, check=False))
            assert codec.resolve([pkt]) == 0
            res.setdefault(f"packet_off{off}_us", []).append(round(tp, 1))
            res.setdefault(f"dense_off{off}_us", []).append(round(td, 1))
            del vbuf, ibuf, qbuf, pkt, q
    print(json.dumps({"n": n, **res}), flush=True)


if __name__ == "__main__":
    main()
