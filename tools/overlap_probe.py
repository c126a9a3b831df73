"""Does overlapping the FedAVG fold of client group g with the encode of group g+1 help?

    python tools/overlap_probe.py [--clients 64] [--groups 4]

Same kernels, same FedAVG order (the fold stays on one stream, continue_sum between groups);
prints the serial and the pipelined step time and checks the two aggregates are bit-equal.
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
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--groups", type=int, default=4)
    ap.add_argument("--n", type=int, default=134_217_728)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    dev = torch.device("cuda", 0)
    M, n, G = a.clients, a.n, a.groups
    k = kept_count(0.1, n)
    grads = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(i))
             .mul_(10.0 ** (-1 - 3 * i / M)) for i in range(M)]
    pkts = [codec.Packet.alloc(n, L.FC_FMT_IDXVAL, dev, k=k) for _ in range(M)]
    w = [1.0 / M] * M
    per = M // G
    groups = [list(range(g * per, (g + 1) * per)) for g in range(G)]
    jobs_all = codec.encode_jobs(grads, pkts)
    jobs_g = [codec.encode_jobs([grads[i] for i in gr], [pkts[i] for i in gr]) for gr in groups]
    views_g = [codec.views_tensor([pkts[i] for i in gr], [w[i] for i in gr], dev) for gr in groups]
    views_all = codec.views_tensor(pkts, w, dev)
    acc = torch.empty(n, dtype=torch.float32, device=dev)
    s_dec = torch.cuda.Stream(device=dev)

    def serial():
        codec.encode_top_batch(grads, k, packets=pkts, jobs=jobs_all, check=False)
        codec.decode_accumulate(pkts, w, out=acc, views=views_all)

    def pipelined():
        main_s = torch.cuda.current_stream(dev)
        evs = []
        for g, gr in enumerate(groups):
            codec.encode_top_batch([grads[i] for i in gr], k, packets=[pkts[i] for i in gr],
                                   jobs=jobs_g[g], check=False)
            ev = torch.cuda.Event()
            ev.record(main_s)
            s_dec.wait_event(ev)
            with torch.cuda.stream(s_dec):
                codec.decode_accumulate([pkts[i] for i in gr], [w[i] for i in gr], out=acc,
                                        views=views_g[g], continue_sum=g > 0)
        main_s.wait_stream(s_dec)

    enc_streams = [torch.cuda.Stream(device=dev) for _ in range(G)]

    def multistream():
        """encode group g on its own stream (the latency-bound sample/resolve launches of one
        group overlap the streaming compaction of another), then one fold on the main stream"""
        main_s = torch.cuda.current_stream(dev)
        ev0 = torch.cuda.Event()
        ev0.record(main_s)
        for g, gr in enumerate(groups):
            enc_streams[g].wait_event(ev0)
            with torch.cuda.stream(enc_streams[g]):
                codec.encode_top_batch([grads[i] for i in gr], k, packets=[pkts[i] for i in gr],
                                       jobs=jobs_g[g], check=False)
        for st in enc_streams:
            main_s.wait_stream(st)
        codec.decode_accumulate(pkts, w, out=acc, views=views_all)

    res = {}
    for name, fn in (("serial", serial), ("pipelined", pipelined), ("multistream", multistream),
                     ("serial2", serial), ("multistream2", multistream)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        res[name] = round((time.perf_counter() - t0) / a.iters * 1e3, 3)
        if name.startswith("serial"):
            ref = acc.clone()
        else:
            res[name + "_bitexact"] = bool(torch.equal(acc.view(torch.int32), ref.view(torch.int32)))
    st = [p.header().status for p in pkts]
    res["retry"] = sum(1 for s in st if s != 0)
    print(json.dumps({"clients": M, "groups": G, "ms": res}), flush=True)


if __name__ == "__main__":
    main()
