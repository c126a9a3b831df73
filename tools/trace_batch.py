"""Phase timeline of the batched encode's k_sample1 / k_resolve (FC_TRACE build): per trace
slot the min / median / max time (us) after the kernel's first workgroup started, over all
workgroups (all clients) that recorded it.
    python tools/trace_batch.py --lib tools/variants/lib_trace.so [--clients 64] [--n 134217728]
Resolve slots (fc_topk.hip): 8 start, 10 per-chunk sizes, 29 candidates binned, 27 bins
flushed, 16/17 bin ticket, 28 beta known, 9 after binning, 11 gathered, 12 T64 wait done,
14 T64 selected, 13 fix-up done, 15 last arriver done."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--n", type=int, default=134_217_728)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--f", type=float, default=0.1)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import numpy as np
    import torch
    from openmsftl_amd import _lib as L
    lib = L.load(os.path.abspath(args.lib))
    lib.fc_trace_read.restype = ctypes.c_int
    lib.fc_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    n, k, M = args.n, kept_count(args.f, args.n), args.clients
    gs = [torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(s))
          .mul_(10.0 ** (-1 - 3 * s / M)) for s in range(M)]
    pk = codec.encode_top_batch(gs, k, streams=1)
    jobs = codec.encode_jobs(gs, pk)
    out = {}
    for part, slots in (("sample", [0, 20, 21, 22, 2, 3, 4, 18, 19, 5, 7, 23, 6]),
                        ("resolve", [8, 10, 29, 27, 16, 17, 28, 9, 11, 12, 14, 13, 15])):
        for _ in range(3):
            codec.encode_top_batch(gs, k, packets=pk, jobs=jobs, check=False, streams=1)
        torch.cuda.synchronize()
        buf = np.zeros(1 << 16, dtype=np.uint64)
        L.check(lib.fc_trace_read(buf.ctypes.data, buf.size), "trace")
        t = buf.reshape(-1, 32).astype(np.float64) / 100.0
        # the last launch to write a slot set wins: the resolve overwrote the sample's rows of
        # the same block ids, so each part is read from its own launch's slots
        col0 = t[:, slots[0]]
        rec = col0 > 0
        t0 = col0[rec].min() if rec.any() else 0.0
        res = {}
        for sl in slots:
            col = t[:, sl]
            col = col[(col > 0) & (col >= t0) & (col < t0 + 2e4)] - t0
            if col.size:
                res[sl] = [round(float(col.min()), 2), round(float(np.median(col)), 2),
                           round(float(col.max()), 2), int(col.size)]
        out[part] = res
    print(json.dumps({"tag": args.tag, "n": n, "clients": M, "phases_us_min_med_max_count": out}), flush=True)


if __name__ == "__main__":
    main()
