"""Phase timeline of the single-gradient encode's small kernels (k_sample1, k_resolve) from a
FC_TRACE build (tools/variants/lib_trace.so): per trace slot, the min / median / max time
(us) after the kernel's first workgroup started, over the workgroups that recorded it.

    python tools/trace_probe.py --lib tools/variants/lib_trace.so [--n 134217728] [--dense]
"""
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
    ap.add_argument("--f", type=float, default=0.1)
    ap.add_argument("--dense", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch
    from openmsftl_amd import _lib as L
    lib = L.load(os.path.abspath(args.lib))
    lib.fc_trace_read.restype = ctypes.c_int
    lib.fc_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    from openmsftl_amd import codec
    from openmsftl_amd.compression import kept_count
    n, k = args.n, kept_count(args.f, args.n)
    g = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    out = torch.empty_like(g)
    pkt = codec.encode_top(g, k)
    for _ in range(5):
        if args.dense:
            codec.compress_top_dense(g, k, out=out, packet=pkt, check=False)
        else:
            codec.encode_top(g, k, packet=pkt, check=False)
    torch.cuda.synchronize()
    buf = np.zeros(1 << 16, dtype=np.uint64)
    L.check(lib.fc_trace_read(buf.ctypes.data, buf.size), "trace")
    t = buf.reshape(-1, 32).astype(np.float64) / 100.0      # 100 MHz -> us
    res = {}
    # "fused": k_fused_mag's chunk workgroups (24 loads issued, 25 bracket received, 26 done),
    # on the sample's clock (same launch)
    for name, slots in (("sample", [0, 20, 21, 22, 2, 3, 4, 18, 19, 5, 7, 23, 6]), ("fused", [24, 25, 26]),
                        ("resolve", [8, 10, 29, 27, 28, 9, 11, 16, 17, 12, 14, 13, 15])):
        rec = t[:, slots[0]] > 0
        if name != "fused":
            t0 = t[rec, slots[0]].min() if rec.any() else 0.0
        res[name] = {}
        for sl in slots:
            col = t[:, sl]
            col = col[(col > 0) & (col >= t0) & (col < t0 + 1e4)] - t0
            if col.size:
                res[name][sl] = [round(float(col.min()), 2), round(float(np.median(col)), 2),
                                 round(float(col.max()), 2), int(col.size)]
    # k_fused_mag's chunk workgroups split into those that had loaded before the bracket was
    # published (slot 6: the first resident round) and the later ones
    rounds = {}
    t6 = t[:, 6].max()
    t0 = t[t[:, 0] > 0, 0].min() if (t[:, 0] > 0).any() else 0.0
    ck = (t[:, 24] > 0) & (t[:, 26] > 0)
    if t6 > 0 and ck.any():
        for nm, sel in (("early", ck & (t[:, 24] <= t6)), ("late", ck & (t[:, 24] > t6))):
            if sel.any():
                rounds[nm] = {int(sl): [round(float(np.percentile(t[sel, sl] - t0, q)), 2) for q in (0, 10, 50, 90, 100)]
                              for sl in (24, 25, 26)}
                rounds[nm]["count"] = int(sel.sum())
    print(json.dumps({"n": n, "dense": args.dense, "phases_us_min_med_max_count": res,
                      "fused_rounds_p0_10_50_90_100": rounds}), flush=True)


if __name__ == "__main__":
    main()
