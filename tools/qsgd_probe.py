"""QSGD (opt-in codec) on one gradient: encode (k_qsgd_norm = SAMPLE class, k_qsgd_quant =
COMPACT) + dense decode (DECODE), HIP-event averages and the wall time per encode+decode.

    python tools/qsgd_probe.py [--lib tools/variants/lib_X.so] [--n 134217728] [--bits 2]
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
    ap.add_argument("--lib", default=None)
    ap.add_argument("--n", type=int, default=134_217_728)
    ap.add_argument("--bits", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default="")
    ap.add_argument("--fold", type=int, default=0, help="also time a FedAVG fold of this many "
                    "packets of --fold-n elements (decode_accumulate_qsgd)")
    ap.add_argument("--fold-n", type=int, default=25_557_032)
    a = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    if a.lib:
        L.load(os.path.abspath(a.lib))
    from openmsftl_amd import codec
    g = torch.randn(a.n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    out = torch.empty_like(g)
    pkt = codec.encode_qsgd(g, a.bits)

    def step():
        codec.encode_qsgd(g, a.bits, packet=pkt)
        codec.decode_qsgd(pkt, out=out)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.iters * 1e6
    with L.KernelTimer() as kt:
        for _ in range(a.iters):
            step()
        torch.cuda.synchronize()
    res = {c: round(kt.avg_us(c), 2) for c in L.TIME_CLASSES if kt.launches.get(c)}
    fold = None
    if a.fold:
        del g, out, pkt
        torch.cuda.empty_cache()
        gf = torch.randn(a.fold_n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
        pk = [codec.encode_qsgd(gf, a.bits, seed=i) for i in range(a.fold)]
        w = [1.0 / a.fold] * a.fold
        acc = codec.decode_accumulate_qsgd(pk, w)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            codec.decode_accumulate_qsgd(pk, w, out=acc)
        torch.cuda.synchronize()
        fus = (time.perf_counter() - t0) / 5 * 1e6
        code_b = pk[0].codes.numel() * pk[0].codes.element_size()
        fold = {"m": a.fold, "n": a.fold_n, "us": round(fus, 1),
                "GBps_codes": round(a.fold * code_b / fus / 1e3, 1)}
    alg = 13.0 * a.n if a.bits <= 2 else None      # bench.py qsgd_single's algorithmic bytes
    print(json.dumps({"tag": a.tag, "n": a.n, "bits": a.bits, "avg_us": res, "wall_us": round(wall, 1),
                      "hbm_frac": round(alg / wall / 8e6, 4) if alg else None, "fold": fold}), flush=True)


if __name__ == "__main__":
    main()
