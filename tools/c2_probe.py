"""configs[1] / configs[2] alone (bench.small_configs) for same-box A/B of library builds.
    python tools/c2_probe.py [--lib path/to/libfedcodec.so] [--tag t] [--steps 100]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tag", default="")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--separate-packets", action="store_true")
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--pipeline", action="store_true")
    args = ap.parse_args()
    import torch
    from openmsftl_amd import _lib as L
    if args.lib:
        L.load(os.path.abspath(args.lib))
    from openmsftl_amd import codec
    import bench
    r = bench.small_configs(torch, codec, L, torch.device("cuda", 0), 0.1, steps=args.steps,
                           slab_packets=not args.separate_packets, streams=args.streams,
                           pipeline=args.pipeline)
    c1, c2 = r["config1_single_16M"], r["config2_128x16M"]
    print(json.dumps({"tag": args.tag, "slab_packets": not args.separate_packets, "c2_ms": c2["ms_per_step"], "c2_frac": c2["hbm_frac"],
                      "c1_dense_us": c1["fused_dense"]["us"], "c1_rt_us": c1["us_per_encode_decode"]}),
          flush=True)


if __name__ == "__main__":
    main()
