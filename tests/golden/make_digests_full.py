"""SHA-256 digests of the oracle's outputs at the sizes bench.py and tools/e2e_bench.py time
(build container; the GPU tests in tests/test_fullsize_parity.py compare the HIP path to them).

    python tests/golden/make_digests_full.py [--jobs 6]

Workloads (BASELINE.json configs; inputs regenerated bit-identically on the GPU box by
``fullsize_grad``: torch's CPU generator, same torch build, then an fp32 scale):
  * configs2  — 128 clients x 16,777,216, top f = 0.1: every client's dense q
    (compression.py:31-37) and the FedAVG aggregate of the 128 rows (aggregation.py:61-63 ->
    gar.py:44, w = fl32(1/128), +0-started row-order fp32 sum);
  * configs3  — the configs[3] per-GPU shard shape at 8 clients x 134,217,728, top f = 0.1:
    dense q per client and the 8-row aggregate;
  * configs4  — 70 clients x 25,557,032, top f = 0.01, FedAVG aggregate only (the ring of
    tools/e2e_bench.py folds groups of 64, so its continued fold is crossed).
The oracle selection is packet_oracle.selected_indices (the composite-key rule, pinned to the
reference's own outputs and digests in tests/test_oracle_golden.py).  Only digests are stored
(tests/golden/digests_full.json).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
from multiprocessing import get_context

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

WORKLOADS = {
    "configs2": {"clients": 128, "n": 16_777_216, "fraction": 0.1, "seed0": 20_000,
                 "per_client": True},
    "configs3": {"clients": 8, "n": 134_217_728, "fraction": 0.1, "seed0": 30_000,
                 "per_client": True},
    "configs4": {"clients": 70, "n": 25_557_032, "fraction": 0.01, "seed0": 40_000,
                 "per_client": False, "group": 64},
}


def scales(name: str, clients: int) -> np.ndarray:
    """Per-client fp32 scale s_c = 10**U(-4, -1) (SURVEY.md §8(d) synthetic gradients)."""
    seed = {"configs2": 2, "configs3": 3, "configs4": 4}[name]
    return (10.0 ** np.random.default_rng(seed).uniform(-4, -1, size=clients)).astype(np.float32)


def fullsize_grad(name: str, c: int) -> np.ndarray:
    """Client c's fp32 gradient: torch CPU randn (seed0 + c) * s_c, as float32."""
    import torch
    w = WORKLOADS[name]
    g = torch.Generator().manual_seed(w["seed0"] + c)
    x = torch.randn(w["n"], generator=g, dtype=torch.float32)
    x.mul_(float(scales(name, w["clients"])[c]))
    return x.numpy()


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _client(args):
    name, c = args
    from oracle import compression_oracle as co
    from oracle import packet_oracle as po
    w = WORKLOADS[name]
    g = fullsize_grad(name, c)
    n = g.shape[0]
    k = co.num_kept(w["fraction"], n)
    idx = po.selected_indices(po.mag_key(g), k)
    q = po.decode_dense(n, idx, g[idx])
    return c, sha(g), sha(q), idx, g[idx]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=6)
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    path = os.path.join(HERE, "digests_full.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    out["generator"] = ("torch.Generator().manual_seed(seed0 + c); torch.randn(n, float32) * "
                        "s_c, s_c = 10**np.random.default_rng(cfg).uniform(-4,-1,M) as float32")
    for name, w in WORKLOADS.items():
        if args.only and name != args.only:
            continue
        M, n = w["clients"], w["n"]
        wt = np.float32(1.0 / M)                           # gar.py:37-40, fp32 G
        acc = np.zeros(n, dtype=np.float32)                # np.sum's +0 start (gar.py:44)
        rec = {k: v for k, v in w.items()}
        rec["k"] = round(w["fraction"] * n)
        rec["input_sha256"], rec["q_sha256"] = {}, {}
        jobs = args.jobs if n <= 30_000_000 else 2
        with get_context("spawn").Pool(jobs) as pool:
            for c, gs, qs, idx, val in pool.imap(_client, [(name, c) for c in range(M)]):
                if c < 2 or w["per_client"]:
                    rec["input_sha256"][str(c)] = gs
                if w["per_client"]:
                    rec["q_sha256"][str(c)] = qs
                # acc = fl(acc + fl(w * q_c)): zero coordinates add fl(+0 * w) = +0 to a sum that
                # is never -0, so only the kept ones change acc
                acc[idx] = np.add(acc[idx], np.multiply(val, wt))
                print(f"[{name}] client {c} done", flush=True)
        rec["aggregate_sha256"] = sha(acc)
        out[name] = rec
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
        print(f"[{name}] aggregate {rec['aggregate_sha256'][:16]}", flush=True)


if __name__ == "__main__":
    main()
