"""Generate golden vectors by running the REFERENCE codec (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Imports OpenMSFTL from /root/reference (read-only; ``import ftl.agents`` must come first,
SURVEY.md §8(c): aggregation.py:11 <-> server.py:11 circular import) and records inputs and
the reference's outputs of ``Compression.compress`` (compression.py:23-77) and
``FedAvg.aggregate`` (gar.py:32-56).  Only data is written (``golden_*.npz`` +
``manifest.json``); nothing of the reference's source travels.  The GPU box never runs this.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.path.insert(0, REF)
    import ftl.agents  # noqa: F401  (import-order requirement)
    from ftl.compression import Compression
    from ftl.gradient_aggregation.gar import FedAvg
    return Compression, FedAvg


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def gaussian(n, seed, scale=1.0):
    return (np.random.default_rng(seed).standard_normal(n, dtype=np.float32)
            * np.float32(scale))


def special_inputs():
    """Edge-case inputs: ties, ±0, NaN/inf, denormals, tiny sizes."""
    rng = np.random.default_rng(7)
    cases = {}
    cases["ties_smallint_1000"] = rng.integers(-3, 4, 1000).astype(np.float32)
    cases["ties_smallint_4096"] = rng.integers(-8, 9, 4096).astype(np.float32)
    cases["allzero_signed_64"] = np.where(rng.random(64) < 0.5, -0.0, 0.0).astype(np.float32)
    g = gaussian(1000, 11)
    g[[3, 500, 999]] = np.nan
    g[[10, 20]] = np.inf
    g[30] = -np.inf
    cases["nan_inf_1000"] = g
    d = (rng.standard_normal(4096) * 1e-40).astype(np.float32)     # denormals
    d[::7] = 0.0
    cases["denormal_4096"] = d
    cases["const_1000"] = np.full(1000, 0.25, dtype=np.float32)
    cases["n1"] = np.array([-2.5], dtype=np.float32)
    cases["n5"] = gaussian(5, 5)
    cases["n7"] = gaussian(7, 3)
    return cases


def main():
    Compression, FedAvg = _import_reference()
    manifest = {"reference": "microsoft/OpenMSFTL @ /root/reference",
                "numpy": np.__version__, "cases": {}}
    arrays = {}

    def add(name, **kw):
        meta = {}
        for key, val in kw.items():
            if key == "input":                       # inputs stored once, by digest
                iname = "input__" + sha(val)[:16]
                arrays[iname] = val
                meta["input"] = iname
            elif isinstance(val, np.ndarray):
                arrays[f"{name}__{key}"] = val
            else:
                meta[key] = val
        manifest["cases"][name] = meta

    # ---- top -------------------------------------------------------------------------
    inputs = {f"gauss_{n}": gaussian(n, 100 + n) for n in (64, 1000, 4096, 65537)}
    inputs.update(special_inputs())
    fracs = (0.1, 0.5, 0.01, 1.0, 0.0, 1.5, -0.1, 0.37)
    for iname, g in inputs.items():
        for f in fracs:
            C = Compression({"compression_function": "top", "fraction_coordinate": f})
            q = C.compress(g.copy())
            add(f"top__{iname}__f{f}", codec="top", fraction=f, n=int(g.shape[0]),
                input=g, output=q, out_dtype=str(q.dtype))

    # ---- full (identity; returns the same object) --------------------------------------
    g = gaussian(1000, 1)
    q = Compression({"compression_function": "full"}).compress(g)
    add("full__gauss_1000", codec="full", same_object=bool(q is g), input=g, output=q)

    # ---- rand / dropout-* (global legacy RNG, seeded) ----------------------------------
    for n in (7, 1000, 65537):
        g = gaussian(n, 200 + n)
        for f in (0.1, 0.5, 0.01):
            seed = 1000 + n
            np.random.seed(seed)
            q = Compression({"compression_function": "rand", "fraction_coordinate": f}).compress(g)
            after = int(np.random.randint(0, 2**31 - 1))  # state after the call
            add(f"rand__n{n}__f{f}", codec="rand", fraction=f, seed=seed, n=n,
                rng_next=after, input=g, output=q, out_dtype=str(q.dtype))
        for fn in ("dropout-biased", "dropout-unbiased"):
            for p in (0.1, 0.3, 0.5, 0.7, 1.0):
                seed = 2000 + n
                np.random.seed(seed)
                q = Compression({"compression_function": fn, "dropout_p": p}).compress(g)
                after = int(np.random.randint(0, 2**31 - 1))
                add(f"{fn}__n{n}__p{p}", codec=fn, p=p, seed=seed, n=n, rng_next=after,
                    input=g, output=q, out_dtype=str(q.dtype))
    g = inputs["nan_inf_1000"]
    for fn in ("dropout-biased", "dropout-unbiased"):
        np.random.seed(77)
        q = Compression({"compression_function": fn, "dropout_p": 0.5}).compress(g)
        add(f"{fn}__nan_inf_1000__p0.5", codec=fn, p=0.5, seed=77, n=1000,
            input=g, output=q, out_dtype=str(q.dtype))

    # ---- errors ------------------------------------------------------------------------
    errs = {}
    for fn, lw in (("qsgd", False), ("bogus", False), ("top", True)):
        try:
            Compression({"compression_function": fn}).compress(gaussian(8, 0), layer_wise=lw)
            errs[f"{fn}|{lw}"] = None
        except Exception as e:  # noqa: BLE001
            errs[f"{fn}|{lw}"] = type(e).__name__
    manifest["errors"] = errs

    # ---- FedAvg over compressed rows (aggregation.py:61-63 -> gar.py:44) ---------------
    for M, n, fn in ((4, 4096, "top"), (10, 1000, "dropout-unbiased"), (128, 4096, "top"),
                     (10, 1000, "full"), (4, 65537, "rand")):
        np.random.seed(3000 + M)
        grads = [gaussian(n, 5000 + i, scale=10.0 ** np.random.uniform(-4, -1))
                 for i in range(M)]
        C = Compression({"compression_function": fn, "fraction_coordinate": 0.1,
                         "dropout_p": 0.1})
        order = np.random.permutation(M)                  # random.sample order, not id order
        G = np.zeros((M, n), dtype=np.float32)
        rows = []
        for ix, cid in enumerate(order):
            G[ix, :] = C.compress(grads[cid])
            rows.append(G[ix].copy())
        agg = FedAvg({"aggregation_scheme": "fed_avg"}).aggregate(G=G, client_ids=order)
        add(f"fedavg__M{M}__n{n}__{fn}", codec=fn, M=M, n=n, G=G, order=order,
            output=agg, out_dtype=str(agg.dtype))

    # ---- large sizes: digests only ------------------------------------------------------
    large = {}
    for n, f, seed in ((16_777_216, 0.1, 16), (16_777_216, 0.01, 16),
                       (25_557_032, 0.01, 25), (25_557_032, 0.1, 25)):
        g = gaussian(n, seed)
        q = Compression({"compression_function": "top", "fraction_coordinate": f}).compress(g)
        nz = np.sort(np.nonzero(q)[0]).astype(np.uint32)
        large[f"top__n{n}__f{f}__seed{seed}"] = {
            "n": n, "fraction": f, "seed": seed,
            "generator": "np.random.default_rng(seed).standard_normal(n, dtype=np.float32)",
            "k": round(f * n), "output_sha256": sha(q), "sorted_idx_sha256": sha(nz),
            "nnz": int(nz.shape[0])}
        del g, q, nz
    manifest["large"] = large

    np.savez_compressed(os.path.join(OUT, "golden_codec.npz"), **arrays)
    with open(os.path.join(OUT, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print(f"wrote {len(manifest['cases'])} cases, {len(large)} large digests")


if __name__ == "__main__":
    main()
