"""Golden vectors for the float64 path, produced by the REFERENCE itself (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_f64.py

float64 gradients reach the codec after RandomGaussian with noise_scale == 0
(attack_models.py:105-106); G then takes that dtype (aggregation.py:61).  DGA's weight
estimators set float64 ``gradient_weights`` on the GAR (aggregation.py:181-198), which promotes
``G * w`` (gar.py:44) to float64 for a float32 G too.  This script imports OpenMSFTL from
/root/reference (``import ftl.agents`` first) and records, as data only
(``golden_f64.npz`` + ``manifest_f64.json``):
  * ``Compression.compress`` on float64 inputs: top / rand / dropout-* (seeded legacy RNG, the
    RNG state after the call), ties, +-0, NaN/inf;
  * ``Aggregator.aggregate_grads`` (aggregation.py:54-78) end to end on float64 clients (flat
    and hierarchical) and on float32 clients with float64 GAR weights.
The GPU box never runs this.
"""
from __future__ import annotations

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
    from ftl.gradient_aggregation.aggregation import Aggregator
    return Compression, Aggregator


class _Client:
    """The three attributes aggregate_grads reads (aggregation.py:61-63, 76)."""

    def __init__(self, cid, grad, C):
        self.client_id, self.grad, self.C = cid, grad, C


def gaussian64(n, seed, scale=1.0):
    return np.random.default_rng(seed).standard_normal(n) * scale


def main():
    Compression, Aggregator = _import_reference()
    manifest = {"reference": "microsoft/OpenMSFTL @ /root/reference", "numpy": np.__version__,
                "cases": {}}
    arrays = {}

    def add(name, **kw):
        meta = {}
        for key, val in kw.items():
            if isinstance(val, np.ndarray):
                arrays[f"{name}|{key}"] = val
            else:
                meta[key] = val
        manifest["cases"][name] = meta

    # ---- compress on float64 ----------------------------------------------------------------
    rng = np.random.default_rng(64)
    inputs = {"gauss_1000": gaussian64(1000, 1), "gauss_16385": gaussian64(16385, 2, 1e-3),
              "ties_smallint_4096": rng.integers(-6, 7, 4096).astype(np.float64)}
    g = gaussian64(1000, 3)
    g[[5, 400, 999]] = np.nan
    g[[7, 8]] = np.inf
    g[9] = -np.inf
    g[10:20] = -0.0
    inputs["nan_inf_zero_1000"] = g
    for iname, g in inputs.items():
        arrays[f"input|{iname}"] = g                          # each input stored once
        for f in (0.1, 0.01, 0.5, 1.0, 0.0):
            q = Compression({"compression_function": "top", "fraction_coordinate": f}).compress(g.copy())
            add(f"top|{iname}|f{f}", codec="top", fraction=f, input=iname, output=q, out_dtype=str(q.dtype))
    for iname in ("gauss_1000", "gauss_16385", "nan_inf_zero_1000"):
        g = inputs[iname]
        for f in (0.1, 0.5):
            seed = 700 + len(g)
            np.random.seed(seed)
            q = Compression({"compression_function": "rand", "fraction_coordinate": f}).compress(g)
            after = int(np.random.randint(0, 2**31 - 1))
            add(f"rand|{iname}|f{f}", codec="rand", fraction=f, seed=seed, rng_next=after,
                input=iname, output=q, out_dtype=str(q.dtype))
        for fn in ("dropout-biased", "dropout-unbiased"):
            for p in (0.1, 0.3, 0.5):
                seed = 900 + len(g)
                np.random.seed(seed)
                q = Compression({"compression_function": fn, "dropout_p": p}).compress(g)
                after = int(np.random.randint(0, 2**31 - 1))
                add(f"{fn}|{iname}|p{p}", codec=fn, p=p, seed=seed, rng_next=after,
                    input=iname, output=q, out_dtype=str(q.dtype))

    # ---- Aggregator.aggregate_grads end to end -------------------------------------------------
    def run_agg(name, grads, cfg_codec, agg_cfg, weights=None, seed=0):
        np.random.seed(seed)
        clients = [_Client(i, g, Compression(cfg_codec)) for i, g in enumerate(grads)]
        A = Aggregator(agg_cfg, model=None, optimizer=None, clip_val=None, lr_scheduler=None)
        if weights is not None:
            A.gar.gradient_weights = weights
        A.aggregate_grads(clients)
        add(name, codec=cfg_codec["compression_function"], M=len(grads), n=int(grads[0].shape[0]),
            agg_cfg=agg_cfg, seed=seed, grads=np.stack(grads),
            weights=weights if weights is not None else np.zeros(0), output=A.agg_grad,
            out_dtype=str(A.agg_grad.dtype))

    M, n = 10, 2048
    g64 = [gaussian64(n, 100 + i, 10.0 ** (-1 - i % 3)) for i in range(M)]
    g32 = [x.astype(np.float32) for x in g64]
    flat = {"aggregation_scheme": "fed_avg"}
    hier = {"aggregation_scheme": "fed_avg", "num_hierarchies": 2, "cluster_size_list": [3, 2]}
    top = {"compression_function": "top", "fraction_coordinate": 0.1}
    for cname, cfg in (("top", top), ("full", {"compression_function": "full"}),
                       ("dropout-unbiased", {"compression_function": "dropout-unbiased",
                                             "dropout_p": 0.3})):
        run_agg(f"agg|f64|{cname}|flat", g64, cfg, flat, seed=11)
        run_agg(f"agg|f64|{cname}|hier", g64, cfg, hier, seed=12)
    # softmax-like float64 weights on float32 clients (DGA, aggregation.py:181-198)
    z = np.random.default_rng(5).standard_normal(M)
    w64 = np.exp(z) / np.exp(z).sum()
    run_agg("agg|f32w64|top|flat", g32, top, flat, weights=w64, seed=13)
    run_agg("agg|f32w64|full|flat", g32, {"compression_function": "full"}, flat, weights=w64, seed=14)
    run_agg("agg|f64w32|full|flat", g64, {"compression_function": "full"}, flat,
            weights=w64.astype(np.float32), seed=15)

    np.savez_compressed(os.path.join(OUT, "golden_f64.npz"), **arrays)
    with open(os.path.join(OUT, "manifest_f64.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print(f"wrote {len(manifest['cases'])} float64 cases")


if __name__ == "__main__":
    main()
