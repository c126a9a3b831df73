"""Golden vectors for the aggregation rows of SURVEY.md §8 (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_agg.py

Runs the REFERENCE (read-only /root/reference; ``import ftl.agents`` first)
and records inputs and outputs of
  * ``FedAvg.aggregate`` (gar.py:32-56) on G matrices with signed zeros, denormal products that
    underflow to -0, and all-(-0) columns — pins the sign-of-zero semantics of gar.py:44;
  * ``Aggregator.__merge_gradient`` (aggregation.py:80-93) followed by ``FedAvg.aggregate``
    (the ``num_hierarchies > 0`` branch of aggregation.py:68-75), one and two stages, with a
    remainder absorbed by the last cluster.
Only data is written (``golden_agg.npz`` + ``manifest_agg.json``).
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
    from ftl.gradient_aggregation.aggregation import Aggregator
    from ftl.gradient_aggregation.gar import FedAvg
    return Aggregator, FedAvg


def signed_zero_G(M, n, seed):
    rng = np.random.default_rng(seed)
    G = (rng.standard_normal((M, n)) * 1e-3).astype(np.float32)
    sel = rng.uniform(size=(M, n))
    G[sel < 0.45] = -0.0
    G[(sel >= 0.45) & (sel < 0.55)] = 0.0
    G[(sel >= 0.55) & (sel < 0.65)] = -np.float32(1e-45)
    G[:, n - n // 16:] = -0.0                           # all-(-0) columns
    return G


def main():
    Aggregator, FedAvg = _import_reference()
    merge = Aggregator._Aggregator__merge_gradient       # (self, G, cluster_size); self unused
    arrays, cases = {}, {}

    def add(name, **kw):
        meta = {}
        for k, v in kw.items():
            if isinstance(v, np.ndarray):
                arrays[f"{name}|{k}"] = v
            else:
                meta[k] = v
        cases[name] = meta

    for M, n, seed in ((1, 4096, 1), (6, 4096, 2), (12, 20011, 3)):
        G = signed_zero_G(M, n, seed)
        agg = FedAvg({"aggregation_scheme": "fed_avg"}).aggregate(G=G, client_ids=np.arange(M))
        add(f"fedavg_signed__M{M}__n{n}", M=M, n=n, G=G, output=agg)

    import contextlib
    import io
    for M, n, sizes, seed in ((10, 4096, [3], 4), (17, 5000, [4, 2], 5), (8, 3001, [8], 6),
                              (9, 2048, [2, 2], 7)):
        rng = np.random.default_rng(seed)
        G = (rng.standard_normal((M, n)) * 10.0 ** rng.uniform(-4, -1, (M, 1))).astype(np.float32)
        G[rng.uniform(size=(M, n)) < 0.5] = 0.0          # sparse rows, as compressed clients send
        G[:, :64] = -0.0
        H = G
        with contextlib.redirect_stdout(io.StringIO()):   # __merge_gradient prints progress
            for cs in sizes:
                H = merge(None, H, cs)
        agg = FedAvg({"aggregation_scheme": "fed_avg"}).aggregate(G=H, client_ids=np.arange(H.shape[0]))
        add(f"hier__M{M}__n{n}__c{'-'.join(map(str, sizes))}", M=M, n=n,
            cluster_size_list=sizes, G=G, merged=H, output=agg)

    np.savez_compressed(os.path.join(OUT, "golden_agg.npz"), **arrays)
    with open(os.path.join(OUT, "manifest_agg.json"), "w") as fh:
        json.dump({"cases": cases}, fh, indent=1, sort_keys=True)
    print(f"wrote {len(cases)} aggregation cases")


if __name__ == "__main__":
    main()
