"""Golden digests on LeNet shapes (build container only; BASELINE configs[0]).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_lenet.py

Runs the REFERENCE (read-only /root/reference; ``import ftl.agents`` first) and
records SHA-256 digests (``manifest_lenet.json``; inputs are regenerated from the seeds here by
``inputs()``, which the tests import):

  * flat-layout staging: the reference ``LeNet`` (ftl/models/lenet.py, 431,080
    parameters) loaded with seeded weights, then ``flatten_params`` (model_helper.py:11-13), a
    client update ``grad = current_weights - flatten_params(learner)`` after the weights move
    (client.py:52-53), ``dist_grads_to_model`` (model_helper.py:26-35) and
    ``dist_weights_to_model`` (:16-23) — every parameter's bytes in ``parameters()`` order;
  * one configs[0] round (driver.py with client_config.json: 4 clients, LeNet-sized gradients,
    compression enabled, FedAVG): reference ``Compression`` per client (top f = 0.1, the
    config's fraction_coordinate; rand f = 0.1 and dropout-unbiased p = 0.1, the config's
    dropout_p, under a seeded global np.random) through the reference
    ``Aggregator.aggregate_grads`` (aggregation.py:54-78) -> ``FedAvg`` (gar.py:32-56): the
    digest of every compressed row and of ``agg_grad``, and the RNG state after the round.
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

LENET_SHAPES = [(20, 1, 5, 5), (20,), (50, 20, 5, 5), (50,), (500, 800), (500,), (10, 500), (10,)]
N_LENET = 431_080
ROUND_CODECS = {
    "top": {"compression_function": "top", "fraction_coordinate": 0.1},
    "rand": {"compression_function": "rand", "fraction_coordinate": 0.1},
    "dropout-unbiased": {"compression_function": "dropout-unbiased", "dropout_p": 0.1},
}
ROUND_SEED = 1234                 # np.random.seed before the round (rand / dropout draws)


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def inputs():
    """Seeded inputs: LeNet weights before / after a client step (per parameter, float32) and
    the 4 clients' LeNet-sized gradients (client.py:53 flat float32)."""
    rng = np.random.default_rng(431)
    w0 = [(rng.standard_normal(s) * 0.05).astype(np.float32) for s in LENET_SHAPES]
    w1 = [(w + (rng.standard_normal(w.shape) * 1e-3).astype(np.float32)).astype(np.float32)
          for w in w0]
    grads = [(rng.standard_normal(N_LENET) * 10.0 ** rng.uniform(-4, -2)).astype(np.float32)
             for _ in range(4)]
    return w0, w1, grads


class _Client:
    def __init__(self, cid, grad, C):
        self.client_id, self.grad, self.C = cid, grad, C


def main():
    sys.path.insert(0, REF)
    import torch
    import ftl.agents  # noqa: F401  (import order)
    from ftl.compression import Compression
    from ftl.gradient_aggregation.aggregation import Aggregator
    from ftl.models import model_helper as mh
    from ftl.models.lenet import LeNet

    w0, w1, grads = inputs()
    man = {"lenet_shapes": [list(s) for s in LENET_SHAPES], "n": N_LENET}
    # ---- flat-layout staging ----
    model = LeNet()
    assert [tuple(p.shape) for p in model.parameters()] == LENET_SHAPES
    with torch.no_grad():
        for p, w in zip(model.parameters(), w0):
            p.copy_(torch.from_numpy(w))
    current = mh.flatten_params(learner=model)                       # model_helper.py:13
    with torch.no_grad():
        for p, w in zip(model.parameters(), w1):                     # "the optimizer step"
            p.copy_(torch.from_numpy(w))
    updated = mh.flatten_params(learner=model)
    grad = current - updated                                         # client.py:53
    mh.dist_grads_to_model(grad, model.parameters())                 # model_helper.py:26-35
    grads_back = np.concatenate([p.grad.numpy().ravel() for p in model.parameters()])
    mh.dist_weights_to_model(current, model.parameters())            # model_helper.py:16-23
    weights_back = np.concatenate([p.data.numpy().ravel() for p in model.parameters()])
    man["flat"] = {"flatten_w0": sha(current), "flatten_w1": sha(updated),
                   "client_grad": sha(grad), "grads_to_model": sha(grads_back),
                   "weights_to_model": sha(weights_back), "dtype": str(grad.dtype)}
    # ---- configs[0] round: 4 clients, compression enabled, FedAVG ----
    man["round"] = {}
    for name, cfg in ROUND_CODECS.items():
        C = Compression(cfg)
        clients = [_Client(i, g, C) for i, g in enumerate(grads)]
        agg = Aggregator({"aggregation_scheme": "fed_avg"}, None, None, None, None)
        np.random.seed(ROUND_SEED)
        agg.aggregate_grads(clients)
        rng_next = int(np.random.randint(0, 2 ** 31 - 1))
        man["round"][name] = {"cfg": cfg, "seed": ROUND_SEED, "rng_next": rng_next,
                              "rows": [sha(r) for r in agg.curr_G],
                              "G_dtype": str(agg.curr_G.dtype),
                              "agg_grad": sha(agg.agg_grad), "agg_dtype": str(agg.agg_grad.dtype)}
        print(f"[round {name}] agg {man['round'][name]['agg_grad'][:16]}", flush=True)
    with open(os.path.join(OUT, "manifest_lenet.json"), "w") as fh:
        json.dump(man, fh, indent=1, sort_keys=True)
    print("wrote manifest_lenet.json", flush=True)


if __name__ == "__main__":
    main()
