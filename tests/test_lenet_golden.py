"""LeNet-shape goldens made by the reference itself (tests/golden/make_golden_lenet.py):

* flat-layout staging (model_helper.py:11-35, client.py:52-53) — the oracle
  (CPU) and ``openmsftl_amd.model_helper.FlatLayout`` (GPU, fc_flat_stage) against the
  reference's own flatten_params / client delta / dist_grads_to_model / dist_weights_to_model
  bytes on the reference LeNet's 8 parameters (431,080 floats);
* BASELINE configs[0]: one 4-client FedAVG round on LeNet-sized gradients with compression
  enabled (top / rand / dropout-unbiased, client_config.json:45-51), reference Compression ->
  Aggregator.aggregate_grads -> FedAvg — the oracle (CPU) and the device Aggregator (GPU) give
  the reference's compressed rows and ``agg_grad`` byte for byte, and leave the global NumPy
  RNG where the reference leaves it.
"""
import hashlib
import importlib.util
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR
from oracle import compression_oracle as co
from oracle import gar_oracle as go
from oracle import model_helper_oracle as mho

MAN = json.load(open(os.path.join(GOLDEN_DIR, "manifest_lenet.json")))
_spec = importlib.util.spec_from_file_location("make_golden_lenet",
                                               os.path.join(GOLDEN_DIR, "make_golden_lenet.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


class _Client:
    def __init__(self, cid, grad, C):
        self.client_id, self.grad, self.C = cid, grad, C


# ---- CPU: the oracle pinned to the reference's bytes -------------------------------------
def test_oracle_flat_staging_matches_reference():
    w0, w1, _ = MG.inputs()
    f = MAN["flat"]
    current = mho.flatten_params(w0)
    assert sha(current) == f["flatten_w0"]
    grad, updated = mho.client_step_delta(current, w1)
    assert sha(updated) == f["flatten_w1"]
    assert sha(grad) == f["client_grad"]
    shapes = [tuple(s) for s in MAN["lenet_shapes"]]
    assert sha(np.concatenate([p.ravel() for p in mho.dist_weights_to_model(grad, shapes)])) \
        == f["grads_to_model"]
    assert sha(np.concatenate([p.ravel() for p in mho.dist_weights_to_model(current, shapes)])) \
        == f["weights_to_model"]


@pytest.mark.parametrize("name", sorted(MG.ROUND_CODECS))
def test_oracle_configs0_round_matches_reference(name):
    _, _, grads = MG.inputs()
    r = MAN["round"][name]
    np.random.seed(r["seed"])
    rows = [co.compress(r["cfg"], g) for g in grads]             # aggregation.py:61-63
    assert int(np.random.randint(0, 2 ** 31 - 1)) == r["rng_next"]
    G = go.build_dense_G(rows, np.float32)
    assert [sha(x) for x in G] == r["rows"]
    assert sha(go.FedAvgOracle({}).aggregate(G)) == r["agg_grad"]


# ---- GPU: the HIP path against the same bytes ---------------------------------------------
@pytest.mark.gpu
def test_flat_layout_lenet_matches_reference():
    torch = pytest.importorskip("torch")
    from openmsftl_amd.model_helper import FlatLayout
    w0, w1, _ = MG.inputs()
    f = MAN["flat"]
    params = [torch.from_numpy(w).cuda() for w in w0]
    lay = FlatLayout(params)
    current = lay.flatten()
    assert sha(current.cpu().numpy()) == f["flatten_w0"]
    for p, w in zip(params, w1):                                  # "the optimizer step"
        p.copy_(torch.from_numpy(w))
    grad = lay.client_delta(current)                              # client.py:52-53
    assert sha(grad.cpu().numpy()) == f["client_grad"]
    assert sha(current.cpu().numpy()) == f["flatten_w1"]
    lay.scatter(grad)                                             # dist_grads_to_model's bytes
    assert sha(np.concatenate([p.cpu().numpy().ravel() for p in params])) == f["grads_to_model"]
    lay.scatter(torch.from_numpy(np.concatenate([w.ravel() for w in w0])).cuda())
    assert sha(np.concatenate([p.cpu().numpy().ravel() for p in params])) == f["weights_to_model"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MG.ROUND_CODECS))
def test_device_aggregator_configs0_round(name):
    """BASELINE configs[0] through the device Aggregator (streamed top-k packets for 'top',
    the drop-in Compression per client for rand / dropout)."""
    pytest.importorskip("torch")
    from openmsftl_amd import Compression
    from openmsftl_amd.aggregation import Aggregator
    _, _, grads = MG.inputs()
    r = MAN["round"][name]
    C = Compression(r["cfg"])
    agg = Aggregator({"aggregation_scheme": "fed_avg"})
    np.random.seed(r["seed"])
    agg.aggregate_grads([_Client(i, g, C) for i, g in enumerate(grads)])
    assert int(np.random.randint(0, 2 ** 31 - 1)) == r["rng_next"]
    assert agg.agg_path == "stream"                  # every configs[0] codec streams
    assert str(agg.agg_grad.dtype) == r["agg_dtype"]
    assert sha(agg.agg_grad) == r["agg_grad"]
    if agg.curr_G is not None:
        assert [sha(x) for x in agg.curr_G.cpu().numpy()] == r["rows"]
