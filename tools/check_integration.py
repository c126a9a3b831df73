"""Apply INTEGRATION.md's recipe to the REFERENCE tree and check what it bound (build
container only: /root/reference does not exist on the GPU box; no GPU call is made).

    PYTHONDONTWRITEBYTECODE=1 python tools/check_integration.py [/root/reference]

Checks, against OpenMSFTL's own modules:
  * both import paths of Compression resolve to the device drop-in (experiment.py:7,
    agents/client.py:8), and the class a Client was built with is the device one;
  * make_aggregator (server.py:52-56 -> aggregation.py:220-244) builds an Aggregator whose
    GAR is the device FedAvg (the name __get_gar resolves, aggregation.py:15,47-48), for the
    conventional and the DGA (softmax) aggregator;
  * Aggregator.aggregate_grads (and so DGAggregator's explicit call, aggregation.py:188-207) is
    the device function; the reference one is kept for pc_analysis;
  * torch never initialised a GPU (torch.cuda.is_initialized() stays False).
Prints one JSON line; exits non-zero on the first failed check.
"""
from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(ref: str = "/root/reference") -> dict:
    if not os.path.isdir(os.path.join(ref, "ftl")):
        raise SystemExit(f"no OpenMSFTL tree at {ref}")
    sys.path.insert(0, ROOT)
    sys.path.insert(0, ref)
    import torch
    import openmsftl_amd.integration as fi
    from openmsftl_amd import aggregation, compression, gar

    ref_agg = fi.install()
    checks = {}
    import ftl.compression as c1
    from ftl.compression.compression import Compression as C2
    import ftl.agents.client as ref_client
    checks["compression_paths"] = c1.Compression is compression.Compression and C2 is compression.Compression
    checks["client_binds_device_codec"] = ref_client.Compression is compression.Compression
    A = ref_agg.make_aggregator({"aggregation_scheme": "fed_avg"}, model=None, optimizer=None,
                                clip_val=None, lr_scheduler=None)
    checks["aggregator_class_is_reference"] = type(A) is ref_agg.Aggregator
    checks["gar_is_device_fedavg"] = isinstance(A.gar, gar.FedAvg)
    checks["aggregate_grads_is_device"] = ref_agg.Aggregator.aggregate_grads is aggregation.aggregate_grads
    checks["reference_kept_for_pc_analysis"] = callable(getattr(ref_agg.Aggregator, "_ref_aggregate_grads", None))
    D = ref_agg.make_aggregator({"aggregation_scheme": "fed_avg",
                                 "dga_config": {"type": "softmax", "T": 1.0}},
                                model=None, optimizer=None, clip_val=None, lr_scheduler=None)
    checks["dga_gar_is_device_fedavg"] = type(D) is ref_agg.DGAggregator and isinstance(D.gar, gar.FedAvg)
    # experiment.py:53-57 builds each client's codec from `ftl.compression.Compression`
    Cl = ref_client.Client(client_id=0, C=c1.Compression({"compression_function": "top",
                                                          "fraction_coordinate": 0.1}))
    checks["client_codec_is_device"] = isinstance(Cl.C, compression.Compression)
    checks["installed"] = fi.installed()
    checks["no_gpu_initialised"] = not torch.cuda.is_initialized()
    ok = all(checks.values())
    print(json.dumps({"ok": ok, "checks": checks}), flush=True)
    if not ok:
        raise SystemExit(1)
    return checks


if __name__ == "__main__":
    main(*sys.argv[1:])
