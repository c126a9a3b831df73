"""Bind the MI355X codec into an importable OpenMSFTL tree.

    import openmsftl_amd.integration as fi
    fi.install()            # before `import ftl.experiment` / `driver.run_main`

What it binds, and why each name (reference file:line):

* ``ftl.compression`` and ``ftl.compression.compression`` -> :mod:`openmsftl_amd.compression`:
  the two import paths of ``Compression`` (experiment.py:7, agents/client.py:8).  Modules
  that already bound the reference class by name are re-pointed too.
* ``ftl.gradient_aggregation.aggregation.FedAvg`` -> :class:`openmsftl_amd.gar.FedAvg`: the
  NAME ``Aggregator.__get_gar`` resolves when an aggregator is built (aggregation.py:15
  ``from .gar import FedAvg``, read at aggregation.py:47-48).  Rebinding ``gar.FedAvg`` alone
  changes nothing: ``aggregation.py`` holds its own reference to the class.
* ``Aggregator.aggregate_grads`` -> :func:`openmsftl_amd.aggregation.aggregate_grads` (the G
  build and the GAR reduction, aggregation.py:54-78); the reference method stays reachable as
  ``Aggregator._ref_aggregate_grads`` and still serves ``pc_analysis`` (randomized SVD).
  ``DGAggregator`` calls ``Aggregator.aggregate_grads`` by name (aggregation.py:188-207), so it
  is covered.  A GAR without ``aggregate_packets`` (``fed_spectral_avg``) receives the host G
  it expects.

``ftl.agents`` is imported before ``ftl.gradient_aggregation`` (importing the
latter first is a circular import, server.py:11 <-> aggregation.py:11).  Nothing here touches
the GPU: the device is resolved on the first ``aggregate_grads`` call.
"""
from __future__ import annotations

import sys

from . import aggregation, compression, gar


def install(aggregator: bool = True, devices=None):
    """Swap the codec (and by default the aggregator's hot path) into ``ftl``.  Returns the
    patched ``ftl.gradient_aggregation.aggregation`` module (or None with aggregator=False).
    ``devices``: the GPUs the streamed aggregation fans out over when an aggregator's config
    names none ("all", a count or a list of indices).  Left out (None), an earlier setting is
    kept; the initial default is the current device only (multi-GPU fan-out
    is opt-in, ``install(devices="all")``)."""
    if devices is not None:
        aggregation.DEFAULT_DEVICES = devices
    sys.modules["ftl.compression"] = compression                  # experiment.py:7
    sys.modules["ftl.compression.compression"] = compression      # client.py:8
    for name in ("ftl.agents.client", "ftl.experiment"):          # already imported: re-point
        mod = sys.modules.get(name)
        if mod is not None and hasattr(mod, "Compression"):
            mod.Compression = compression.Compression
    if not aggregator:
        return None
    import ftl.agents  # noqa: F401  (import order)
    import ftl.gradient_aggregation.aggregation as ref_agg
    ref_agg.FedAvg = gar.FedAvg                                   # aggregation.py:15, 47-48
    cls = ref_agg.Aggregator
    if "_ref_aggregate_grads" not in cls.__dict__:
        cls._ref_aggregate_grads = cls.aggregate_grads
    cls.aggregate_grads = aggregation.aggregate_grads
    cls.agg_path = None
    cls.agg_draws = None
    return ref_agg


def installed() -> bool:
    """True when ``install()`` has bound the device path into the loaded ``ftl`` modules."""
    ref_agg = sys.modules.get("ftl.gradient_aggregation.aggregation")
    return (sys.modules.get("ftl.compression.compression") is compression and ref_agg is not None
            and ref_agg.FedAvg is gar.FedAvg
            and ref_agg.Aggregator.aggregate_grads is aggregation.aggregate_grads)
