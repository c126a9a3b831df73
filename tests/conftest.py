import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")


class Golden:
    def __init__(self):
        with open(os.path.join(GOLDEN_DIR, "manifest.json")) as fh:
            self.manifest = json.load(fh)
        self.arrays = np.load(os.path.join(GOLDEN_DIR, "golden_codec.npz"))

    def cases(self, prefix=""):
        return sorted(k for k in self.manifest["cases"] if k.startswith(prefix))

    def meta(self, name):
        return self.manifest["cases"][name]

    def input(self, name):
        return self.arrays[self.meta(name)["input"]]

    def arr(self, name, key):
        return self.arrays[f"{name}__{key}"]


_GOLDEN = None


def golden() -> Golden:
    global _GOLDEN
    if _GOLDEN is None:
        _GOLDEN = Golden()
    return _GOLDEN


@pytest.fixture(scope="session")
def gold():
    return golden()


def has_tie_at_boundary(g: np.ndarray, k: int) -> bool:
    """True when the k-th largest magnitude's tie group straddles the cut."""
    from oracle.packet_oracle import mag_key
    n = g.shape[0]
    if k <= 0 or k >= n:
        return False
    keys = np.sort(mag_key(g))[::-1]          # NaN is one key, above +inf
    return bool(keys[k - 1] == keys[k])


class AggGolden:
    """tests/golden/make_golden_agg.py: FedAvg sign-of-zero and hierarchical-merge cases."""

    def __init__(self):
        with open(os.path.join(GOLDEN_DIR, "manifest_agg.json")) as fh:
            self.manifest = json.load(fh)
        self.arrays = np.load(os.path.join(GOLDEN_DIR, "golden_agg.npz"))

    def cases(self, prefix=""):
        return sorted(k for k in self.manifest["cases"] if k.startswith(prefix))

    def meta(self, name):
        return self.manifest["cases"][name]

    def arr(self, name, key):
        return self.arrays[f"{name}|{key}"]


_AGG = None


def agg_golden() -> AggGolden:
    global _AGG
    if _AGG is None:
        _AGG = AggGolden()
    return _AGG
