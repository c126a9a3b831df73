"""NumPy restatement of the flat-layout staging — TEST INFRASTRUCTURE (oracle).

Restates ``ftl/models/model_helper.py:11-13`` (``flatten_params``: concatenation of the
row-major ``flatten()`` of every parameter in ``parameters()`` order),
``model_helper.py:16-35`` (``dist_weights_to_model`` / ``dist_grads_to_model``: the inverse
slice-by-offset scatter) and ``ftl/agents/client.py:52-54`` (the client update
``grad = current_weights - updated_model_weights`` in np.float32, then
``current_weights = updated_model_weights``).  Pure NumPy; parity is exact by construction
(copies and one IEEE fp32 subtraction per element).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def flatten_params(params: Sequence[np.ndarray]) -> np.ndarray:
    """model_helper.py:13."""
    return np.concatenate([np.asarray(w).flatten() for w in params])


def dist_weights_to_model(weights: np.ndarray, shapes: Sequence[Tuple[int, ...]]) -> List[np.ndarray]:
    """model_helper.py:16-23 (returns the new parameter arrays instead of writing a model)."""
    out, offset = [], 0
    for shp in shapes:
        size = int(np.prod(shp)) if len(shp) else 1
        out.append(weights[offset:offset + size].reshape(shp).copy())
        offset += size
    return out


def client_step_delta(current_weights: np.ndarray, params: Sequence[np.ndarray]):
    """client.py:52-54 -> (grad, new current_weights)."""
    updated = flatten_params(params)
    return current_weights - updated, updated
