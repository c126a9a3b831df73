"""Device flat-layout staging (ftl/models/model_helper.py:11-35; agents/client.py:44,52-53).

The reference flattens every parameter to a host NumPy vector after each client step
(``flatten_params``), forms the client's update ``grad = current_weights - updated_weights``
(client.py:52-53) and later scatters the aggregate back into the model
(``dist_grads_to_model`` / ``dist_weights_to_model``).  Here the same layout lives on the GPU
and one HIP launch (``fc_flat_stage``) does flatten + delta, so the gradient the codec
consumes never leaves the device.  Element order and fp32 arithmetic match the reference
(``np.concatenate`` of ``flatten()``-ed parameters; np.float32 subtraction).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch

from . import _lib as L
from .codec import _require_cuda_f32, _stream, _vp


class FlatLayout:
    """Offsets of a parameter list in the flat vector (``model.parameters()`` order)."""

    def __init__(self, parameters: Iterable[torch.Tensor]):
        self.params: List[torch.Tensor] = [p for p in parameters]
        if not self.params:
            raise ValueError("no parameters")
        dev = self.params[0].device
        for p in self.params:
            if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev:
                raise TypeError("parameters must be contiguous float32 tensors on one GPU")
        sizes = [p.numel() for p in self.params]
        offs = [0]
        for s in sizes:
            offs.append(offs[-1] + s)
        self.n, self.max_size, self.device = offs[-1], max(sizes), dev
        self._offs = torch.tensor(offs, dtype=torch.int64).to(dev)
        self._refresh()

    def _refresh(self):
        self._ptrs = torch.tensor([p.data.data_ptr() for p in self.params], dtype=torch.int64).to(self.device)

    def _run(self, flat, grad, scatter):
        lib = L.load()
        _require_cuda_f32(flat, "flat", align=4)
        if grad is not None:
            _require_cuda_f32(grad, "grad", align=4)
        L.check(lib.fc_flat_stage(_vp(self._ptrs), _vp(self._offs), len(self.params), self.max_size,
                                  _vp(flat), _vp(grad), int(scatter), _stream(self.device)),
                "fc_flat_stage")

    def flatten(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """model_helper.py:11-13 ``flatten_params`` (device result)."""
        if out is None:
            out = torch.empty(self.n, dtype=torch.float32, device=self.device)
        self._run(out, None, False)
        return out

    def client_delta(self, current_weights: torch.Tensor,
                     grad: Optional[torch.Tensor] = None) -> torch.Tensor:
        """client.py:52-54: grad = current_weights - flatten_params(learner); current_weights
        is updated in place to the new flat weights (one pass)."""
        if grad is None:
            grad = torch.empty(self.n, dtype=torch.float32, device=self.device)
        self._run(current_weights, grad, False)
        return grad

    def scatter(self, flat: torch.Tensor) -> None:
        """model_helper.py:16-23 ``dist_weights_to_model``: parameters <- flat."""
        self._run(flat, None, True)
