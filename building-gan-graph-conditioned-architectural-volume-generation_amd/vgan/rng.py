"""Random draws of the training step, with two interchangeable sources.

The reference consumes the CPU default generator in a fixed order per step
(``trainer.py:459-502``): z = randn(1, N, Z) before each G forward, one
Bernoulli(0.8) dropout mask per encoder block (``nn.Dropout`` at
``models.py:75,85,195,205``), one Exp(1) draw for the Gumbel noise
(``F.gumbel_softmax``, ``models.py:150``) and eps = rand(N, 1) for the gradient
penalty (``trainer.py:298``).

* ``RNG("host")`` draws exactly those tensors, with the same ops and shapes, on
  the CPU default generator and copies them to the device -- the GPU path then
  sees bit-identical randomness to the reference CPU run (parity mode).
* ``RNG("device")`` draws them on the GPU generator (fast mode; hipGraph-safe).
"""
from __future__ import annotations

from typing import Sequence

import torch


class RNG:
    def __init__(self, mode: str = "device"):
        if mode not in ("device", "host"):
            raise ValueError("RNG mode must be 'device' or 'host'")
        self.mode = mode

    def _dev(self, device):
        return torch.device("cpu") if self.mode == "host" else device

    def _out(self, t: torch.Tensor, device) -> torch.Tensor:
        return t.to(device, non_blocking=True) if self.mode == "host" else t

    def normal(self, shape: Sequence[int], device) -> torch.Tensor:
        return self._out(torch.randn(*shape, device=self._dev(device)), device)

    def uniform(self, shape: Sequence[int], device) -> torch.Tensor:
        return self._out(torch.rand(*shape, device=self._dev(device)), device)

    def exponential(self, shape: Sequence[int], device) -> torch.Tensor:
        return self._out(torch.empty(*shape, device=self._dev(device)).exponential_(), device)

    def keep_mask(self, shape: Sequence[int], p: float, device) -> torch.Tensor:
        """Dropout multiplier: Bernoulli(1 - p) / (1 - p), as ATen's CPU dropout."""
        noise = torch.empty(*shape, device=self._dev(device)).bernoulli_(1 - p)
        noise.div_(1 - p)
        return self._out(noise, device)
