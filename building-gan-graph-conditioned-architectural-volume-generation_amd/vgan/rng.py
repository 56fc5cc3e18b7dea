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
* ``RNG("device")`` draws them on the GPU (fast mode; hipGraph-safe) from one
  counter-based Philox keyed by (seed, device iteration counter, call-site
  salt): z, eps and the Gumbel noise through ``vg_rng_fill`` (no torch
  generator inside the captured graphs, hence none of the two int64 seed /
  offset fills torch adds to every replay), each dropout mask as a
  ``DropSpec`` that the GraphNorm kernel materialises in-kernel -- no extra
  launches.  ``reset()`` at the start of every iteration
  body advances the device counter (one tiny launch, captured in the graph),
  so hipGraph replays draw fresh masks.
* ``RNG("fixed")`` (tests only) hands out the same seeded tensors for the k-th
  draw of every iteration body (``reset()`` at each body start), so an eager
  step and a hipGraph replay see identical randomness.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Dict, Sequence

import torch


@dataclass
class DropSpec:
    """A dropout mask to be drawn inside the consuming kernel."""
    p: float
    seed: int
    iter: torch.Tensor  # int64 [1] on the device
    salt: int
    shape: tuple


class RNG:
    def __init__(self, mode: str = "device", seed: Optional[int] = None):
        if mode not in ("device", "host", "fixed"):
            raise ValueError("RNG mode must be 'device', 'host' or 'fixed'")
        self.mode = mode
        # device mode: seeded from the CPU generator (torch.manual_seed(SEED + rank)
        # in the bench / DP ranks), so ranks draw different streams
        self.seed = (torch.initial_seed() if mode == "device" else 0) if seed is None else int(seed)
        self._k = 0
        self._fixed = {}
        self._salt = 0
        self._iters: Dict[torch.device, torch.Tensor] = {}
        self._early = 0  # resets before the device counter existed (it starts there)

    def reset(self, defer: bool = False):
        """Start of an iteration body (fixed draws restart; device masks advance).
        The device counter counts resets whenever it is created, so an eager
        body and a captured one draw the same numbers from the same state.
        ``defer``: the device counters are returned, not advanced -- the caller
        advances them in its own launch (vg_iter_begin)."""
        self._k = 0
        self._salt = 0
        if not self._iters:
            self._early += 1
        if defer:
            return list(self._iters.values())
        for t in self._iters.values():
            t.add_(1)
        return []

    def state_dict(self) -> Dict[str, int]:
        """Seed and device iteration counter (device mode): a resumed run
        continues the same stream of z / dropout / Gumbel / eps draws."""
        iters = [int(t.item()) for t in self._iters.values()]
        # no device counter yet: the value it will start from (resets so far count)
        start = getattr(self, "_pending_iter", 0) + self._early
        return {"mode": self.mode, "seed": int(self.seed), "iter": max(iters) if iters else start}

    def load_state_dict(self, state: Dict[str, int]) -> None:
        if state.get("mode") != self.mode:
            return  # another randomness source: nothing to continue
        self.seed = int(state["seed"])
        self._pending_iter = int(state["iter"])
        self._early = 0
        for t in self._iters.values():
            t.fill_(self._pending_iter)

    def _iter(self, device) -> torch.Tensor:
        device = torch.device(device)
        t = self._iters.get(device)
        if t is None:
            t = self._iters[device] = torch.full((1,), getattr(self, "_pending_iter", 0) + self._early,
                                                 dtype=torch.int64, device=device)
        return t

    def _fixed_draw(self, kind: str, shape, device, make):
        key = (self._k, kind, tuple(shape))
        self._k += 1
        t = self._fixed.get(key)
        if t is None:
            g = torch.Generator(device="cpu").manual_seed(self.seed * 1000003 + len(self._fixed))
            t = make(g).to(device)
            self._fixed[key] = t
        return t

    def _dev(self, device):
        return torch.device("cpu") if self.mode == "host" else device

    def _out(self, t: torch.Tensor, device) -> torch.Tensor:
        return t.to(device, non_blocking=True) if self.mode == "host" else t

    def _device_draw(self, kind: int, shape, device) -> torch.Tensor:
        """vg_rng_fill on (salt, the device iteration counter): no torch
        generator inside captured graphs, so replays need no seed / offset
        refills."""
        from ._lib import LIB, check, ptr, stream_handle

        device = torch.device(device)
        out = torch.empty(*shape, dtype=torch.float32, device=device)
        self._salt += 1
        check(LIB.vg_rng_fill(ptr(out), out.numel(), kind, int(self.seed) & ((1 << 64) - 1), ptr(self._iter(device)),
                              0x40000000 | self._salt, stream_handle(device)), "vg_rng_fill")
        return out

    def normal(self, shape: Sequence[int], device) -> torch.Tensor:
        if self.mode == "fixed":
            return self._fixed_draw("n", shape, device, lambda g: torch.randn(*shape, generator=g))
        if self.mode == "device" and torch.device(device).type == "cuda":
            return self._device_draw(0, shape, device)
        return self._out(torch.randn(*shape, device=self._dev(device)), device)

    def uniform(self, shape: Sequence[int], device) -> torch.Tensor:
        if self.mode == "fixed":
            return self._fixed_draw("u", shape, device, lambda g: torch.rand(*shape, generator=g))
        if self.mode == "device" and torch.device(device).type == "cuda":
            return self._device_draw(1, shape, device)
        return self._out(torch.rand(*shape, device=self._dev(device)), device)

    def uniform_spec(self, shape: Sequence[int], device):
        """Device mode: (seed, iteration counter, salt) of the uniform draw
        ``uniform(shape, device)`` would make -- for a kernel that draws it
        itself (vg_critic_input_drawn); None in the other modes."""
        if self.mode != "device" or torch.device(device).type != "cuda":
            return None
        self._salt += 1
        return int(self.seed) & ((1 << 64) - 1), self._iter(device), 0x40000000 | self._salt

    def exponential(self, shape: Sequence[int], device) -> torch.Tensor:
        if self.mode == "fixed":
            return self._fixed_draw("e", shape, device, lambda g: torch.empty(*shape).exponential_(generator=g))
        if self.mode == "device" and torch.device(device).type == "cuda":
            return self._device_draw(2, shape, device)
        return self._out(torch.empty(*shape, device=self._dev(device)).exponential_(), device)

    def keep_mask(self, shape: Sequence[int], p: float, device):
        """Dropout multiplier: Bernoulli(1 - p) / (1 - p), as ATen's CPU dropout
        (a ``DropSpec`` drawn in-kernel in device mode)."""
        if self.mode == "device":
            self._salt += 1
            return DropSpec(float(p), int(self.seed) & ((1 << 64) - 1), self._iter(device), self._salt, tuple(shape))
        if self.mode == "fixed":
            return self._fixed_draw("k", shape, device,
                                    lambda g: torch.empty(*shape).bernoulli_(1 - p, generator=g).div_(1 - p))
        noise = torch.empty(*shape, device=self._dev(device)).bernoulli_(1 - p)
        noise.div_(1 - p)
        return self._out(noise, device)
