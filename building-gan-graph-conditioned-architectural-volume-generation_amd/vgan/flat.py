"""Flat parameter / gradient buffers and the one-kernel Adam over them.

Each model's parameters are re-seated as views into ONE contiguous fp32 buffer
(G: 274,185 floats = 1.10 MB, D: 15,665 = 63 KB) and their ``.grad`` as views
into one flat gradient buffer.  Each parameter starts on a 128-byte boundary
(ALIGN floats; the gaps stay zero in both buffers, and Adam keeps them zero):
the GEMMs take their float4 operand loads only from 16-byte-aligned weights,
and a packed layout left most weights after the GAT stack's 1- and 2-wide
attention vectors misaligned.  Consequences:

* ``optimizer.step()`` (``trainer.py:481,495``) is one ``vg_adam`` launch over
  the buffer instead of a Python loop over ~100 tensors;
* zero_grad is one memset;
* the data-parallel all-reduce (``vgan.dist``) is one RCCL call per backward on
  the whole gradient -- the right bucket size for xGMI at these sizes.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional

import torch
import torch.nn as nn

from . import ops


# floats: every parameter's view starts on a 128-byte boundary (VGAN_FLAT_ALIGN=1: packed, for A/B runs)
ALIGN = max(1, int(os.environ.get("VGAN_FLAT_ALIGN", "32")))


def _padded(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class FlatParams:
    def __init__(self, module: nn.Module):
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("module has no trainable parameters")
        dev = params[0].device
        total = sum(_padded(p.numel()) for p in params)
        self.param = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.params: List[nn.Parameter] = params
        off = 0
        for p in params:
            n = p.numel()
            self.param[off:off + n].copy_(p.detach().reshape(-1))
            p.data = self.param[off:off + n].view_as(p)
            p.grad = self.grad[off:off + n].view_as(p)
            off += _padded(n)
        self.numel = total  # buffer length, padding included
        self.num_params = sum(p.numel() for p in params)

    def zero_grad(self, device: bool = True) -> None:
        """``device=False``: the caller zeroes the buffer in its own launch
        (vg_iter_begin); only the parameters' .grad views are checked."""
        if device:
            self.grad.zero_()
        # re-seat views an external set_to_none (or a .grad assignment) dropped;
        # the identity check is cheap, the pointer check runs only on a change
        views = getattr(self, "_views", None)
        if views is not None and all(p.grad is v for p, v in zip(self.params, views)):
            return
        for p in self.params:
            if p.grad is None or p.grad.data_ptr() != self._view_ptr(p):
                self._reseat_grad(p)
        self._views = [p.grad for p in self.params]

    def live_mask(self) -> torch.Tensor:
        """Bool mask over the buffer: True on parameter elements, False on the
        alignment gaps."""
        m = torch.zeros(self.numel, dtype=torch.bool, device=self.param.device)
        for p in self.params:
            off = self._offset(p)
            m[off:off + p.numel()] = True
        return m

    def _offset(self, p) -> int:
        return (p.data.data_ptr() - self.param.data_ptr()) // 4

    def _view_ptr(self, p) -> int:
        return self.grad.data_ptr() + 4 * self._offset(p)

    def _reseat_grad(self, p) -> None:
        off = self._offset(p)
        if p.grad is not None:
            self.grad[off:off + p.numel()].copy_(p.grad.reshape(-1))
        p.grad = self.grad[off:off + p.numel()].view_as(p)


class FlatAdam(torch.optim.Optimizer):
    """torch.optim.Adam semantics (amsgrad/maximize not supported) over a FlatParams.

    When built ``from_optimizer`` it mirrors that optimizer's hyper-parameters
    at every step, so an LR scheduler attached to the caller's optimizer
    (``CosineAnnealingLR`` at ``train.py:38``) keeps driving the learning rate.
    """

    def __init__(self, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, source: Optional[torch.optim.Optimizer] = None):
        super().__init__(flat.params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self.flat = flat
        self.source = source
        self.exp_avg = torch.zeros_like(flat.param)
        self.exp_avg_sq = torch.zeros_like(flat.param)
        self.step_count = 0
        dev = flat.param.device
        # device-resident step count and learning rate: a captured hipGraph
        # replays correct bias corrections and follows the LR scheduler
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float64, device=dev)
        self._lr_host = float(lr)

    @classmethod
    def from_optimizer(cls, flat: FlatParams, opt: Optional[torch.optim.Optimizer]) -> "FlatAdam":
        if opt is None:
            return cls(flat)
        g = opt.param_groups[0]
        if len(opt.param_groups) != 1 or g.get("amsgrad", False) or g.get("maximize", False):
            raise NotImplementedError("FlatAdam mirrors a single-group, non-amsgrad Adam")
        return cls(flat, lr=g["lr"], betas=g["betas"], eps=g["eps"], weight_decay=g.get("weight_decay", 0.0),
                   source=opt)

    def hyper(self) -> Dict[str, object]:
        g = (self.source or self).param_groups[0]
        return {"lr": g["lr"], "betas": g["betas"], "eps": g["eps"], "weight_decay": g.get("weight_decay", 0.0)}

    def sync_lr(self) -> None:
        """Copy the (scheduler-driven) learning rate to the device; call outside
        graph capture (the trainer does it before every step)."""
        lr = float(self.hyper()["lr"])
        if lr != self._lr_host:
            self.lr_t.fill_(lr)
            self._lr_host = lr

    @torch.no_grad()
    def step(self, closure=None, counted: bool = False):
        """``counted``: the device step count was already incremented for this
        update (vg_iter_begin at the start of the iteration)."""
        self.step_count += 1
        if self.source is not None:
            # what the LR scheduler's wrapper of source.step() records: this
            # update IS the caller's optimizer.step() (the scheduler otherwise
            # warns that it stepped first)
            self.source._opt_called = True
        h = self.hyper()
        b1, b2 = h["betas"]
        if not self.flat.param.is_cuda:
            raise RuntimeError("FlatAdam runs on the HIP path only")
        if not torch.cuda.is_current_stream_capturing():
            self.sync_lr()
        if not counted:
            self.step_t.add_(1)
        ops.adam_flat_dev(self.flat.param, self.flat.grad, self.exp_avg, self.exp_avg_sq, b1, b2, h["eps"],
                          h["weight_decay"], self.lr_t, self.step_t)
        return None

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def state_dict_flat(self) -> Dict[str, object]:
        return {"step": int(self.step_t.item()), "exp_avg": self.exp_avg.clone(),
                "exp_avg_sq": self.exp_avg_sq.clone()}

    # ------------------------------------------- torch.optim.Adam state format
    # Checkpoints keep the reference's keys (trainer.py:731-733 saves
    # optimizer.state_dict() of a torch Adam and :632-633 loads it back), so
    # the flat moments are written into / read from that per-parameter form.
    def _slices(self, params):
        for p in params:
            off = self.flat._offset(p)
            if not 0 <= off < self.flat.numel:
                raise ValueError("optimizer parameter is not in this flat buffer")
            yield p, off, p.numel()

    def export_to(self, opt: Optional[torch.optim.Optimizer]) -> None:
        """Write step / exp_avg / exp_avg_sq into ``opt.state`` (a torch Adam
        over the same parameters; this optimizer itself when ``opt`` is None)
        in torch.optim.Adam's layout: a float32 scalar tensor step and
        per-parameter moment tensors."""
        opt = self if opt is None else opt
        step = float(self.step_t.item())
        for group in opt.param_groups:
            for p, off, n in self._slices(group["params"]):
                if step == 0:
                    opt.state.pop(p, None)  # torch Adam keeps no state before its first step
                    continue
                opt.state[p] = {"step": torch.tensor(step, dtype=torch.float32),
                                "exp_avg": self.exp_avg[off:off + n].view_as(p).clone(),
                                "exp_avg_sq": self.exp_avg_sq[off:off + n].view_as(p).clone()}

    def import_from(self, opt: Optional[torch.optim.Optimizer]) -> None:
        """Read a torch Adam state (after ``opt.load_state_dict``) into the
        flat moments and the device step counter."""
        opt = self if opt is None else opt
        steps = set()
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            for group in opt.param_groups:
                for p, off, n in self._slices(group["params"]):
                    st = opt.state.get(p)
                    if not st:
                        steps.add(0)
                        continue
                    steps.add(int(float(st["step"])))
                    self.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1))
                    self.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
        if len(steps) > 1:
            raise ValueError(f"parameters of one optimizer at different Adam steps {sorted(steps)}")
        step = steps.pop() if steps else 0
        self.step_t.fill_(step)
        self.step_count = step
        self._lr_host = None  # the restored learning rate goes to the device now
        self.sync_lr()

    def state_dict(self):
        """torch.optim.Adam-format state (loadable by a torch Adam over the same
        parameters)."""
        self.export_to(None)
        sd = super().state_dict()
        for g in sd["param_groups"]:
            g.update({k: v for k, v in dict(amsgrad=False, maximize=False, foreach=None, capturable=False,
                                            differentiable=False, fused=None).items() if k not in g})
        return sd

    def load_state_dict(self, state_dict) -> None:
        super().load_state_dict(state_dict)
        self.import_from(None)


def param_iter(modules: Iterable[nn.Module]):
    for m in modules:
        yield from m.parameters()
