"""Dense layers of the path on the hand-written f32 MFMA GEMMs.

``Linear`` is ``torch.nn.Linear`` (same parameters, same initialisation, same
state_dict keys) whose forward, input gradient and weight/bias gradient run on
``vg_gemm`` / ``vg_gemm_tn`` (csrc/gemm.hip).  Library GEMMs cost 19 us at
minimum per call on these tall-skinny shapes and 77-692 us for the weight
gradient (profiles/r01_*).  With ``create_graph=True`` (the WGAN-GP second
order) the backward is built from the differentiable matmuls _MMnt / _MMnn /
_MMtn (same kernels, each one's adjoints expressed with the others), so double
backward keeps working and stays on the MFMA path.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.autograd import Function

from . import ops


class _MMnt(Function):
    """C = A B^T on vg_gemm; closed under differentiation with _MMnn / _MMtn."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return ops.gemm(a, b, True)

    @staticmethod
    def backward(ctx, gc):
        a, b = ctx.saved_tensors
        ga = _MMnn.apply(gc, b) if ctx.needs_input_grad[0] else None
        gb = _MMtn.apply(gc, a) if ctx.needs_input_grad[1] else None
        return ga, gb


class _MMnn(Function):
    """C = A B."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return ops.gemm(a, b, False)

    @staticmethod
    def backward(ctx, gc):
        a, b = ctx.saved_tensors
        ga = _MMnt.apply(gc, b) if ctx.needs_input_grad[0] else None
        gb = _MMtn.apply(a, gc) if ctx.needs_input_grad[1] else None
        return ga, gb


class _MMtn(Function):
    """C = A^T B (split-K over the long dimension)."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return ops.gemm_tn(a, b, want_colsum=False)[0]

    @staticmethod
    def backward(ctx, gc):
        a, b = ctx.saved_tensors
        ga = _MMnt.apply(b, gc) if ctx.needs_input_grad[0] else None
        gb = _MMnn.apply(a, gc) if ctx.needs_input_grad[1] else None
        return ga, gb


class _LinearFn(Function):
    """y = act(x W^T + b) on vg_gemm; act is ACT_NONE or ACT_RELU (the
    [Linear, ReLU] blocks of the discriminator's MLPs, models.py:166-175, with
    the ReLU in the GEMM epilogue)."""

    @staticmethod
    def forward(ctx, x, weight, bias, act):
        if act not in (ops.ACT_NONE, ops.ACT_RELU):
            raise ValueError("_LinearFn: act must be ACT_NONE or ACT_RELU")
        y = ops.gemm(x, weight, True, bias, act)
        ctx.act = act
        if act == ops.ACT_RELU:
            ctx.save_for_backward(x, weight, y)
        else:
            ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, gy):
        if ctx.act == ops.ACT_RELU:
            x, weight, y = ctx.saved_tensors
            if torch.is_grad_enabled():
                gy = gy * (y > 0).to(gy.dtype)  # differentiable in gy (create_graph)
            else:
                gy = torch.ops.aten.threshold_backward(gy, y, 0)
            return _linear_backward(ctx, gy, saved=(x, weight)) + (None,)
        return _linear_backward(ctx, gy) + (None,)


def _linear_backward(ctx, gy, saved=None, needs=None):
    """(g_x, g_weight, g_bias) of y = x W^T (+ b) for _LinearFn / _LinAttFn /
    _LinearLNActFn (``saved`` = (x, weight) and ``needs`` = the three
    needs-grad flags when the ctx holds more)."""
    x, weight = saved if saved is not None else ctx.saved_tensors
    needs = needs if needs is not None else ctx.needs_input_grad
    gx = gw = gb = None
    if torch.is_grad_enabled():  # create_graph: differentiable MFMA matmuls
        gy = gy.contiguous()
        if needs[0]:
            gx = _MMnn.apply(gy, weight)
        if needs[1]:
            gw = _MMtn.apply(gy, x)
        if ctx.has_bias and needs[2]:
            gb = gy.sum(0)
        return gx, gw, gb
    gy = gy.contiguous()
    if needs[0]:
        hint = ops.gn_hint_for(x)  # x is a GraphNorm output: its backward's partials from this GEMM
        gx = ops.gemm_gn_bwd(gy, weight, hint) if hint is not None else ops.gemm(gy, weight, False)
    pw, pb = ctx.params
    if needs[1] and ops._direct(pw, pb):  # accumulate into .grad directly
        ops.gemm_tn_into(gy, x, pw.grad, pb.grad if ctx.has_bias else None)
        return gx, None, None
    if needs[1] or (ctx.has_bias and needs[2]):
        gw, gb = ops.gemm_tn(gy, x, want_colsum=ctx.has_bias)
    return gx, gw, (gb if ctx.has_bias else None)


class _LinAttFn(Function):
    """GATConv.lin (no bias) with the attention projections h . att_src,
    h . att_dst as two extra, non-differentiable outputs (their dependence on
    h and att is differentiated inside ops.gat_conv)."""

    @staticmethod
    def forward(ctx, x, weight, att_src, att_dst):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = False
        ctx.params = (weight, None)
        h, a_s, a_d = ops.lin_att(x, weight, att_src, att_dst)
        ctx.mark_non_differentiable(a_s, a_d)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for a_s / a_d
        return h, a_s, a_d

    @staticmethod
    def backward(ctx, gh, _g_as, _g_ad):
        if gh is None:
            return None, None, None, None
        gx, gw, _ = _linear_backward(ctx, gh)
        return gx, gw, None, None


class _LinearLNActFn(Function):
    """leaky_relu(LayerNorm(x W^T + b)) with the LayerNorm in the GEMM's
    epilogue (vg_gemm_ln_act); the backward is the LayerNorm+activation
    backward (vg_ln_act_bwd) followed by the Linear backward."""

    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, eps, slope):
        from ._lib import LIB, check, dense, ptr, stream_handle

        n, k = x.shape
        m = weight.shape[0]
        dev = x.device
        y = torch.empty(n, m, dtype=torch.float32, device=dev)
        save = any(ctx.needs_input_grad[:5])
        h = torch.empty_like(y) if save else None
        mean = torch.empty(n, dtype=torch.float32, device=dev) if save else None
        rstd = torch.empty(n, dtype=torch.float32, device=dev) if save else None
        check(dense("vg_gemm_ln_act")(ptr(x), k, ptr(weight), n, m, k, ptr(bias), ptr(gamma), ptr(beta), float(eps),
                                 float(slope), ptr(h), ptr(y), ptr(mean), ptr(rstd), stream_handle(dev)),
              "vg_gemm_ln_act")
        ctx.eps, ctx.slope = eps, slope
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)
        ctx.ln_params = (gamma, beta)
        if save:
            ctx.save_for_backward(x, weight, h, gamma, beta, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, h, gamma, beta, mean, rstd = ctx.saved_tensors
        needs = ctx.needs_input_grad
        if torch.is_grad_enabled():  # create_graph: differentiable restatement of both halves
            bias = ctx.params[1]
            ins = [x, weight, bias, gamma, beta]
            with torch.enable_grad():
                leaves = [None if t is None else t.detach().requires_grad_(bool(nd))
                          for t, nd in zip(ins, needs[:5])]
                y = ops.ln_act(_LinearFn.apply(leaves[0], leaves[1], leaves[2], ops.ACT_NONE), leaves[3], leaves[4],
                               ctx.eps, ctx.slope)
                want = [t for t in leaves if t is not None and t.requires_grad]
                got = iter(torch.autograd.grad(y, want, gy, create_graph=True, allow_unused=True))
            return tuple(next(got) if t is not None and t.requires_grad else None for t in leaves) + (None, None)
        gh, g_gamma, g_beta = ops.ln_act_backward(h, gamma, beta, ctx.eps, ctx.slope, mean, rstd, gy,
                                                  ctx.ln_params, want_params=needs[3] or needs[4])
        gx, gw, gb = _linear_backward(ctx, gh, saved=(x, weight), needs=needs[:3])
        return gx, gw, gb, g_gamma, g_beta, None, None


def linear_ln_act(x: torch.Tensor, weight: torch.Tensor, bias, gamma: torch.Tensor, beta: torch.Tensor,
                  eps: float = 1e-5, slope: float = 0.2) -> torch.Tensor:
    """[Linear -> LayerNorm -> LeakyReLU] in one launch (M <= 128 outputs)."""
    if not x.is_cuda:
        raise RuntimeError("vgan HIP ops require tensors on a ROCm device (no CPU fallback)")
    return _LinearLNActFn.apply(x.contiguous(), weight, bias, gamma, beta, eps, slope)


def linear_att(x: torch.Tensor, weight: torch.Tensor, att_src: torch.Tensor, att_dst: torch.Tensor):
    """(x W^T, projections on att_src / att_dst) -- one launch (vg_gat_lin_att)."""
    if not x.is_cuda:
        raise RuntimeError("vgan HIP ops require tensors on a ROCm device (no CPU fallback)")
    return _LinAttFn.apply(x.contiguous(), weight, att_src, att_dst)


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None) -> torch.Tensor:
    if not x.is_cuda:
        raise RuntimeError("vgan HIP ops require tensors on a ROCm device (no CPU fallback)")
    if x.dim() == 2:
        return _LinearFn.apply(x.contiguous(), weight, bias, ops.ACT_NONE)
    y = _LinearFn.apply(x.reshape(-1, x.shape[-1]).contiguous(), weight, bias, ops.ACT_NONE)
    return y.reshape(*x.shape[:-1], y.shape[-1])


class Linear(nn.Linear):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.weight, self.bias)


class MLP(nn.Sequential):
    """nn.Sequential of the reference's [Linear, (LayerNorm,) activation]
    blocks (same children, same state_dict keys); every Linear -> LayerNorm
    -> LeakyReLU triple runs as one GEMM with the LayerNorm in its epilogue
    (or GEMM + vg_ln_act_fwd past 128 outputs), every Linear -> ReLU pair as
    one GEMM with the ReLU in its epilogue."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return run_blocks(list(self), x)


def run_blocks(mods, x: torch.Tensor) -> torch.Tensor:
    """MLP.forward over a list of children (also used for an MLP's tail)."""
    i = 0
    while i < len(mods):
        m = mods[i]
        if (isinstance(m, nn.Linear) and i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
                and x.dim() == 2):  # ReLU in the GEMM epilogue
            x = _LinearFn.apply(x.contiguous(), m.weight, m.bias, ops.ACT_RELU)
            i += 2
            continue
        if (isinstance(m, nn.Linear) and i + 2 < len(mods) and isinstance(mods[i + 1], nn.LayerNorm)
                and isinstance(mods[i + 2], nn.LeakyReLU) and len(mods[i + 1].normalized_shape) == 1
                and mods[i + 1].elementwise_affine):
            ln = mods[i + 1]
            if m.out_features <= 128 and x.dim() == 2:  # LayerNorm in the GEMM epilogue
                x = linear_ln_act(x, m.weight, m.bias, ln.weight, ln.bias, ln.eps, mods[i + 2].negative_slope)
            else:
                x = ops.ln_act(linear(x, m.weight, m.bias), ln.weight, ln.bias, ln.eps,
                               mods[i + 2].negative_slope)
            i += 3
        else:
            x = m(x)
            i += 1
    return x
