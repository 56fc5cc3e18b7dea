"""vg_linear_chain: the critic's decoder chains (models.py:273-279) in one
launch per pass -- forward 64-32-16-8-1 (ReLU between), tangent 64-32-16-8 and
adjoint 1-8-16-32 (ReLU derivative from the forward outputs) -- against a
torch fp32 restatement of the per-layer products, and the critic engine with
the chains against its per-layer GEMMs (vg_gemm)."""
from __future__ import annotations

import pytest
import torch

from parity_util import rel_err
from test_critic_gpu import _RecRNG, _engine_setup
from vgan import _lib
from vgan._lib import LIB, ptr

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


def _run(cuda, widths, wt, acts, rows, bias=True, seed=0, bf16=False):
    """Run the chain, then each layer's f64 reference from the previous
    layer's STORED output (bf16: both operands rounded first)."""
    g = torch.Generator(device=cuda).manual_seed(seed)
    x = torch.randn(rows, widths[0], device=cuda, generator=g)
    layers, params = [], []
    for i in range(len(widths) - 1):
        a, b = widths[i], widths[i + 1]
        W = torch.randn(*((b, a) if not wt else (a, b)), device=cuda, generator=g) / a ** 0.5
        bb = torch.randn(b, device=cuda, generator=g) if bias else None
        aux = torch.randn(rows, b, device=cuda, generator=g)
        out = torch.full((rows, b), float("nan"), device=cuda)
        params.append((W, bb, aux, out))
        layers.append(dict(weight=W.data_ptr(), bias=bb.data_ptr() if bb is not None else None, aux=aux.data_ptr(),
                           ld_aux=b, out=out.data_ptr(), ld_out=b, w_trans=wt, act=acts[i]))
    with _lib.gemm_precision_scope("bf16" if bf16 else "f32"):
        assert _lib.linear_chain(ptr(x), widths[0], rows, widths, layers, _lib.stream_handle(cuda))
    torch.cuda.synchronize()
    outs, inp = [], x
    for i, (W, bb, aux, out) in enumerate(params):
        Wd = _bf(W).double() if bf16 else W.double()
        xin = _bf(inp).double() if bf16 else inp.double()
        y = xin @ (Wd.t() if not wt else Wd)
        if bb is not None:
            y = y + bb.double()
        if acts[i] == 1:
            y = torch.relu(y)
        elif acts[i] == 3:
            y = torch.where(aux.double() > 0, y, torch.zeros_like(y))
        outs.append((out, y))
        inp = out
    return outs


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("rows", [1, 63, 64, 1000, 12_345])
@pytest.mark.parametrize("case", ["forward", "tangent", "adjoint"])
def test_linear_chain_matches_fp32_layers(cuda, rows, case, bf16):
    """bf16: against f64 products of the bf16-rounded operands (each layer's
    f32 output rounded again as the next layer's operand)."""
    if case == "forward":
        outs = _run(cuda, [64, 32, 16, 8, 1], 0, [1, 1, 1, 0], rows, bias=True, seed=rows, bf16=bf16)
    elif case == "tangent":
        outs = _run(cuda, [64, 32, 16, 8], 0, [3, 3, 3], rows, bias=False, seed=rows + 1, bf16=bf16)
    else:
        outs = _run(cuda, [1, 8, 16, 32], 1, [3, 3, 3], rows, bias=False, seed=rows + 2, bf16=bf16)
    for out, y in outs:  # every layer's output stored, f32 FMAs vs f64
        assert torch.isfinite(out).all()
        assert (out.double() - y).abs().max().item() <= 1e-5 * max(1.0, y.abs().max().item())


def test_linear_chain_rejects_other_widths(cuda):
    x = torch.zeros(100, 48, device=cuda)
    W = torch.zeros(48, 48, device=cuda)
    layers = [dict(weight=W.data_ptr(), out=x.data_ptr(), ld_out=48)] * 2
    assert not _lib.linear_chain(ptr(x), 48, 100, [48, 48, 48], layers, _lib.stream_handle(cuda))


@pytest.mark.parametrize("training", [True, False])
def test_critic_engine_with_decoder_chains(cuda, training, monkeypatch):
    """Loss and D gradient with the decoder chains (one launch per pass)
    against the per-layer GEMMs: f32 rounding (FMA order vs MFMA order)."""
    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6, 7), seed=29)
    D.train(training)
    hd, sd = hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0)
    calls = []
    orig = LIB.vg_linear_chain

    def counted(*a):
        calls.append(1)
        return orig(*a)

    monkeypatch.setattr(LIB, "vg_linear_chain", counted)
    out = {}
    for chain in (True, False):
        monkeypatch.setattr(_lib, "_CHAIN", chain)
        calls.clear()
        flat.zero_grad()
        loss = eng.loss_and_grad(loc, vox, hd, sd, _RecRNG(6))
        torch.cuda.synchronize()
        out[chain] = (loss.item(), flat.grad.clone(), len(calls))
    assert out[True][2] == 4 and out[False][2] == 0  # passes A, B, C, D
    assert abs(out[True][0] - out[False][0]) <= 1e-5 * max(1.0, abs(out[False][0]))
    assert rel_err(out[True][1], out[False][1]) < 1e-4
