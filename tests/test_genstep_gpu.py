"""The explicit generator iteration (vgan/genstep.py) against the autograd path
it replaces (trainer.py:483-491 through the differentiable HIP ops), which
tests/test_b32_gpu.py and tests/test_models_gpu.py pin to the reference.

From identical parameters and device-RNG state both draw the same z, dropout
masks and Gumbel noise; the forwards run the same kernels, so the labels and
the loss are bit-identical.  The gradients differ only in the grouping of
fused reductions (the last encoder GraphNorm's column partials come from the
decoder GEMM's epilogue, the discriminator's label gradient from a GEMM over
the label columns only): whole gradient within 1e-5 relative, every parameter
within 1e-4 of its own norm (plus a floor at 1e-6 of the whole gradient's norm
for the exactly-zero GATConv-bias gradients); with bf16 operands within their
own rounding (5e-3 whole; 5e-2 per parameter with a floor at 1e-4 of the
whole gradient's norm for the 1-2 channel blocks' products, sums of 12.7k
bf16-rounded terms that cancel).
"""
import pytest
import torch

from parity_util import grads_close
from vgan.config import Configuration
from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
from vgan.synth import SyntheticDataset
from vgan.trainer import Trainer

pytestmark = pytest.mark.gpu


def _trainer(cfg, gen, seed=777):
    cfg.runtime["gen"] = gen
    torch.manual_seed(seed)
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    return Trainer(G, D, None, og, od, None, cfg)


def _grads(tr):
    flat = tr.flat_g
    return {k: flat.grad[flat._offset(p):flat._offset(p) + p.numel()].clone()
            for k, p in tr.generator.named_parameters()}


def _cfg(cuda, precision="f32"):
    cfg = Configuration()
    cfg.DEVICE = str(cuda)
    cfg.runtime["rng"] = "device"
    cfg.runtime["precision"] = precision
    return cfg


@pytest.mark.parametrize("batch,precision", [(4, "f32"), (32, "f32"), (32, "bf16")])
def test_engine_matches_autograd_iteration(cuda, batch, precision):
    from vgan._lib import gemm_precision_scope

    loc, vox = SyntheticDataset(batch, seed=31).batch(range(batch))
    loc, vox = loc.to(cuda), vox.to(cuda)
    a, b = _trainer(_cfg(cuda, precision), "engine"), _trainer(_cfg(cuda, precision), "autograd")
    assert a.gen_engine is not None and b.gen_engine is None
    for it in range(2):  # the second draws from the advanced device counter
        outs = []
        for tr in (a, b):
            with gemm_precision_scope(precision):
                g_loss, hard = tr._gen_iteration(loc, vox)
            outs.append((g_loss.detach().clone(), hard.detach().clone(), _grads(tr)))
        torch.cuda.synchronize()
        (la, ha, ga), (lb, hb, gb) = outs
        assert torch.equal(ha, hb), it
        assert abs(float(la) - float(lb)) <= 1e-6 * max(1.0, abs(float(lb))), (it, float(la), float(lb))
        # bf16: a last-bit f32 difference upstream can round an operand to the
        # neighbouring bf16 value (2^-8 relative) in the weight-gradient
        # products; the 1-2 channel blocks in the middle of the encoder show it most
        rtol, total_rtol, floor = (1e-4, 1e-5, 1e-6) if precision == "f32" else (5e-2, 5e-3, 1e-4)
        ok, worst, total = grads_close(ga, gb, rtol=rtol, total_rtol=total_rtol, floor=floor)
        scale = float(torch.cat([v.reshape(-1) for v in gb.values()]).norm())
        wk = worst[0]
        print(f"batch {batch} {precision} iteration {it}: loss {float(la):.6f}; engine vs autograd G gradient "
              f"relative error {total:.2e}, worst parameter {worst}: |diff| {float((ga[wk] - gb[wk]).norm()):.3e}, "
              f"|grad| {float(gb[wk].norm()):.3e}, |whole| {scale:.3e}")
        assert ok, (it, worst, total)


def test_engine_steps_track_autograd_steps(cuda):
    """Full eager steps (critic iterations + generator iteration + Adam) with
    the engine and with autograd, each from the same state: they agree to
    rounding (Adam turns the exactly-zero bias gradients' rounding noise into
    +-lr moves either way, hence the bound on the fraction of elements that
    moved apart)."""
    cfg = _cfg(cuda)
    loc, vox = SyntheticDataset(8, seed=5).batch(range(8))
    loc, vox = loc.to(cuda), vox.to(cuda)
    a, b = _trainer(cfg, "engine"), _trainer(_cfg(cuda), "autograd")
    for k in range(3):
        oa, ob = a.step(loc, vox), b.step(loc, vox)
        torch.cuda.synchronize()
        print(f"step {k}: d_losses engine {oa['d_losses'].tolist()} autograd {ob['d_losses'].tolist()}")
        assert torch.allclose(oa["d_losses"], ob["d_losses"], rtol=1e-4, atol=1e-5), k
        assert abs(float(oa["g_loss"]) - float(ob["g_loss"])) <= 1e-4 * max(1.0, abs(float(ob["g_loss"]))), k
        d = (a.flat_g.param - b.flat_g.param).abs()
        print(f"step {k}: max |G param diff| {float(d.max()):.2e}, moved apart {float((d > 1e-6).float().mean()):.2e}")
        assert float(d.max()) <= 5e-4 and float((d > 1e-6).float().mean()) < 2e-3
        with torch.no_grad():  # the next step from identical state (no drift compounding)
            for x, y in zip(b._state_tensors(), a._state_tensors()):
                x.copy_(y)


def test_engine_inside_graph_capture(cuda):
    """step_graphed records the engine's iteration (no autograd inside the
    captured generator graph) and replays it like the eager step."""
    cfg = _cfg(cuda)
    loc, vox = SyntheticDataset(8, seed=6).batch(range(8))
    loc, vox = loc.to(cuda), vox.to(cuda)
    a, b = _trainer(cfg, "engine"), _trainer(_cfg(cuda), "engine")
    for k in range(3):
        oa, ob = a.step(loc, vox), b.step_graphed(loc, vox)
        torch.cuda.synchronize()
        assert torch.allclose(oa["d_losses"], ob["d_losses"], rtol=1e-4, atol=1e-5), k
        assert abs(float(oa["g_loss"]) - float(ob["g_loss"])) <= 1e-4 * max(1.0, abs(float(oa["g_loss"]))), k
        with torch.no_grad():
            for x, y in zip(b._state_tensors(), a._state_tensors()):
                x.copy_(y)
