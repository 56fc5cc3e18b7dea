"""Full-model parity on the GPU against fixtures produced by running the
reference code (tests/golden/make_golden.py).

Gate (BASELINE.json north star): generated node-type logits within 1e-3 fp32 of
the reference CPU path on identical inputs.  Gradients (incl. the WGAN-GP
second-order term) within 1e-3 relative (L2).  One full train step (config #1,
sanity; and a 4-building reduced config) with the CPU RNG replayed: losses
within 1e-3 relative, parameters after the Adam steps within 2e-3 absolute
(Adam's first steps move every parameter by ~lr = 2e-4 regardless of the
gradient's size, so sign flips of near-zero gradients bound the difference).
Per-parameter gradient checks use ``grads_close``: relative 1e-3 with a floor of
1e-6 x the whole gradient's norm (exactly-zero gradients are rounding noise).
"""
import pytest
import torch

from parity_util import _FixedUniform, grads_close, load_fixture, tiny_config, vgan_batches
from vgan.config import Configuration
from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
from vgan.trainer import Trainer

pytestmark = pytest.mark.gpu


def _models(cfg, fx_g, fx_d):
    G = VoxelGNNGenerator(cfg, 17, 12)
    D = VoxelGNNDiscriminator(cfg, 17, 12)
    G.load_state_dict(fx_g)
    D.load_state_dict(fx_d)
    return G, D


def test_forward_eval_logits_within_1e3(cuda):
    f = load_fixture("forward_eval.pt")
    cfg = Configuration()
    G, D = _models(cfg, f["G"], f["D"])
    G.eval()
    D.eval()
    loc, vox = vgan_batches(f["batch"])
    with torch.no_grad():
        logits, hard, soft = G(loc, vox, f["z"].cuda(), noise=f["gumbel_noise"].cuda())
        d_real = D(loc, vox, vox.types_onehot.unsqueeze(0))
        d_hard = D(loc, vox, hard.unsqueeze(0))
    assert (logits.cpu() - f["logits"]).abs().max().item() < 1e-3
    assert (soft.cpu() - f["label_soft"]).abs().max().item() < 1e-3
    agree = (hard.cpu().argmax(1) == f["label_hard"].argmax(1)).float().mean().item()
    assert agree > 0.999
    assert (d_real.cpu() - f["d_real"]).abs().max().item() < 1e-3
    assert (d_hard.cpu() - f["d_hard"]).abs().max().item() < 1e-3


def test_discriminator_loss_and_second_order_grads(cuda):
    f = load_fixture("forward_eval.pt")
    cfg = Configuration()
    G, D = _models(cfg, f["G"], f["D"])
    G.eval()
    D.eval()
    loc, vox = vgan_batches(f["batch"])
    with torch.no_grad():
        _, hard, soft = G(loc, vox, f["z"].cuda(), noise=f["gumbel_noise"].cuda())
    tr = Trainer(G, D, None, None, None, None, cfg)
    tr.rng = _FixedUniform(f["gp_eps"].cuda())
    tr.adam_d.zero_grad()
    d_loss = tr._compute_discriminator_loss(loc, vox, hard.unsqueeze(0), soft.unsqueeze(0))
    d_loss.backward()
    assert abs(d_loss.item() - float(f["d_loss"])) < 1e-3 * max(1.0, abs(float(f["d_loss"])))
    ok, worst, total = grads_close({k: p.grad for k, p in D.named_parameters()}, f["d_grads"])
    assert ok, (worst, total)


def test_generator_loss_and_grads(cuda):
    f = load_fixture("forward_eval.pt")
    cfg = Configuration()
    G, D = _models(cfg, f["G"], f["D"])
    G.eval()
    D.eval()
    loc, vox = vgan_batches(f["batch"])
    tr = Trainer(G, D, None, None, None, None, cfg)
    tr.adam_g.zero_grad()
    logits, hard, _ = G(loc, vox, f["z"].cuda(), noise=f["gumbel_noise"].cuda())
    g_loss = tr._compute_generator_loss(loc, vox, logits, hard.unsqueeze(0))
    g_loss.backward()
    assert abs(g_loss.item() - float(f["g_loss"])) < 1e-3 * max(1.0, abs(float(f["g_loss"])))
    ok, worst, total = grads_close({k: p.grad for k, p in G.named_parameters()}, f["g_grads"])
    assert ok, (worst, total)


@pytest.mark.parametrize("name", ["step_sanity.pt", "step_tiny.pt"])
def test_full_step_matches_reference(cuda, name):
    f = load_fixture(name)
    cfg = Configuration(sanity_checking=(name == "step_sanity.pt"))
    if name == "step_tiny.pt":
        tiny_config(cfg)
    cfg.runtime["rng"] = "host"  # replay the reference's CPU draws
    G, D = _models(cfg, f["G0"], f["D0"])
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    tr = Trainer(G, D, None, og, od, None, cfg)
    loc, vox = vgan_batches(f["batch"])
    torch.manual_seed(int(f["step_seed"]))
    out = tr.step(loc, vox)
    d_ref = f["d_losses"].float()
    assert torch.allclose(out["d_losses"].cpu(), d_ref, rtol=1e-3, atol=1e-3), (out["d_losses"], d_ref)
    assert abs(out["g_loss"].item() - float(f["g_loss"][0])) < 1e-3 * max(1.0, abs(float(f["g_loss"][0])))
    for ref_sd, mod in ((f["G1"], G), (f["D1"], D)):
        sd = mod.state_dict()
        worst = max((sd[k].cpu() - v).abs().max().item() for k, v in ref_sd.items())
        assert worst < 2e-3
        moved = sum(((sd[k].cpu() - v).abs() < 1e-5).sum().item() for k, v in ref_sd.items())
        total = sum(v.numel() for v in ref_sd.values())
        assert moved / total > 0.95  # nearly every parameter lands on the reference value
