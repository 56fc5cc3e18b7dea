"""The critic iteration issued from C++ (vg_critic_loss_and_grad,
include/vgan.h) against the Python critic engine it restates
(vgan/critic.py CriticEngine.loss_and_grad, trainer.py:291-332 + :476-479):
same launches, same order, same arguments -- so d_loss, the gradient penalty
and every discriminator gradient must be BIT-identical, in f32 and in bf16,
eagerly and inside a recorded step graph."""
import pytest
import torch

import vgan.critic as critic_mod
from vgan.config import Configuration
from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
from vgan.synth import SyntheticDataset
from vgan.trainer import Trainer

pytestmark = pytest.mark.gpu


def _trainer(cuda, precision, buildings):
    cfg = Configuration()
    cfg.DEVICE = cuda
    cfg.runtime["rng"] = "device"
    cfg.runtime["precision"] = precision
    torch.manual_seed(cfg.SEED)
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    tr = Trainer(G, D, None, torch.optim.Adam(G.parameters(), lr=2e-4, betas=cfg.BETAS),
                 torch.optim.Adam(D.parameters(), lr=2e-4, betas=cfg.BETAS), None, cfg)
    ds = SyntheticDataset(buildings, seed=99)
    loc, vox = ds.batch(range(buildings))
    return tr, loc.to(cuda), vox.to(cuda)


def _iteration(tr, loc, vox, hard, soft, native, counter):
    """one critic loss + backward from zeroed gradients and a fixed device-RNG state"""
    old = critic_mod._NATIVE
    critic_mod._NATIVE = native
    try:
        for p in tr.discriminator.parameters():
            if p.grad is not None:
                p.grad.zero_()
        tr.rng.reset()
        tr.rng._iter(hard.device).fill_(counter)
        calls = tr.critic.__dict__.get("native_calls", 0)
        loss = tr.critic.loss_and_grad(loc, vox, hard, soft, tr.rng)
        torch.cuda.synchronize()
        used = tr.critic.__dict__.get("native_calls", 0) > calls
        return (loss.clone(), tr.critic.last_gp.clone(),
                {k: p.grad.clone() for k, p in tr.discriminator.named_parameters()}, used)
    finally:
        critic_mod._NATIVE = old


@pytest.mark.parametrize("precision,buildings", [("f32", 32), ("f32", 4), ("bf16", 8)])
def test_native_critic_bit_identical_to_python_engine(cuda, precision, buildings):
    tr, loc, vox = _trainer(cuda, precision, buildings)
    from vgan._lib import gemm_precision_scope

    with gemm_precision_scope(precision):
        with torch.no_grad():
            _, hard, soft = tr._generate(loc, vox)
        hard, soft = hard.clone(), soft.clone()
        for counter in (7, 8):
            l_py, gp_py, g_py, used_py = _iteration(tr, loc, vox, hard, soft, False, counter)
            l_nat, gp_nat, g_nat, used_nat = _iteration(tr, loc, vox, hard, soft, True, counter)
            assert used_nat and not used_py
            assert torch.isfinite(l_nat).all() and torch.equal(l_nat, l_py) and torch.equal(gp_nat, gp_py)
            for k in g_py:
                assert torch.equal(g_nat[k], g_py[k]), k
            assert any(float(v.abs().max()) > 0 for v in g_nat.values())


def test_native_critic_in_recorded_step_graphs(cuda):
    """step_graphed (captured critic iterations) and step_fresh (one recorded
    critic body updated per batch) with the native engine equal the same
    steps through the Python engine, bitwise, over three steps."""
    def run(native, mode):
        old = critic_mod._NATIVE
        critic_mod._NATIVE = native
        try:
            tr, loc, vox = _trainer(cuda, "f32", 8)
            out = []
            for _ in range(3):
                r = tr.step_graphed(loc, vox) if mode == "graphed" else tr.step_fresh(loc, vox)
                out.append(torch.cat([r["d_losses"].reshape(-1), r["g_loss"].reshape(-1)]).clone())
            torch.cuda.synchronize()
            return torch.stack(out), torch.cat([p.detach().reshape(-1) for p in tr.discriminator.parameters()]), \
                tr.critic.__dict__.get("native_calls", 0)
        finally:
            critic_mod._NATIVE = old

    for mode in ("graphed", "fresh"):
        l_py, p_py, c_py = run(False, mode)
        l_nat, p_nat, c_nat = run(True, mode)
        assert c_py == 0 and c_nat > 0, (mode, c_py, c_nat)
        assert torch.equal(l_py, l_nat), mode
        assert torch.equal(p_py, p_nat), mode
