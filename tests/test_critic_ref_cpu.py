"""The explicit four-pass critic gradient (tests/critic_ref.py) equals plain
double backward of the WGAN-GP critic loss, in float64 on the CPU."""
import torch

import critic_ref as C
from oracle import reference as R
from vgan.config import Configuration
from vgan.synth import SyntheticDataset


def _setup(seed=0, n_build=2):
    cfg = Configuration()
    torch.manual_seed(seed)
    D = R.Discriminator(cfg).double()
    P = {k: v.detach().clone() for k, v in D.state_dict().items()}
    loc, vox = SyntheticDataset(16, seed=seed + 1).batch(range(n_build))
    n = vox.x.shape[0]
    ei = vox.edge_index
    g = torch.Generator().manual_seed(seed + 2)
    mvx = torch.rand(n, 29, generator=g, dtype=torch.float64)
    types = torch.randint(0, 7, (n,), generator=g)
    real = F_onehot(types)
    hard = F_onehot(torch.randint(0, 7, (n,), generator=g))
    soft = torch.softmax(torch.randn(n, 7, generator=g, dtype=torch.float64) * 2, dim=1)
    eps = torch.rand(n, 1, generator=g, dtype=torch.float64)
    mix = eps * real + (1 - eps) * soft
    nb = 2 * cfg.DISCRIMINATOR_ENCODER_REPEAT
    units = {}
    for c in ("real", "fake", "mix"):
        keeps = [torch.bernoulli(torch.full((n, w), 0.8, dtype=torch.float64), generator=g) / 0.8
                 for w in R.gat_widths(cfg.DISCRIMINATOR_HIDDEN_DIM, cfg.DISCRIMINATOR_ENCODER_REPEAT)[1:]]
        units[c] = C.d_units(nb, 4, ei, n, keeps)
    x0s = {"real": torch.cat([mvx, real], 1), "fake": torch.cat([mvx, hard], 1), "mix": torch.cat([mvx, mix], 1)}
    return cfg, P, units, x0s


def F_onehot(t):
    return torch.nn.functional.one_hot(t, 7).to(torch.float64)


def test_four_pass_engine_equals_double_backward():
    cfg, P, units, x0s = _setup()
    lam = float(cfg.LAMBDA_GP)
    l1, gp1, g1 = C.run(units, x0s, slice(29, 36), lam, P)
    l2, gp2, g2 = C.autograd_loss(units, x0s, slice(29, 36), lam, P)
    assert abs(l1.item() - l2.item()) <= 1e-12 * max(1, abs(l2.item()))
    assert abs(gp1.item() - gp2.item()) <= 1e-12 * max(1, abs(gp2.item()))
    top = max(v.abs().max().item() for v in g2.values())
    for k in P:  # GAT biases feeding GraphNorm have exactly-zero gradients: global floor
        scale = g2[k].abs().max().item()
        assert (g1[k] - g2[k]).abs().max().item() <= 1e-10 * scale + 1e-12 * top, k


def test_chain_matches_oracle_discriminator():
    cfg, P, units, x0s = _setup()
    # same chain as oracle Discriminator forward (eval mode: keeps of ones)
    torch.manual_seed(0)
    D = R.Discriminator(cfg).double().eval()
    loc, vox = SyntheticDataset(16, seed=1).batch(range(2))
    n = vox.x.shape[0]
    ones = [None] * (2 * cfg.DISCRIMINATOR_ENCODER_REPEAT)
    chain = C.d_units(len(ones), 4, vox.edge_index, n, ones)
    x = x0s["real"]
    for u in chain:
        x = u.fwd(x, P)
    mvx, lab = x0s["real"][:, :29], x0s["real"][:, 29:]
    y = torch.nn.Sequential(D.mlp_encoder)(torch.cat([mvx, lab], 1))
    y = D.encoder(y, vox.edge_index)
    y = D.decoder(y)
    assert torch.allclose(x, y, rtol=1e-12, atol=1e-12)
