"""Locate the GPU-vs-oracle D-gradient gap at a critic iteration (GPU box).
Runs the per-iteration parity loop; at iteration IT splits the D loss into its
three terms and compares each term's parameter gradient and the per-node GP
gradient norms against the oracle in float64."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import torch
from parity_util import load_fixture, oracle_batches, vgan_batches, tiny_config, grads_close
from oracle import reference as R
from vgan.config import Configuration
from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
from vgan.trainer import Trainer
from vgan import data as vdata

name, IT = "step_tiny.pt", int(sys.argv[1]) if len(sys.argv) > 1 else 2
f = load_fixture(name)
cfg = tiny_config(Configuration())
cfg.runtime["rng"] = "host"
torch.manual_seed(0)
G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
G.load_state_dict(f["G0"]); D.load_state_dict(f["D0"])
tr = Trainer(G, D, None, torch.optim.Adam(G.parameters(), lr=2e-4, betas=cfg.BETAS),
             torch.optim.Adam(D.parameters(), lr=2e-4, betas=cfg.BETAS), None, cfg)
Go, Do = R.Generator(cfg), R.Discriminator(cfg)
Go.load_state_dict(f["G0"]); Do.load_state_dict(f["D0"])
od = torch.optim.Adam(Do.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
loc, vox = vgan_batches(f["batch"])
ol, ov = oracle_batches(f["batch"])
cuda = torch.device("cuda")
torch.manual_seed(int(f["step_seed"]))


def terms_gpu(hard, soft):
    prep = vdata.prepared(loc, vox, cfg.NUM_CLASSES)
    d_real = D(loc, vox, prep.onehot_f.unsqueeze(0))
    d_fake = D(loc, vox, hard)
    eps = tr.rng.uniform((prep.onehot_f.shape[0], 1), cuda)
    mix = (eps * prep.onehot_f + (1 - eps) * soft.squeeze(0)).requires_grad_(True)
    score = D(loc, vox, mix.unsqueeze(0))
    (g,) = torch.autograd.grad(score, mix, torch.ones_like(score), create_graph=True)
    gp = ((g.norm(dim=1) - 1) ** 2).mean() * cfg.LAMBDA_GP
    return d_real, d_fake, g, gp, list(D.named_parameters())


def terms_ref(Dm, hard, soft, dt):
    oh = ov.types_onehot.to(dt)
    d_real = Dm(ol, ov, oh.unsqueeze(0))
    d_fake = Dm(ol, ov, hard.to(dt))
    eps = torch.rand(oh.shape[0], 1).to(dt)
    mix = (eps * oh + (1 - eps) * soft.squeeze(0).to(dt)).requires_grad_(True)
    score = Dm(ol, ov, mix.unsqueeze(0))
    (g,) = torch.autograd.grad(score, mix, torch.ones_like(score), create_graph=True)
    gp = ((g.norm(dim=1) - 1) ** 2).mean() * cfg.LAMBDA_GP
    return d_real, d_fake, g, gp, list(Dm.named_parameters())


def pgrads(loss, named):
    gs = torch.autograd.grad(loss, [p for _, p in named], retain_graph=True, allow_unused=True)
    return {k: (g if g is not None else torch.zeros_like(p)) for (k, p), g in zip(named, gs)}


for it in range(cfg.N_CRITIC):
    with torch.no_grad():
        _, ho, so = Go(ol, ov, torch.randn(1, ov.num_nodes, cfg.Z_DIM))
    mid = torch.get_rng_state()
    if it == IT:
        import copy
        outs = {}
        for tag, fn in (("gpu", lambda: terms_gpu(ho.unsqueeze(0).to(cuda), so.unsqueeze(0).to(cuda))),
                        ("f32", lambda: terms_ref(Do, ho.unsqueeze(0), so.unsqueeze(0), torch.float32)),
                        ("f64", lambda: terms_ref(copy.deepcopy(Do).double(), ho.unsqueeze(0), so.unsqueeze(0),
                                                  torch.float64))):
            torch.set_rng_state(mid)
            dr, df, g, gp, named = fn()
            outs[tag] = dict(dr=dr.detach().cpu().double(), df=df.detach().cpu().double(),
                             gn=g.norm(dim=1).detach().cpu().double(), gp=gp.item(),
                             G_real=pgrads(-dr.mean(), named), G_fake=pgrads(df.mean(), named), G_gp=pgrads(gp, named))
        for tag in ("gpu", "f32"):
            a, b = outs[tag], outs["f64"]
            print(f"[{tag} vs f64] d_real max|d| {(a['dr'] - b['dr']).abs().max():.3e}  d_fake {(a['df'] - b['df']).abs().max():.3e}"
                  f"  gp {a['gp']:.8f} vs {b['gp']:.8f}  gradnorm max|d| {(a['gn'] - b['gn']).abs().max():.3e}")
            dn = (a['gn'] - b['gn']).abs()
            top = torch.topk(dn, 5)
            print("   worst nodes", top.indices.tolist(), [f"{v:.2e}" for v in top.values.tolist()],
                  "norms", [f"{v:.4f}" for v in b['gn'][top.indices].tolist()])
            for term in ("G_real", "G_fake", "G_gp"):
                print("  ", term, grads_close(a[term], b[term], rtol=1e-3)[1:])
        break
    tr.adam_d.zero_grad()
    d_loss = tr._compute_discriminator_loss(loc, vox, ho.unsqueeze(0).to(cuda), so.unsqueeze(0).to(cuda))
    d_loss.backward()
    torch.set_rng_state(mid)
    od.zero_grad()
    R.discriminator_loss(Do, cfg, ol, ov, ho.unsqueeze(0), so.unsqueeze(0)).backward()
    od.step()
    with torch.no_grad():
        for p, q in zip(D.parameters(), Do.parameters()):
            p.copy_(q.to(p.device))
