import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import torch
from parity_util import load_fixture, vgan_batches, oracle_batches, _FixedUniform, rel_err
from vgan.config import Configuration
from vgan.models import VoxelGNNGenerator, VoxelGNNDiscriminator
from vgan.trainer import Trainer
from oracle import reference as R
f = load_fixture("forward_eval.pt")
cfg = Configuration()
G = VoxelGNNGenerator(cfg, 17, 12); D = VoxelGNNDiscriminator(cfg, 17, 12)
G.load_state_dict(f["G"]); D.load_state_dict(f["D"]); G.eval(); D.eval()
loc, vox = vgan_batches(f["batch"])
with torch.no_grad():
    _, hard, soft = G(loc, vox, f["z"].cuda(), noise=f["gumbel_noise"].cuda())
tr = Trainer(G, D, None, None, None, None, cfg)
tr.rng = _FixedUniform(f["gp_eps"].cuda())
gp = tr._compute_gradient_penalty(loc, vox, soft.unsqueeze(0))
print("gp mine", gp.item(), "ref", float(f["gp"]))
# oracle gradient wrt mix
ol, ov = oracle_batches(f["batch"])
Do = R.Discriminator(cfg); Do.load_state_dict(f["D"]); Do.eval()
eps = f["gp_eps"]
mix_o = (eps * ov.types_onehot + (1 - eps) * f["label_soft"]).requires_grad_(True)
so = Do(ol, ov, mix_o.unsqueeze(0))
go, = torch.autograd.grad(so, mix_o, torch.ones_like(so))
mix_g = (eps.cuda() * vox.types_onehot.float() + (1 - eps.cuda()) * soft).detach().requires_grad_(True)
sg = D(loc, vox, mix_g.unsqueeze(0))
print("score rel", rel_err(sg, so))
gg1, = torch.autograd.grad(sg, mix_g, torch.ones_like(sg))
print("first-order grad (fused) rel", rel_err(gg1, go))
sg = D(loc, vox, mix_g.unsqueeze(0))
gg2, = torch.autograd.grad(sg, mix_g, torch.ones_like(sg), create_graph=True)
print("create_graph grad rel", rel_err(gg2, go))
