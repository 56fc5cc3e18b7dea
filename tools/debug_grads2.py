import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import torch
from parity_util import load_fixture, vgan_batches, oracle_batches, rel_err
from vgan.config import Configuration
from vgan.models import VoxelGNNDiscriminator
from oracle import reference as R
f = load_fixture("forward_eval.pt")
cfg = Configuration()
D = VoxelGNNDiscriminator(cfg, 17, 12); D.load_state_dict(f["D"]); D.eval()
Do = R.Discriminator(cfg).double(); Do.load_state_dict({k: v.double() for k, v in f["D"].items()}); Do.eval()
loc, vox = vgan_batches(f["batch"]); ol, ov = oracle_batches(f["batch"])
ov.x = ov.x.double(); ol.x = ol.x.double()
lab = f["label_soft"]
def grads(mod, l, v, label, second):
    mod.zero_grad()
    mix = label.clone().requires_grad_(True)
    s = mod(l, v, mix.unsqueeze(0))
    if second:
        g, = torch.autograd.grad(s, mix, torch.ones_like(s), create_graph=True)
        loss = ((g.norm(dim=1) - 1) ** 2).mean()
    else:
        loss = s.mean()
    loss.backward()
    return loss.item(), {k: (p.grad.detach().cpu().double().clone() if p.grad is not None else None) for k, p in mod.named_parameters()}
for second in (False, True):
    lo, go = grads(Do, ol, ov, lab.double(), second)
    lg, gg = grads(D, loc, vox, lab.cuda(), second)
    print("second" if second else "first", lo, lg)
    for k in go:
        if go[k] is None: continue
        e = rel_err(gg[k], go[k])
        print(f"   {k:40s} rel {e:.2e}  |g| {go[k].norm().item():.3e}")
