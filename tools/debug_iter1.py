import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import torch
from parity_util import load_fixture, vgan_batches, oracle_batches
from vgan.config import Configuration
from vgan.models import VoxelGNNGenerator, VoxelGNNDiscriminator
from vgan.trainer import Trainer
from oracle import reference as R
f = load_fixture("step_sanity.pt")
cfg = Configuration(sanity_checking=True); cfg.runtime["rng"] = "host"
G = VoxelGNNGenerator(cfg, 17, 12); D = VoxelGNNDiscriminator(cfg, 17, 12)
G.load_state_dict(f["G0"]); D.load_state_dict(f["D0"])
tr = Trainer(G, D, None, None, None, None, cfg)
Go, Do = R.Generator(cfg), R.Discriminator(cfg)
Go.load_state_dict(f["G0"]); Do.load_state_dict(f["D0"])
od = torch.optim.Adam(Do.parameters(), lr=2e-4, betas=(0.5, 0.999))
loc, vox = vgan_batches(f["batch"]); ol, ov = oracle_batches(f["batch"])
torch.manual_seed(int(f["step_seed"]))
for it in range(3):
    st = torch.get_rng_state()
    with torch.no_grad():
        z = torch.randn(1, ov.num_nodes, cfg.Z_DIM)
        _, ho, so = Go(ol, ov, z)
    mid = torch.get_rng_state()
    od.zero_grad()
    # oracle pieces
    d_real = Do(ol, ov, ov.types_onehot.unsqueeze(0))
    d_fake = Do(ol, ov, ho.unsqueeze(0))
    st_gp = torch.get_rng_state()
    gp = R.gradient_penalty(Do, cfg, ol, ov, so.unsqueeze(0))
    end = torch.get_rng_state()
    # GPU pieces with the same RNG states
    torch.set_rng_state(st)
    with torch.no_grad():
        _, h, s = tr._generate(loc, vox)
    assert torch.equal(torch.get_rng_state(), mid)
    dr = D(loc, vox, vox.types_onehot.unsqueeze(0)); df = D(loc, vox, h)
    assert torch.equal(torch.get_rng_state(), st_gp)
    gpg = tr._compute_gradient_penalty(loc, vox, s)
    assert torch.equal(torch.get_rng_state(), end)
    print(f"it {it}: real {dr.mean().item():.7f} vs {d_real.mean().item():.7f} | fake {df.mean().item():.7f} vs {d_fake.mean().item():.7f} | gp {gpg.item():.7f} vs {gp.item():.7f}")
    print("    per-node d_real maxdiff", (dr.detach().cpu() - d_real.detach()).abs().max().item(), " d_fake", (df.detach().cpu()-d_fake.detach()).abs().max().item())
    # repeatability of the GPU GP
    torch.set_rng_state(st_gp)
    gpg2 = tr._compute_gradient_penalty(loc, vox, s)
    print("    gp repeat", gpg2.item())
    torch.set_rng_state(end)
    (d_fake.mean() - d_real.mean() + gp).backward()
    od.step()
    with torch.no_grad():
        for p, q in zip(D.parameters(), Do.parameters()):
            p.copy_(q.to(p.device))

# ---- instrument GN inputs at iteration 1 (re-run from scratch)
import vgan.ops as vops
orig = vops.graphnorm_relu_dropout
log = []
def wrapped(x, w, b, ms, keep, eps=1e-5):
    sd = x.detach().std(0, unbiased=False)
    log.append((x.shape[1], sd.min().item(), (sd == 0).sum().item(), x.detach().abs().max().item()))
    return orig(x, w, b, ms, keep, eps)
vops.graphnorm_relu_dropout = wrapped
import vgan.models as vm
vm.ops.graphnorm_relu_dropout = wrapped
G.load_state_dict(f["G0"]); D.load_state_dict(f["D0"])
Do.load_state_dict(f["D0"]); od = torch.optim.Adam(Do.parameters(), lr=2e-4, betas=(0.5, 0.999))
torch.manual_seed(int(f["step_seed"]))
for it in range(2):
    st = torch.get_rng_state()
    with torch.no_grad():
        _, ho, so = Go(ol, ov, torch.randn(1, ov.num_nodes, cfg.Z_DIM))
    od.zero_grad()
    d_real = Do(ol, ov, ov.types_onehot.unsqueeze(0)); d_fake = Do(ol, ov, ho.unsqueeze(0))
    st_gp = torch.get_rng_state()
    gp = R.gradient_penalty(Do, cfg, ol, ov, so.unsqueeze(0))
    end = torch.get_rng_state()
    torch.set_rng_state(st_gp)
    log.clear()
    with torch.no_grad():
        s = so.cuda().unsqueeze(0)
    gpg = tr._compute_gradient_penalty(loc, vox, s)
    print("iter", it, "gp", gpg.item(), gp.item())
    for rec in log: print("    GN C=%d min std %.3e zeros %d max|x| %.3e" % rec)
    torch.set_rng_state(end)
    (d_fake.mean() - d_real.mean() + gp).backward(); od.step()
    with torch.no_grad():
        for p, q in zip(D.parameters(), Do.parameters()):
            p.copy_(q.to(p.device))
# compare the GP gradient rows directly at iteration 1
eps = torch.rand(ov.num_nodes, 1)
mix_o = (eps * ov.types_onehot + (1 - eps) * so).requires_grad_(True)
sc_o = Do(ol, ov, mix_o.unsqueeze(0))
go, = torch.autograd.grad(sc_o, mix_o, torch.ones_like(sc_o))
mix_g = mix_o.detach().cuda().requires_grad_(True)
D.rng.mode = "host"
