"""Trace GPU vs CPU-oracle divergence through the critic iterations of the
step_sanity fixture (host RNG replay on both sides)."""
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
tr = Trainer(G, D, None, torch.optim.Adam(G.parameters(), lr=2e-4, betas=(0.5, 0.999)),
             torch.optim.Adam(D.parameters(), lr=2e-4, betas=(0.5, 0.999)), None, cfg)
Go, Do = R.Generator(cfg), R.Discriminator(cfg)
Go.load_state_dict(f["G0"]); Do.load_state_dict(f["D0"])
od = torch.optim.Adam(Do.parameters(), lr=2e-4, betas=(0.5, 0.999))
loc, vox = vgan_batches(f["batch"]); ol, ov = oracle_batches(f["batch"])
gen_state = None
torch.manual_seed(int(f["step_seed"]))
for it in range(5):
    st = torch.get_rng_state()
    # GPU side
    with torch.no_grad():
        _, hard, soft = tr._generate(loc, vox)
    tr.adam_d.zero_grad()
    dl = tr._compute_discriminator_loss(loc, vox, hard, soft); dl.backward()
    gpu_grads = {k: p.grad.detach().cpu().clone() for k, p in D.named_parameters()}
    tr.adam_d.step()
    st_after = torch.get_rng_state()
    # oracle side, same RNG state
    torch.set_rng_state(st)
    with torch.no_grad():
        z = torch.randn(1, ov.num_nodes, cfg.Z_DIM)
        _, ho, so = Go(ol, ov, z)
    od.zero_grad()
    dlo = R.discriminator_loss(Do, cfg, ol, ov, ho.unsqueeze(0), so.unsqueeze(0)); dlo.backward()
    od.step()
    assert torch.equal(torch.get_rng_state(), st_after), "RNG consumption differs"
    flips = (hard.squeeze(0).argmax(1).cpu() != ho.argmax(1)).sum().item()
    sdiff = (soft.squeeze(0).cpu() - so).abs().max().item()
    gerr = max(((gpu_grads[k] - p.grad).norm() / p.grad.norm().clamp_min(1e-30)).item() for k, p in Do.named_parameters() if p.grad.norm() > 1e-6)
    pd = torch.cat([(p.detach().cpu() - q.detach()).abs().reshape(-1) for p, q in zip(D.parameters(), Do.parameters())])
    print(f"it {it}: d_loss gpu {dl.item():.6f} cpu {dlo.item():.6f}  argmax flips {flips}  soft maxdiff {sdiff:.2e}  "
          f"grad rel max {gerr:.2e}  param maxdiff {pd.max().item():.2e} frac>1e-5 {(pd > 1e-5).float().mean().item():.3f}")
    # resync parameters to isolate per-iteration error
    if len(sys.argv) > 1:
        with torch.no_grad():
            for p, q in zip(D.parameters(), Do.parameters()):
                p.copy_(q.to(p.device))
