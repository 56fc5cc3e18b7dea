"""Is the per-iteration gradient tolerance intrinsic?  Oracle f32 vs oracle f64
on the same inputs at each critic iteration of a golden step (CPU only)."""
import copy
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import torch
from parity_util import load_fixture, oracle_batches, tiny_config, grads_close
from oracle import reference as R
from vgan.config import Configuration

name = sys.argv[1] if len(sys.argv) > 1 else "step_tiny.pt"
f = load_fixture(name)
cfg = Configuration(sanity_checking=(name == "step_sanity.pt"))
if name == "step_tiny.pt":
    tiny_config(cfg)
Go, Do = R.Generator(cfg), R.Discriminator(cfg)
Go.load_state_dict(f["G0"]); Do.load_state_dict(f["D0"])
od = torch.optim.Adam(Do.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
ol, ov = oracle_batches(f["batch"])


def to64(b):
    return type(b)(**{k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else v)
                      for k, v in b._d.items()})


torch.manual_seed(int(f["step_seed"]))
for it in range(cfg.N_CRITIC):
    with torch.no_grad():
        _, ho, so = Go(ol, ov, torch.randn(1, ov.num_nodes, cfg.Z_DIM))
    mid = torch.get_rng_state()
    od.zero_grad()
    d = R.discriminator_loss(Do, cfg, ol, ov, ho.unsqueeze(0), so.unsqueeze(0))
    d.backward()
    g32 = {k: p.grad.clone() for k, p in Do.named_parameters()}
    after = torch.get_rng_state()
    torch.set_rng_state(mid)
    D64 = copy.deepcopy(Do).double()
    d64 = R.discriminator_loss(D64, cfg, to64(ol), to64(ov), ho.unsqueeze(0).double(), so.unsqueeze(0).double())
    d64.backward()
    g64 = {k: p.grad for k, p in D64.named_parameters()}
    assert torch.equal(torch.get_rng_state(), after)
    print(it, "loss rel", abs(d.item() - d64.item()) / abs(d64.item()),
          "grads 5e-3:", grads_close(g32, g64, rtol=5e-3), "1e-3:", grads_close(g32, g64)[1:])
    od.step()
