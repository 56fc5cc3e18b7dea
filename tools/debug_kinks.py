"""Smallest |pre-activation| at every ReLU of the oracle D (f64) for the three D
forwards at critic iteration IT of the step_tiny golden step (CPU)."""
import copy
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import torch
import torch.nn as nn
from parity_util import load_fixture, oracle_batches, tiny_config
from oracle import reference as R
from vgan.config import Configuration

IT = int(sys.argv[1]) if len(sys.argv) > 1 else 2
f = load_fixture("step_tiny.pt")
cfg = tiny_config(Configuration())
Go, Do = R.Generator(cfg), R.Discriminator(cfg)
Go.load_state_dict(f["G0"]); Do.load_state_dict(f["D0"])
od = torch.optim.Adam(Do.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
ol, ov = oracle_batches(f["batch"])
torch.manual_seed(int(f["step_seed"]))
for it in range(cfg.N_CRITIC):
    with torch.no_grad():
        _, ho, so = Go(ol, ov, torch.randn(1, ov.num_nodes, cfg.Z_DIM))
    mid = torch.get_rng_state()
    if it == IT:
        D64 = copy.deepcopy(Do).double()
        rec = []
        for name, m in D64.named_modules():
            if isinstance(m, nn.ReLU):
                m.register_forward_pre_hook(lambda mod, inp, name=name: rec.append((name, inp[0].detach().clone())))
        dbl = lambda b: type(b)(**{k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else v)
                                   for k, v in b._d.items()})
        R.discriminator_loss(D64, cfg, dbl(ol), dbl(ov), ho.unsqueeze(0).double(), so.unsqueeze(0).double())
        for k, (name, x) in enumerate(rec):
            a = x.abs()
            scale = x.abs().mean().item()
            mn, idx = a.min().item(), int(a.argmin())
            print(f"{k:2d} {name:28s} min|x| {mn:.3e} (scale {scale:.3e}) at node {idx // x.shape[1]} ch {idx % x.shape[1]}")
        break
    od.zero_grad()
    R.discriminator_loss(Do, cfg, ol, ov, ho.unsqueeze(0), so.unsqueeze(0)).backward()
    od.step()
