"""Kernel launches per phase of one eager critic + generator iteration
(torch.profiler runtime events attributed to record_function ranges)."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from collections import Counter
import torch
from torch.profiler import profile, record_function, ProfilerActivity
from bench import build_trainer, make_pool  # noqa: E402  (sets sys.path for vgan)
from vgan.config import Configuration
from vgan import data as vdata

cuda = torch.device("cuda:0")
cfg = Configuration()
cfg.DEVICE = cuda
pool = make_pool(cfg, 0, 1, 1, 32, cuda)
tr = build_trainer(cfg)
loc, vox = pool[0]
tr.step(loc, vox)
torch.cuda.synchronize()
D = tr.discriminator


def critic():
    with record_function("phase:G_nograd"):
        with torch.no_grad():
            _, hard, soft = tr._generate(loc, vox)
    tr.adam_d.zero_grad()
    prep = vdata.prepared(loc, vox, cfg.NUM_CLASSES)
    with record_function("phase:D_real"):
        d_real = D(loc, vox, prep.onehot_f.unsqueeze(0))
    with record_function("phase:D_fake"):
        d_fake = D(loc, vox, hard)
    with record_function("phase:D_mix"):
        eps = tr.rng.uniform((prep.onehot_f.shape[0], 1), cuda)
        mix = (eps * prep.onehot_f + (1 - eps) * soft.squeeze(0)).requires_grad_(True)
        score = D(loc, vox, mix.unsqueeze(0))
    with record_function("phase:GP_grad"):
        (g,) = torch.autograd.grad(score, mix, torch.ones_like(score), create_graph=True)
        gp = ((g.norm(dim=1) - 1) ** 2).mean() * cfg.LAMBDA_GP
        loss = d_fake.mean() - d_real.mean() + gp
    with record_function("phase:backward"):
        loss.backward()
    with record_function("phase:adam"):
        tr.adam_d.step()
    with record_function("phase:G_iter"):
        logits, hard, _ = tr._generate(loc, vox)
        tr.adam_g.zero_grad()
        g_loss = tr._compute_generator_loss(loc, vox, logits, hard)
    with record_function("phase:G_backward"):
        g_loss.backward()


with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    critic()
    torch.cuda.synchronize()
evs = prof.events()
phases = [e for e in evs if e.name.startswith("phase:")]
names = Counter(e.name for e in evs if e.device_type == torch.autograd.DeviceType.CPU and
                (e.name.startswith("hip") or e.name.startswith("cuda")))
print("runtime api events:", names.most_common(12))
LAUNCH = {n for n in names if "Launch" in n or "Memset" in n or "Memcpy" in n}
launches = [e for e in evs if e.name in LAUNCH]
for ph in phases:
    inside = [e for e in launches if ph.time_range.start <= e.time_range.start <= ph.time_range.end]
    # attribute to the innermost torch op that launched it
    print(f"{ph.name:18s} launches {len(inside):6d}")
ops = Counter()
for e in evs:
    if e.device_type == torch.autograd.DeviceType.CPU and not e.name.startswith(("hip", "cuda", "phase")):
        k = sum(1 for c in e.cpu_children if c.name in LAUNCH)
        if k:
            ops[e.name] += k
print("direct launchers:", ops.most_common(40))
