"""Kernel launches per phase of one eager step (torch.profiler runtime events
attributed to record_function ranges)."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from collections import Counter
import torch
from torch.profiler import profile, record_function, ProfilerActivity
from bench import build_trainer, make_pool  # noqa: E402  (sets sys.path for vgan)
from vgan.config import Configuration
from vgan import ops

cuda = torch.device("cuda:0")
cfg = Configuration()
cfg.DEVICE = cuda
pool = make_pool(cfg, 0, 1, 1, 32, cuda)
tr = build_trainer(cfg)
loc, vox = pool[0]
tr.step(loc, vox)
torch.cuda.synchronize()


def step():
    with record_function("phase:labels_G5"):
        labels = tr._critic_labels(loc, vox)
    with record_function("phase:critic_iter"):
        d = tr._critic_iteration(loc, vox, labels, 0)
        tr.adam_d.step(counted=True)
    with record_function("phase:gen_fwd"):
        tr.rng.reset()
        logits, hard, _ = tr._generate(loc, vox)
        tr.adam_g.zero_grad()
        for p in tr.discriminator.parameters():
            p.requires_grad_(False)
    with record_function("phase:gen_loss"):
        g_loss = tr._compute_generator_loss(loc, vox, logits, hard)
    with record_function("phase:gen_bwd"):
        with ops.direct_param_grads():
            g_loss.backward()
        for p in tr.discriminator.parameters():
            p.requires_grad_(True)
        tr.adam_g.step(counted=True)


with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    step()
    torch.cuda.synchronize()
evs = prof.events()
phases = [e for e in evs if e.name.startswith("phase:")]
names = Counter(e.name for e in evs if e.device_type == torch.autograd.DeviceType.CPU and
                (e.name.startswith("hip") or e.name.startswith("cuda")))
LAUNCH = {n for n in names if "Launch" in n or "Memset" in n or "Memcpy" in n}
launches = [e for e in evs if e.name in LAUNCH]
seen = set()
for ph in phases:
    if ph.name in seen:
        continue
    seen.add(ph.name)
    inside = [e for e in launches if ph.time_range.start <= e.time_range.start <= ph.time_range.end]
    print(f"{ph.name:18s} launches {len(inside):6d}")
ops_ = Counter()
for e in evs:
    if e.device_type == torch.autograd.DeviceType.CPU and not e.name.startswith(("hip", "cuda", "phase")):
        k = sum(1 for c in e.cpu_children if c.name in LAUNCH)
        if k:
            ops_[e.name] += k
print("torch-op launchers:", ops_.most_common(25))
