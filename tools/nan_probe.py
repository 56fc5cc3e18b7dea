"""Where a long training stream first goes non-finite.

The stream of tests/test_bf16_gpu.py::test_bf16_training_tracks_f32_over_200_steps
(10 batches of 16 synthetic buildings, cycled; graphed steps from
torch.manual_seed(SEED), device RNG), per precision and step mode: per step
d_loss, g_loss, the largest |parameter| and |gradient| of G and D; at the
first non-finite loss or parameter, which parameters / gradients are
non-finite.  GPU; not imported by the product or the tests.

usage: python tools/nan_probe.py [steps] [precisions] [modes]
       e.g. python tools/nan_probe.py 200 bf16,f32 graphed,eager
"""
from __future__ import annotations

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import parity_util  # noqa: E402,F401  (sys.path for the package)


def run(precision: str, mode: str, steps: int, batches):
    from vgan.config import Configuration
    from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
    from vgan.trainer import Trainer

    cuda = torch.device("cuda")
    cfg = Configuration()
    cfg.DEVICE = cuda
    cfg.runtime["precision"] = precision
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    tr = Trainer(G, D, None, og, od, None, cfg)
    hist = []
    first_bad = None
    for s in range(steps):
        loc, vox = batches[s % len(batches)]
        r = tr.step_graphed(loc, vox) if mode == "graphed" else tr.step(loc, vox)
        dl = float(r["d_loss_mean"]) if "d_loss_mean" in r else float(torch.stack(list(r["d_losses"])).mean())
        gl = float(r["g_loss"])

        def mx(ps, grad=False):
            v = [(p.grad if grad else p).detach().abs().max() for p in ps if (p.grad is not None or not grad)]
            return float(torch.stack(v).max()) if v else 0.0

        row = {"step": s, "d_loss": dl, "g_loss": gl, "G_max": mx(G.parameters()), "D_max": mx(D.parameters()),
               "G_grad_max": mx(G.parameters(), True), "D_grad_max": mx(D.parameters(), True)}
        hist.append(row)
        bad = not all(map(lambda v: v == v and abs(v) != float("inf"), row.values()))
        if bad:
            first_bad = {
                "step": s,
                "nonfinite_params": [k for k, p in list(G.named_parameters(prefix="G")) +
                                     list(D.named_parameters(prefix="D")) if not torch.isfinite(p).all()],
                "nonfinite_grads": [k for k, p in list(G.named_parameters(prefix="G")) +
                                    list(D.named_parameters(prefix="D"))
                                    if p.grad is not None and not torch.isfinite(p.grad).all()],
                "before": hist[-3:],
            }
            break
    return {"precision": precision, "mode": mode, "steps_run": len(hist), "first_bad": first_bad,
            "every_10th": hist[::10]}


def main():
    from vgan.synth import SyntheticDataset

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    precs = (sys.argv[2] if len(sys.argv) > 2 else "bf16,f32").split(",")
    modes = (sys.argv[3] if len(sys.argv) > 3 else "graphed").split(",")
    cuda = torch.device("cuda")
    ds = SyntheticDataset(160, seed=777)
    batches = []
    for b in range(10):
        loc, vox = ds.batch(range(16 * b, 16 * b + 16))
        batches.append((loc.to(cuda), vox.to(cuda)))
    for p in precs:
        for m in modes:
            out = run(p, m, steps, batches)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
