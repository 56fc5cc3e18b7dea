"""Where the bf16 generator gradient departs from the f32 reference at batch 32.

One generator iteration (trainer.py:484-495) from the batch-32 fixture's
initial parameters and replayed CPU draws, five ways:

  ref      the CPU oracle in f32 (pinned to the reference, tests/test_oracle_golden.py)
  f32      the HIP path in f32
  bf16     the HIP path with bf16 operands (configs[2])
  f32_rp   the HIP path in f32 with every G and D parameter rounded to bf16
  ref_rp   the CPU oracle in f32 with the same rounded parameters

f32_rp / ref_rp measure the conditioning of the G gradient: how far a
relative perturbation of bf16's size (2^-9) in the parameters alone moves it.
Prints (relative L2, cosine) for each pair and the parameters that carry the
bf16 error.  GPU; not imported by the product or the tests.
"""
from __future__ import annotations

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from parity_util import _rel_cos, b32_inputs, load_fixture  # noqa: E402


def rounded(sd):
    return {k: (v.to(torch.bfloat16).float() if v.is_floating_point() else v) for k, v in sd.items()}


def main():
    from oracle import reference as R
    from vgan._lib import gemm_precision_scope
    from vgan.config import Configuration
    from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
    from vgan.trainer import Trainer

    cuda = torch.device("cuda")
    f = load_fixture("forward_b32.pt")
    inp = b32_inputs(f, device="cuda")
    cfg = Configuration()
    torch.manual_seed(int(f["init_seed"]))
    G0, D0 = R.Generator(cfg), R.Discriminator(cfg)
    sd_g = {k: v.clone() for k, v in G0.state_dict().items()}
    sd_d = {k: v.clone() for k, v in D0.state_dict().items()}
    loc, vox = inp["vgan"]
    ol, ov = inp["oracle"]
    torch.manual_seed(4242)
    state = torch.get_rng_state()

    def oracle(g, d):
        Go, Do = R.Generator(cfg), R.Discriminator(cfg)
        Go.load_state_dict(g)
        Do.load_state_dict(d)
        torch.set_rng_state(state)
        Go.zero_grad()
        lo, ho, _ = Go(ol, ov, torch.randn(1, ov.num_nodes, cfg.Z_DIM))
        loss = R.generator_loss(Do, cfg, ol, ov, lo, ho.unsqueeze(0))
        loss.backward()
        return float(loss), {k: p.grad.clone() for k, p in Go.named_parameters()}, ho.argmax(1)

    def ours(prec, g, d):
        cfg.runtime["rng"] = "host"
        cfg.runtime["precision"] = prec
        G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
        G.load_state_dict(g)
        D.load_state_dict(d)
        tr = Trainer(G, D, None, torch.optim.Adam(G.parameters(), lr=2e-4, betas=cfg.BETAS),
                     torch.optim.Adam(D.parameters(), lr=2e-4, betas=cfg.BETAS), None, cfg)
        with gemm_precision_scope(prec):
            torch.set_rng_state(state)
            tr.adam_g.zero_grad()
            loss, hard = tr._gen_iteration(loc, vox)
            torch.cuda.synchronize()
        return float(loss), {k: p.grad.detach().cpu().clone() for k, p in G.named_parameters()}, \
            hard.squeeze(0).cpu().argmax(1)

    runs = {
        "ref": oracle(sd_g, sd_d),
        "ref_rp": oracle(rounded(sd_g), rounded(sd_d)),
        "f32": ours("f32", sd_g, sd_d),
        "bf16": ours("bf16", sd_g, sd_d),
        "f32_rp": ours("f32", rounded(sd_g), rounded(sd_d)),
    }
    out = {"loss": {k: v[0] for k, v in runs.items()}, "pairs": {}, "label_mismatch_vs_ref": {}}
    for k in runs:
        out["label_mismatch_vs_ref"][k] = float((runs[k][2] != runs["ref"][2]).float().mean())
    for a, b in (("f32", "ref"), ("bf16", "ref"), ("bf16", "f32"), ("f32_rp", "ref"), ("ref_rp", "ref"),
                 ("f32_rp", "f32"), ("bf16", "f32_rp")):
        rel, cos = _rel_cos(runs[a][1], runs[b][1])
        out["pairs"][f"{a}~{b}"] = {"rel": rel, "cos": cos}
    ref = runs["ref"][1]
    tot = torch.cat([v.reshape(-1).double() for v in ref.values()]).norm().item()
    rows = []
    for k, r in ref.items():
        r = r.double()
        e16 = (runs["bf16"][1][k].double() - r).norm().item()
        erp = (runs["ref_rp"][1][k].double() - r).norm().item()
        rows.append((e16 / tot, k, r.norm().item() / tot, e16 / max(r.norm().item(), 1e-30),
                     erp / max(r.norm().item(), 1e-30)))
    rows.sort(reverse=True)
    out["worst_params"] = [{"param": k, "share_of_total_err": round(s, 4), "grad_share": round(g, 4),
                            "bf16_rel": round(e, 4), "ref_rp_rel": round(p, 4)} for s, k, g, e, p in rows[:15]]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
