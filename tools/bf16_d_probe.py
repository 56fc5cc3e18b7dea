"""Where the bf16 discriminator gradient departs from the f32 reference at batch 32.

One critic iteration (trainer.py:470-479) from the batch-32 fixture's initial
parameters, the oracle's labels and the same GP draws, four ways:

  ref       the CPU oracle in f32 (pinned to the reference, tests/test_oracle_golden.py)
  ref_bf    the CPU oracle with every nn.Linear / GATConv.lin forward operand rounded
            to bf16 (the conditioning of the D gradient under bf16 operands)
  f32       the HIP critic engine in f32
  bf16      the HIP critic engine with bf16 operands (configs[2])

Prints (relative L2, cosine) per pair and the parameters carrying the bf16
error.  GPU; not imported by the product or the tests.
"""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from parity_util import _FixedUniform, _rel_cos, b32_inputs, load_fixture  # noqa: E402


def main():
    from oracle import reference as R
    from vgan._lib import gemm_precision_scope
    from vgan.config import Configuration
    from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
    from vgan.trainer import Trainer

    cuda = torch.device("cuda")
    name = sys.argv[1] if len(sys.argv) > 1 else "forward_b32.pt"
    f = load_fixture(name)
    inp = b32_inputs(f, device="cuda")
    cfg = Configuration()
    torch.manual_seed(int(f["init_seed"]))
    G0, D0 = R.Generator(cfg), R.Discriminator(cfg)
    if "G" in f:
        G0.load_state_dict(f["G"])
        D0.load_state_dict(f["D"])
    loc, vox = inp["vgan"]
    ol, ov = inp["oracle"]
    torch.manual_seed(4242)
    with torch.no_grad():
        _, ho, so = G0(ol, ov, torch.randn(1, ov.num_nodes, cfg.Z_DIM))
    gp_state = torch.get_rng_state()
    eps = torch.rand(ov.num_nodes, 1)  # the GP's draw (trainer.py:298)

    lin = F.linear

    def lin_bf(x, w, b=None):
        return lin(x.to(torch.bfloat16).float(), w.to(torch.bfloat16).float(), b)

    def oracle(bf):
        D = R.Discriminator(cfg)
        D.load_state_dict(D0.state_dict())
        D.eval()  # no dropout: the same D on both sides
        torch.set_rng_state(gp_state)
        F.linear = lin_bf if bf else lin
        try:
            R.discriminator_loss(D, cfg, ol, ov, ho.unsqueeze(0), so.unsqueeze(0)).backward()
        finally:
            F.linear = lin
        return {k: p.grad.clone() for k, p in D.named_parameters()}

    def gpu(precision):
        cfg.runtime["precision"] = precision
        G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
        G.load_state_dict(G0.state_dict())
        D.load_state_dict(D0.state_dict())
        G.eval()
        D.eval()
        tr = Trainer(G, D, None, None, None, None, cfg)
        tr.rng = _FixedUniform(eps.to(cuda))
        tr.adam_d.zero_grad()
        with gemm_precision_scope(precision):
            tr._critic_loss_backward(loc, vox, ho.unsqueeze(0).to(cuda), so.unsqueeze(0).to(cuda))
        torch.cuda.synchronize()
        return {k: p.grad.detach().cpu().clone() for k, p in D.named_parameters()}

    res = {"ref": oracle(False), "ref_bf": oracle(True), "f32": gpu("f32"), "bf16": gpu("bf16")}
    out = {"fixture": name, "eval_iteration0": {}}
    for a, b in (("f32", "ref"), ("ref_bf", "ref"), ("bf16", "ref"), ("bf16", "f32")):
        out["eval_iteration0"][f"{a}_vs_{b}"] = _rel_cos(res[a], res[b])
    per = []
    for k in res["ref"]:
        r = res["ref"][k].double()
        per.append((float((res["bf16"][k].double() - r).norm() / r.norm().clamp_min(1e-30)),
                    float((res["ref_bf"][k].double() - r).norm() / r.norm().clamp_min(1e-30)),
                    float(r.norm()), k))
    per.sort(reverse=True)
    out["eval_iteration0"]["worst_bf16_params"] = [
        {"param": k, "bf16_rel": round(a, 4), "ref_bf_rel": round(b, 4), "norm": n} for a, b, n, k in per[:6]]

    # the test's loop (tests/parity_util.step_iterations_bf16_vs_oracle): train
    # mode, replayed CPU draws, D continued from the oracle's Adam step
    cfg.runtime["rng"] = "host"
    cfg.runtime["precision"] = "bf16"
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    G.load_state_dict(G0.state_dict())
    D.load_state_dict(D0.state_dict())
    tr = Trainer(G, D, None, torch.optim.Adam(G.parameters(), lr=2e-4, betas=cfg.BETAS),
                 torch.optim.Adam(D.parameters(), lr=2e-4, betas=cfg.BETAS), None, cfg)
    Go, Do = R.Generator(cfg), R.Discriminator(cfg)
    Go.load_state_dict(G0.state_dict())
    Do.load_state_dict(D0.state_dict())
    od = torch.optim.Adam(Do.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    torch.manual_seed(4242)
    its = []
    with gemm_precision_scope("bf16"):
        for it in range(cfg.N_CRITIC):
            state = torch.get_rng_state()
            with torch.no_grad():
                tr._generate(loc, vox)
            mid = torch.get_rng_state()
            torch.set_rng_state(state)
            with torch.no_grad():
                _, h_o, s_o = Go(ol, ov, torch.randn(1, ov.num_nodes, cfg.Z_DIM))
            tr.adam_d.zero_grad()
            tr._critic_loss_backward(loc, vox, h_o.unsqueeze(0).to(cuda), s_o.unsqueeze(0).to(cuda))
            got = {k: p.grad.detach().cpu().clone() for k, p in D.named_parameters()}
            refs = {}
            for bf in (True, False):
                Dx = R.Discriminator(cfg)
                Dx.load_state_dict(Do.state_dict())
                torch.set_rng_state(mid)
                F.linear = lin_bf if bf else lin
                try:
                    R.discriminator_loss(Dx, cfg, ol, ov, h_o.unsqueeze(0), s_o.unsqueeze(0)).backward()
                finally:
                    F.linear = lin
                refs[bf] = {k: p.grad.clone() for k, p in Dx.named_parameters()}
            torch.set_rng_state(mid)
            od.zero_grad()
            R.discriminator_loss(Do, cfg, ol, ov, h_o.unsqueeze(0), s_o.unsqueeze(0)).backward()
            worst = sorted(((float((got[k].double() - refs[False][k].double()).norm() /
                                   refs[False][k].double().norm().clamp_min(1e-30)), k) for k in got), reverse=True)
            its.append({"it": it, "bf16_vs_ref": _rel_cos(got, refs[False]),
                        "ref_bf_vs_ref": _rel_cos(refs[True], refs[False]),
                        "worst": [(k, round(v, 3)) for v, k in worst[:4]]})
            print(json.dumps(its[-1]), file=sys.stderr, flush=True)
            od.step()
            with torch.no_grad():
                for p, q in zip(D.parameters(), Do.parameters()):
                    p.copy_(q.to(p.device))
    out["train_iterations"] = its
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
