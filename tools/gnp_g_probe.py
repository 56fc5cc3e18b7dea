"""The generator gradient with GraphNorm statistics from the aggregation's
partials (vgan.ops._GN_FWD_FUSE) and from the separate statistics pass,
each against the CPU oracle in f32 and f64 (tests/test_gnp_gpu.py's
test_critic_engine_and_generator_with_gnp setting: buildings 5-7, G from
seed 19, loss (logits . w) + (soft . w)).  GPU; not imported by the product or
the tests."""
from __future__ import annotations

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from parity_util import rel_err  # noqa: E402
from test_ops_gpu import _graph  # noqa: E402


def main():
    from oracle import reference as R
    from vgan import ops
    from vgan.config import Configuration
    from vgan.flat import FlatParams
    from vgan.models import VoxelGNNGenerator
    from vgan.rng import RNG

    cuda = torch.device("cuda")
    mode = sys.argv[1] if len(sys.argv) > 1 else "eval"
    loc, vox = _graph((5, 6, 7))
    cfg = Configuration()
    cfg.DEVICE = cuda
    n = vox.num_nodes
    torch.manual_seed(19)
    G = VoxelGNNGenerator(cfg, 17, 12).to(cuda)
    getattr(G, mode)()
    sd = {k: v.detach().cpu().clone() for k, v in G.state_dict().items()}
    flat_g = FlatParams(G)
    z = torch.randn(1, n, cfg.Z_DIM)
    noise = torch.empty(n, 7).exponential_()
    wgt = torch.randn(n, 7)
    lc, vc = loc.to(cuda), vox.to(cuda)
    out = {"mode": mode}
    grads = {}
    for fuse in (True, False):
        ops._GN_FWD_FUSE = fuse
        G.rng = RNG("fixed", seed=3)
        flat_g.zero_grad()
        logits, _, soft = G(lc, vc, z.to(cuda), noise=noise.to(cuda))
        with ops.direct_param_grads(), ops.deferred_param_folds(cuda):
            ((logits * wgt.to(cuda)).sum() + (soft * wgt.to(cuda)).sum()).backward()
        torch.cuda.synchronize()
        grads[f"gpu_fuse{int(fuse)}"] = {k: p.grad.detach().cpu().double().clone() for k, p in G.named_parameters()}
    if mode == "eval":  # no dropout: the oracle runs the same function
        from parity_util import oracle_batches  # noqa: F401
        from vgan.graph import GraphBatch  # noqa: F401

        cfg_cpu = Configuration()
        cfg_cpu.DEVICE = "cpu"
        for dt in (torch.float32, torch.float64):
            Go = R.Generator(cfg_cpu)
            Go.load_state_dict(sd)
            Go = Go.to(dt).eval()
            prev = torch.get_default_dtype()
            torch.set_default_dtype(dt)
            try:
                ol = type(loc)(**{k: (getattr(loc, k).to(dt) if k == "x" else getattr(loc, k)) for k in loc.keys()})
                ov = type(vox)(**{k: (getattr(vox, k).to(dt) if k == "x" else getattr(vox, k)) for k in vox.keys()})
                lg, _, sf = Go(ol, ov, z.to(dt), noise=noise.to(dt))
                ((lg * wgt.to(dt)).sum() + (sf * wgt.to(dt)).sum()).backward()
            finally:
                torch.set_default_dtype(prev)
            grads[f"oracle_{str(dt)[6:]}"] = {k: p.grad.detach().double().clone() for k, p in Go.named_parameters()}
    keys = list(grads)
    flat = {k: torch.cat([v.reshape(-1) for v in grads[k].values()]) for k in keys}
    for i, a in enumerate(keys):
        for b in keys[i + 1:]:
            out[f"{a}_vs_{b}"] = rel_err(flat[a], flat[b])
    ref = "oracle_float64" if "oracle_float64" in grads else "gpu_fuse0"
    for k in keys:
        if k == ref:
            continue
        per = sorted(((rel_err(grads[k][p], grads[ref][p]), p) for p in grads[ref]), reverse=True)[:5]
        out[f"worst_{k}_vs_{ref}"] = [(p, round(e, 5)) for e, p in per]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
