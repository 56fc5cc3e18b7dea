"""Stage-by-stage error of the f16 generator forward (vgan.half) against the
f32 forward on the same batch: prints the relative RMS error after every stage."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))
import torch  # noqa: E402

from vgan import data as vdata  # noqa: E402
from vgan.config import Configuration  # noqa: E402
from vgan.half import HalfGenerator  # noqa: E402
from vgan.models import VoxelGNNGenerator  # noqa: E402
from vgan.synth import SyntheticDataset  # noqa: E402

dev = torch.device("cuda:0")
cfg = Configuration()
torch.manual_seed(11)
G = VoxelGNNGenerator(cfg, 17, 12).to(dev).eval()
loc, vox = (g.to(dev) for g in SyntheticDataset(16, seed=9).batch(range(4)))
n = vox.num_nodes
z = torch.randn(1, n, cfg.Z_DIM, device=dev)
hg = HalfGenerator(G)
hg.trace = []
l16 = hg.logits(loc, vox, z)
with torch.no_grad():
    prep = vdata.prepared(loc, vox, 7)
    ref = {}
    em = G.matched_features_encoder(prep.matched_x)
    ref["em"] = em
    x = G.mlp_encoder(torch.cat([em, prep.voxel_x, z.reshape(n, -1)], -1))
    ref["x"] = x
    from vgan import ops
    h = x
    enc = G.encoder
    for b in range(enc.num_blocks):
        conv, norm = getattr(enc, f"module_{4 * b}"), getattr(enc, f"module_{4 * b + 1}")
        h = ops.graphnorm_relu_dropout(conv(h, prep.csr), norm.weight, norm.bias, norm.mean_scale, None, norm.eps, 1)
        ref[f"gat{b}"] = h
        # same stage fed with the f16 path's input (isolates the stage's own error)
    l32 = G.decoder(torch.cat([h, x, em, prep.voxel_x, z.reshape(n, -1)], -1))
for name, t in hg.trace:
    r = ref[name]
    e = float((t - r).pow(2).mean().sqrt() / r.pow(2).mean().sqrt().clamp_min(1e-12))
    print(f"{name:6s} C={r.shape[1]:4d} rms rel err {e:.3e}  |ref| rms {float(r.pow(2).mean().sqrt()):.3e}")
e = float((l16 - l32).pow(2).mean().sqrt() / l32.pow(2).mean().sqrt())
print(f"logits rms rel err {e:.3e}")
