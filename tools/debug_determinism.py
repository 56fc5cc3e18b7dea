"""Is the step bitwise reproducible? eager vs eager, graph vs graph, eager vs graph (fixed RNG)."""
import sys
sys.path.insert(0, "tests")
import torch
from test_graph_gpu import _trainer, _batch
from parity_util import tiny_config
from vgan.config import Configuration

cuda = torch.device("cuda:0")
cfg = tiny_config(Configuration())
cfg.runtime["rng"] = "fixed"


def run(graphed, det=False):
    torch.use_deterministic_algorithms(det, warn_only=True)
    tr = _trainer(cfg)
    loc, vox = _batch(cuda)
    outs = []
    for _ in range(3):
        o = tr.step_graphed(loc, vox) if graphed else tr.step(loc, vox)
        outs.append((o["d_losses"].mean() if not graphed else o["d_loss_mean"]).item())
    torch.cuda.synchronize()
    return outs, tr.flat_d.param.clone(), tr.flat_g.param.clone()


e1, e2 = run(False), run(False)
g1, g2 = run(True), run(True)
print("eager", e1[0], e2[0], (e1[1] - e2[1]).abs().max().item())
print("graph", g1[0], g2[0], (g1[1] - g2[1]).abs().max().item())
print("e-g", (e1[1] - g1[1]).abs().max().item())
d1 = run(False, det=True)
print("eager det", d1[0])
