"""The no-grad generator encoder with every GraphNorm applied inside the next
block's projection GEMM (GATEncoder._forward_nograd_fused: critic labels,
validation, inference) against the module path (separate GraphNorm apply,
then the projection) on the same batch, weights and device-RNG state.  The
projection sees the apply kernel's values up to FMA contraction, so the
encoder outputs agree to float rounding; the Gumbel labels of the stacked
label forward (what the critic consumes) agree except at exact ties."""
import pytest
import torch

from parity_util import rel_err
from vgan import data as vdata
from vgan.config import Configuration
from vgan.models import GATEncoder, VoxelGNNGenerator
from vgan.rng import RNG
from vgan.synth import SyntheticDataset

pytestmark = pytest.mark.gpu


def _gen(cuda, seed=5):
    cfg = Configuration()
    cfg.DEVICE = str(cuda)
    torch.manual_seed(seed)
    return cfg, VoxelGNNGenerator(cfg, 17, 12).to(cuda)


@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("copies", [1, 5])
def test_fused_nograd_encoder_matches_module_path(cuda, training, copies):
    cfg, G = _gen(cuda)
    G.train(training)
    loc, vox = SyntheticDataset(8, seed=3).batch(range(8))
    loc, vox = loc.to(cuda), vox.to(cuda)
    prep = vdata.prepared(loc, vox, cfg.NUM_CLASSES)
    csr = prep.csr.stacked(copies)
    enc = G.encoder
    x = torch.randn(csr.num_nodes, enc.widths[0], device=cuda)
    outs = []
    for fused in (True, False):
        GATEncoder.fused_nograd = fused
        try:
            rng = RNG("device", seed=1234)
            rng.reset()
            with torch.no_grad():
                outs.append(enc(x, csr, rng, segments=copies))
        finally:
            GATEncoder.fused_nograd = True
    torch.cuda.synchronize()
    assert outs[0].shape == outs[1].shape
    assert rel_err(outs[0], outs[1]) < 1e-5, rel_err(outs[0], outs[1])


def test_fused_nograd_labels_match_module_path(cuda):
    """The stacked critic-label forward of the trainer (5 copies, dropout on):
    logits to float rounding, hard labels equal but for near-ties."""
    cfg, G = _gen(cuda)
    G.train(True)
    loc, vox = SyntheticDataset(32, seed=9).batch(range(32))
    loc, vox = loc.to(cuda), vox.to(cuda)
    res = []
    for fused in (True, False):
        GATEncoder.fused_nograd = fused
        try:
            rng = RNG("device", seed=77)
            G.rng = rng
            rng.reset()
            z = rng.normal((5, vox.num_nodes, cfg.Z_DIM), cuda)
            noise = rng.exponential((5 * vox.num_nodes, cfg.NUM_CLASSES), cuda)
            with torch.no_grad():
                res.append(G(loc, vox, z, noise=noise))
        finally:
            GATEncoder.fused_nograd = True
    torch.cuda.synchronize()
    (l1, h1, _), (l2, h2, _) = res
    assert rel_err(l1, l2) < 1e-4, rel_err(l1, l2)
    agree = (h1.argmax(-1) == h2.argmax(-1)).float().mean().item()
    assert agree > 0.999, agree
