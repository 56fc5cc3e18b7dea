"""Model construction parity (no GPU): same seed -> same initial weights and
the same state_dict keys as the reference (via the oracle restatement, which the
golden fixtures pin to the reference bit-for-bit)."""
import pytest
import torch

from oracle import reference as R
from parity_util import tiny_config
from vgan.config import Configuration
from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator


@pytest.mark.parametrize("tiny", [False, True])
def test_init_matches_reference_bitwise(tiny):
    cfg = Configuration()
    cfg.DEVICE = "cpu"
    if tiny:
        tiny_config(cfg)
    torch.manual_seed(777)
    g_ref, d_ref = R.Generator(cfg), R.Discriminator(cfg)
    torch.manual_seed(777)
    g, d = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    for mine, ref in ((g, g_ref), (d, d_ref)):
        a, b = mine.state_dict(), ref.state_dict()
        assert list(a.keys()) == list(b.keys())
        for k in a:
            assert torch.equal(a[k], b[k]), k


def test_param_counts_match_survey():
    cfg = Configuration()
    cfg.DEVICE = "cpu"
    g, d = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    assert sum(p.numel() for p in g.parameters()) == 274185
    assert sum(p.numel() for p in d.parameters()) == 15665


def test_forward_refuses_cpu():
    from vgan.graph import GraphBatch
    from vgan.synth import make_building

    cfg = Configuration()
    cfg.DEVICE = "cpu"
    g = VoxelGNNGenerator(cfg, 17, 12)
    loc, vox = make_building(1, 1)
    lb, vb = GraphBatch.from_data_list([loc]), GraphBatch.from_data_list([vox])
    with pytest.raises(RuntimeError, match="ROCm device"):
        g(lb, vb, torch.zeros(1, vox.num_nodes, cfg.Z_DIM))
