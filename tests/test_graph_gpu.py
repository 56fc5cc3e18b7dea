"""The hipGraph-captured step reproduces the eager step.

The eager step is not bitwise reproducible run to run (torch's reduction
kernels vectorise by pointer alignment, and eager allocations move), and the
WGAN-GP loss is discontinuous at ReLU kinks, so multi-step trajectories are
compared per iteration from identical state: each captured iteration body
(critic, generator) must give the eager body's loss and gradients.  Randomness
comes from the test-only ``fixed`` RNG (the same seeded draws in every body).
Replays themselves must be bitwise deterministic, and with device RNG must
draw fresh noise every iteration.
"""
import pytest
import torch

from parity_util import grads_close, tiny_config
from vgan.config import Configuration
from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
from vgan.synth import SyntheticDataset
from vgan.trainer import Trainer

pytestmark = pytest.mark.gpu


def _trainer(cfg, seed=5):
    torch.manual_seed(seed)
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    return Trainer(G, D, None, og, od, None, cfg)


def _batch(cuda, n=4):
    loc, vox = SyntheticDataset(64, seed=3).batch(range(n))
    return loc.to(cuda), vox.to(cuda)


def _flat_grads(flat, module):
    return {k: flat.grad[flat._offset(p):flat._offset(p) + p.numel()].clone() for k, p in module.named_parameters()}


@pytest.mark.parametrize("tiny", [True, False])
def test_graph_iterations_match_eager_bodies(cuda, tiny):
    cfg = Configuration()
    if tiny:
        tiny_config(cfg)
    cfg.runtime["rng"] = "fixed"
    eager, graphed = _trainer(cfg), _trainer(cfg)
    loc, vox = _batch(cuda)
    graphs = graphed.capture(loc, vox, whole=False)  # the per-piece graphs, replayed one by one
    acc_e = torch.zeros(2, device=cuda)
    for it in range(cfg.N_CRITIC):
        graphed.flat_d.param.copy_(eager.flat_d.param)  # same state in, one iteration out
        graphed.adam_d.exp_avg.copy_(eager.adam_d.exp_avg)
        graphed.adam_d.exp_avg_sq.copy_(eager.adam_d.exp_avg_sq)
        graphed.adam_d.step_t.copy_(eager.adam_d.step_t)
        graphs["acc"].zero_()
        acc_e.zero_()
        graphs["critic"][0].replay()
        eager._critic_body(loc, vox, acc_e, True)
        torch.cuda.synchronize()
        assert abs(graphs["acc"][0].item() - acc_e[0].item()) <= 1e-4 * max(1.0, abs(acc_e[0].item())), it
        ok, worst, total = grads_close(_flat_grads(graphed.flat_d, graphed.discriminator),
                                       _flat_grads(eager.flat_d, eager.discriminator), rtol=5e-3)
        assert ok, (it, worst, total)
    assert int(graphed.adam_d.step_t.item()) == int(eager.adam_d.step_t.item()) == cfg.N_CRITIC
    graphed.flat_d.param.copy_(eager.flat_d.param)
    graphed.flat_g.param.copy_(eager.flat_g.param)
    graphs["gen"].replay()
    eager._gen_body(loc, vox, acc_e, True)
    torch.cuda.synchronize()
    assert abs(graphs["acc"][-1].item() - acc_e[-1].item()) <= 1e-4 * max(1.0, abs(acc_e[-1].item()))
    ok, worst, total = grads_close(_flat_grads(graphed.flat_g, graphed.generator),
                                   _flat_grads(eager.flat_g, eager.generator), rtol=5e-3)
    assert ok, (worst, total)
    assert int(graphed.adam_g.step_t.item()) == 1


def test_graph_replay_is_deterministic(cuda):
    cfg = tiny_config(Configuration())
    cfg.runtime["rng"] = "fixed"
    runs = []
    for _ in range(2):
        tr = _trainer(cfg)
        loc, vox = _batch(cuda)
        losses = [tr.step_graphed(loc, vox)["d_loss_mean"].item() for _ in range(3)]
        runs.append((losses, tr.flat_d.param.clone(), tr.flat_g.param.clone()))
    assert runs[0][0] == runs[1][0]
    assert torch.equal(runs[0][1], runs[1][1]) and torch.equal(runs[0][2], runs[1][2])


def test_graph_replays_draw_fresh_noise(cuda):
    cfg = tiny_config(Configuration())
    tr = _trainer(cfg)
    loc, vox = _batch(cuda)
    outs = [tr.step_graphed(loc, vox)["d_loss_mean"].item() for _ in range(3)]
    assert len(set(outs)) == 3  # different z / dropout / Gumbel / GP eps each replay
    assert all(abs(v) < 1e4 for v in outs)
    assert int(tr.adam_d.step_t.item()) == 3 * cfg.N_CRITIC and int(tr.adam_g.step_t.item()) == 3


def test_whole_step_graph_equals_piece_graphs(cuda):
    """step_graphed over ONE graph of the whole step (stacked labels, the
    critic iterations, the generator iteration) and over the per-piece graphs
    replayed back to back: the same launches in the same order, so losses,
    labels and every parameter and Adam moment bit for bit over three steps."""
    cfg = Configuration()
    cfg.runtime["rng"] = "device"
    a, b = _trainer(cfg), _trainer(cfg)
    assert a._stacked_labels() and b._stacked_labels()
    la, va = _batch(cuda)
    lb, vb = _batch(cuda)
    ga = a.capture(la, va, whole=True)
    gb = b.capture(lb, vb, whole=False)
    assert ga.get("whole") is not None and gb.get("whole") is None and len(gb["critic"]) == cfg.N_CRITIC
    for _ in range(3):
        oa, ob = a.step_graphed(la, va), b.step_graphed(lb, vb)
        torch.cuda.synchronize()
        assert torch.equal(oa["d_losses"], ob["d_losses"]) and torch.equal(oa["g_loss"], ob["g_loss"])
        assert torch.equal(oa["label_hard"], ob["label_hard"])
    for fa, fb in ((a.flat_g, b.flat_g), (a.flat_d, b.flat_d)):
        assert torch.equal(fa.param, fb.param)
    for ma, mb in ((a.adam_g, b.adam_g), (a.adam_d, b.adam_d)):
        assert torch.equal(ma.exp_avg, mb.exp_avg) and torch.equal(ma.exp_avg_sq, mb.exp_avg_sq)
