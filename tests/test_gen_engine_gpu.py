"""The generator iteration issued from C++ (vg_gen_loss_and_grad,
csrc/gen_engine.hip) against the Python schedule it restates
(vgan/genstep.py GeneratorEngine.loss_and_grad, VGAN_GEN_NATIVE=0 there),
which tests/test_genstep_gpu.py pins to the autograd path and
tests/test_b32_gpu.py to the reference (trainer.py:483-491, 334-385).

Same kernels, same order, same arguments, same device-RNG salts: the loss,
the labels and every generator gradient are BIT-IDENTICAL, f32 and bf16; and
whole steps (critic iterations, the generator iteration, Adam) leave
bit-identical parameters, so the RNG salts continue identically after the
native call.  The native engine is the one that runs (its call counter moves).
"""
import pytest
import torch

from vgan import genstep
from vgan.config import Configuration
from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
from vgan.synth import SyntheticDataset
from vgan.trainer import Trainer

pytestmark = pytest.mark.gpu


def _trainer(cuda, precision="f32", seed=777):
    cfg = Configuration()
    cfg.DEVICE = str(cuda)
    cfg.runtime["rng"] = "device"
    cfg.runtime["precision"] = precision
    cfg.runtime["gen"] = "engine"
    torch.manual_seed(seed)
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    return Trainer(G, D, None, og, od, None, cfg)


def _run(monkeypatch, native: bool, fn):
    monkeypatch.setattr(genstep, "_NATIVE", native)
    return fn()


@pytest.mark.parametrize("batch,precision", [(4, "f32"), (32, "f32"), (32, "bf16")])
def test_native_iteration_is_bit_identical(cuda, monkeypatch, batch, precision):
    from vgan._lib import gemm_precision_scope

    loc, vox = SyntheticDataset(batch, seed=41).batch(range(batch))
    loc, vox = loc.to(cuda), vox.to(cuda)
    a, b = _trainer(cuda, precision), _trainer(cuda, precision)
    for it in range(2):  # the second draws from the advanced device counter and salts
        outs = []
        for tr, native in ((a, True), (b, False)):
            def one():
                with gemm_precision_scope(precision):
                    return tr._gen_iteration(loc, vox)
            g_loss, hard = _run(monkeypatch, native, one)
            outs.append((g_loss.detach().clone(), hard.detach().clone(), tr.flat_g.grad.clone()))
        torch.cuda.synchronize()
        (la, ha, ga), (lb, hb, gb) = outs
        print(f"batch {batch} {precision} iteration {it}: loss native {float(la):.7f} python {float(lb):.7f}; "
              f"max |grad diff| {float((ga - gb).abs().max()):.3e}")
        assert torch.equal(ha, hb), it
        assert torch.equal(la, lb), it
        assert torch.equal(ga, gb), it
    assert a.gen_engine.__dict__.get("native_calls", 0) == 2
    assert b.gen_engine.__dict__.get("native_calls", 0) == 0


def test_native_fresh_steps_are_bit_identical(cuda, monkeypatch):
    """Trainer.step_fresh (the path Trainer.train() takes on a new batch):
    three whole steps with the native generator iteration and three with the
    Python one, from the same state -- bit-identical losses and parameters
    (the critic's draws after the generator's see the same salts)."""
    loc, vox = SyntheticDataset(8, seed=9).batch(range(8))
    loc, vox = loc.to(cuda), vox.to(cuda)
    a, b = _trainer(cuda), _trainer(cuda)
    for k in range(3):
        oa = _run(monkeypatch, True, lambda: a.step_fresh(loc, vox))
        ob = _run(monkeypatch, False, lambda: b.step_fresh(loc, vox))
        torch.cuda.synchronize()
        assert torch.equal(oa["d_losses"], ob["d_losses"]), k
        assert torch.equal(oa["g_loss"], ob["g_loss"]), k
        assert torch.equal(oa["label_hard"], ob["label_hard"]), k
        assert torch.equal(a.flat_g.param, b.flat_g.param), k
        assert torch.equal(a.flat_d.param, b.flat_d.param), k
    assert a.gen_engine.__dict__.get("native_calls", 0) == 3


def test_native_iteration_inside_graph_capture(cuda, monkeypatch):
    """step_graphed records the native iteration (its arena sized by an eager
    step before the capture) and replays it: bit-identical to step_graphed
    recording the Python schedule."""
    loc, vox = SyntheticDataset(8, seed=6).batch(range(8))
    loc, vox = loc.to(cuda), vox.to(cuda)
    a, b = _trainer(cuda), _trainer(cuda)
    _run(monkeypatch, True, lambda: a.step(loc, vox))  # sizes a's arena outside any capture
    _run(monkeypatch, False, lambda: b.step(loc, vox))
    calls = a.gen_engine.__dict__.get("native_calls", 0)
    for k in range(3):
        oa = _run(monkeypatch, True, lambda: a.step_graphed(loc, vox))
        ob = _run(monkeypatch, False, lambda: b.step_graphed(loc, vox))
        torch.cuda.synchronize()
        assert torch.equal(oa["d_losses"], ob["d_losses"]), k
        assert torch.equal(oa["g_loss"], ob["g_loss"]), k
        assert torch.equal(a.flat_g.param, b.flat_g.param), k
    assert a.gen_engine.__dict__.get("native_calls", 0) > calls  # recorded inside the capture
