"""states.pt compatibility with the reference trainer (trainer.py:608-636 load,
:715-736 save), on the CPU: the checkpoint logic is host code (the flat Adam
moments are exported to / imported from torch.optim.Adam state dicts).

* a vgan checkpoint has exactly the reference's keys (plus ``vgan_rng``) and
  its optimizer / model state dicts load into a plain torch Adam over the
  oracle's restatement of the reference models -- what the reference's own
  ``Trainer.__init__`` does with it;
* a checkpoint built the reference's way (torch Adam after real steps) resumes
  a vgan Trainer with the same parameters, moments, step and learning rate;
* save -> new Trainer on the same log_dir -> identical state.
"""
import os

import pytest
import torch

from oracle import reference as R
from vgan.config import Configuration
from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
from vgan.trainer import Trainer

REF_KEYS = {"epoch_start", "epoch_end", "best_f1_score", "f1_score_train", "f1_score_validation",
            "f1_score_min_train", "f1_score_min_validation", "f1_score_min_weightedsum", "recall_score_train",
            "recall_score_validation", "accuracy_score_train", "accuracy_score_validation", "generator",
            "discriminator", "optimizer_generator", "optimizer_discriminator", "scheduler_generator"}


def _cfg():
    cfg = Configuration()
    cfg.DEVICE = "cpu"
    cfg.EPOCHS = 10
    return cfg


def _trainer(cfg, log_dir, seed=777):
    torch.manual_seed(seed)
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(og, T_max=cfg.EPOCHS)
    return Trainer(G, D, None, og, od, sched, cfg, log_dir=str(log_dir))


def _perturb(tr, seed=3):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for flat, adam, step in ((tr.flat_g, tr.adam_g, 7), (tr.flat_d, tr.adam_d, 12)):
            live = flat.live_mask()  # the alignment gaps stay zero
            flat.param.add_(0.01 * torch.randn(flat.param.shape, generator=g) * live)
            adam.exp_avg.copy_(torch.randn(flat.param.shape, generator=g) * live)
            adam.exp_avg_sq.copy_(torch.rand(flat.param.shape, generator=g) * live)
            adam.step_t.fill_(step)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # scheduler.step() before optimizer.step()
        for _ in range(3):
            tr.scheduler_generator.step()


def test_checkpoint_has_reference_keys_and_loads_into_torch_adam(tmp_path):
    cfg = _cfg()
    tr = _trainer(cfg, tmp_path)
    _perturb(tr)
    figures = {"f1_score_train": 0.5, "f1_score_min_validation": 0.25}
    path = tr.save_checkpoint(4, 0.75, figures)
    states = torch.load(path, map_location="cpu", weights_only=True)
    assert set(states) == REF_KEYS | {"vgan_rng"}
    assert states["epoch_start"] == 4 and states["epoch_end"] == cfg.EPOCHS + 1 and states["best_f1_score"] == 0.75
    assert states["f1_score_train"] == 0.5 and states["f1_score_min_validation"] == 0.25
    # the reference's resume (trainer.py:630-634) on its own model classes
    torch.manual_seed(1)
    Gr, Dr = R.Generator(cfg), R.Discriminator(cfg)
    Gr.load_state_dict(states["generator"])
    Dr.load_state_dict(states["discriminator"])
    og = torch.optim.Adam(Gr.parameters(), lr=1.0, betas=cfg.BETAS)
    od = torch.optim.Adam(Dr.parameters(), lr=1.0, betas=cfg.BETAS)
    og.load_state_dict(states["optimizer_generator"])
    od.load_state_dict(states["optimizer_discriminator"])
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(og, T_max=cfg.EPOCHS)
    sched.load_state_dict(states["scheduler_generator"])
    assert og.param_groups[0]["lr"] == tr.optimizer_generator.param_groups[0]["lr"]
    for (name, p), (name2, q) in zip(Gr.named_parameters(), tr.generator.named_parameters()):
        assert name == name2 and torch.equal(p, q)
        st = og.state[p]
        off = tr.flat_g._offset(q)
        assert float(st["step"]) == 7.0
        assert torch.equal(st["exp_avg"].reshape(-1), tr.adam_g.exp_avg[off:off + q.numel()])
        assert torch.equal(st["exp_avg_sq"].reshape(-1), tr.adam_g.exp_avg_sq[off:off + q.numel()])
    assert all(float(s["step"]) == 12.0 for s in od.state.values()) and len(od.state) == len(list(Dr.parameters()))


def test_resume_from_reference_written_checkpoint(tmp_path):
    """A states.pt written the reference's way -- torch Adam after real steps,
    CosineAnnealingLR, its exact keys -- resumes a vgan Trainer."""
    cfg = _cfg()
    torch.manual_seed(5)
    Gr, Dr = R.Generator(cfg), R.Discriminator(cfg)
    og = torch.optim.Adam(Gr.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(Dr.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(og, T_max=cfg.EPOCHS)
    for _ in range(2):
        for m, opt in ((Gr, og), (Dr, od)):
            opt.zero_grad()
            for p in m.parameters():
                p.grad = torch.randn_like(p)
            opt.step()
        sched.step()
    states = {"epoch_start": 3, "epoch_end": cfg.EPOCHS + 1, "best_f1_score": 0.5, "f1_score_train": 0.1,
              "f1_score_validation": 0.2, "f1_score_min_train": 0.3, "f1_score_min_validation": 0.4,
              "f1_score_min_weightedsum": 0.5, "recall_score_train": 0.6, "recall_score_validation": 0.7,
              "accuracy_score_train": 0.8, "accuracy_score_validation": 0.9,
              "generator": Gr.state_dict(), "discriminator": Dr.state_dict(),
              "optimizer_generator": og.state_dict(), "optimizer_discriminator": od.state_dict(),
              "scheduler_generator": sched.state_dict()}
    os.makedirs(tmp_path, exist_ok=True)
    torch.save(states, os.path.join(tmp_path, "states.pt"))
    tr = _trainer(cfg, tmp_path, seed=11)  # different init: everything must come from the file
    assert tr.states["epoch_start"] == 3 and tr.states["best_f1_score"] == 0.5
    assert tr.scheduler_generator.last_epoch == 2
    assert tr.optimizer_generator.param_groups[0]["lr"] == og.param_groups[0]["lr"]
    for (flat, adam, ref_m, ref_opt, m) in ((tr.flat_g, tr.adam_g, Gr, og, tr.generator),
                                            (tr.flat_d, tr.adam_d, Dr, od, tr.discriminator)):
        assert int(adam.step_t.item()) == 2
        for (name, p), (_, q) in zip(ref_m.named_parameters(), m.named_parameters()):
            assert torch.equal(p, q), name
            off = flat._offset(q)
            assert torch.equal(ref_opt.state[p]["exp_avg"].reshape(-1), adam.exp_avg[off:off + q.numel()]), name
            assert torch.equal(ref_opt.state[p]["exp_avg_sq"].reshape(-1), adam.exp_avg_sq[off:off + q.numel()])


def test_save_resume_round_trip(tmp_path):
    cfg = _cfg()
    tr = _trainer(cfg, tmp_path)
    _perturb(tr)
    tr.save_checkpoint(6, 0.9)
    tr2 = _trainer(cfg, tmp_path, seed=123)
    for a, b in ((tr.flat_g.param, tr2.flat_g.param), (tr.flat_d.param, tr2.flat_d.param),
                 (tr.adam_g.exp_avg, tr2.adam_g.exp_avg), (tr.adam_g.exp_avg_sq, tr2.adam_g.exp_avg_sq),
                 (tr.adam_d.exp_avg, tr2.adam_d.exp_avg), (tr.adam_d.exp_avg_sq, tr2.adam_d.exp_avg_sq),
                 (tr.adam_g.step_t, tr2.adam_g.step_t), (tr.adam_d.step_t, tr2.adam_d.step_t)):
        assert torch.equal(a, b)
    assert tr2.scheduler_generator.last_epoch == tr.scheduler_generator.last_epoch
    assert float(tr2.adam_g.lr_t.item()) == tr.optimizer_generator.param_groups[0]["lr"]
    assert tr2.states["epoch_start"] == 6
    # a non-best epoch moves only epoch_start (trainer.py:742-745)
    tr2._bump_epoch_start(7)
    assert torch.load(os.path.join(tmp_path, "states.pt"), weights_only=True)["epoch_start"] == 7


def test_flat_adam_state_dict_is_torch_adam_format(tmp_path):
    """FlatAdam's own state_dict (no caller optimizer) loads into a torch Adam."""
    cfg = _cfg()
    torch.manual_seed(2)
    G = VoxelGNNGenerator(cfg, 17, 12)
    from vgan.flat import FlatAdam, FlatParams

    flat = FlatParams(G)
    adam = FlatAdam(flat, lr=3e-4, betas=(0.5, 0.999))
    adam.exp_avg.normal_().mul_(flat.live_mask())  # the alignment gaps stay zero
    adam.exp_avg_sq.uniform_().mul_(flat.live_mask())
    adam.step_t.fill_(4)
    sd = adam.state_dict()
    ref = torch.optim.Adam(G.parameters(), lr=1.0)
    ref.load_state_dict(sd)
    assert ref.param_groups[0]["lr"] == 3e-4 and ref.param_groups[0]["betas"] == (0.5, 0.999)
    adam2 = FlatAdam(flat)
    adam2.load_state_dict(ref.state_dict())
    assert torch.equal(adam2.exp_avg, adam.exp_avg) and torch.equal(adam2.exp_avg_sq, adam.exp_avg_sq)
    assert int(adam2.step_t.item()) == 4 and adam2.param_groups[0]["lr"] == 3e-4
    with pytest.raises(ValueError):  # moments at different steps cannot share one flat step
        st = ref.state_dict()
        first = next(iter(st["state"]))
        st["state"][first]["step"] = torch.tensor(9.0)
        ref.load_state_dict(st)
        adam2.import_from(ref)


def test_flat_params_aligned_views():
    """Every parameter view starts on a 128-byte boundary of the flat buffer
    (the GEMMs' float4 operand loads need 16-byte-aligned weights), holds the
    module's initial values, and the gaps between views stay zero."""
    cfg = _cfg()
    torch.manual_seed(4)
    G = VoxelGNNGenerator(cfg, 17, 12)
    from vgan.flat import ALIGN, FlatParams

    init = {k: p.detach().clone() for k, p in G.named_parameters()}
    flat = FlatParams(G)
    assert ALIGN * 4 % 128 == 0
    for k, p in G.named_parameters():
        assert (p.data_ptr() - flat.param.data_ptr()) % 128 == 0, k
        assert p.grad is not None and p.grad.data_ptr() - flat.grad.data_ptr() == p.data_ptr() - flat.param.data_ptr()
        assert torch.equal(p.detach(), init[k]), k
    live = flat.live_mask()
    assert int(live.sum()) == flat.num_params == 274185
    assert flat.numel >= flat.num_params and not flat.param[~live].any() and not flat.grad[~live].any()


def test_rng_state_before_the_device_counter_exists():
    """RNG.state_dict taken after resets but before the device counter was
    created records those resets: the resumed stream starts where the
    original one would have (not at iteration 0)."""
    from vgan.rng import RNG

    a = RNG("device", seed=5)
    for _ in range(3):
        a.reset()
    st = a.state_dict()
    assert st["iter"] == 3
    b = RNG("device", seed=1)
    b.load_state_dict(st)
    assert b.seed == 5 and b._pending_iter + b._early == 3
    b.reset()
    assert b.state_dict()["iter"] == 4
