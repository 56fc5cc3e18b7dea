"""The training loop the reference's train.py:50 runs (``Trainer.train``) and the
drop-in's state around it, on the GPU.

* one and three epochs of ``train()`` over a GraphStore through the native
  loaders: every epoch figure (the 7-tuple of trainer.py:512-520 and the
  6-tuple of :570-577) equals the reference's own reductions
  (``torch.tensor(list).mean().item()``, ``min``) of sklearn's metrics
  (``oracle.reference.metrics``, the restatement of trainer.py:387-443) over
  the very labels the trainer produced -- including validation batches
  replayed from captured graphs (resident evaluation set);
* a checkpoint written mid-training resumes a fresh Trainer that continues
  bit for bit (models, Adam, scheduler, device RNG stream);
* data parallelism: the RCCL all-reduce recorded inside the step graphs (one
  rank, forced active) changes nothing; two gloo ranks sharing the GPU run
  full steps on their own batches and end with bit-identical parameters.
"""
import os
import subprocess
import sys
import warnings

import pytest
import torch

from oracle import reference as R
from parity_util import PKG_ROOT, ROOT
from vgan.config import Configuration
from vgan.loader import GraphDataLoaders
from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
from vgan.store import write_store
from vgan.synth import SyntheticDataset
from vgan.trainer import Trainer

pytestmark = pytest.mark.gpu


def _cfg(cuda, epochs=1, batch=4):
    cfg = Configuration()
    cfg.DEVICE = str(cuda)
    cfg.EPOCHS = epochs
    cfg.BATCH_SIZE = batch
    cfg.runtime["rng"] = "device"
    return cfg


def _trainer(cfg, loaders=None, log_dir=None, seed=777):
    torch.manual_seed(seed)
    G, D = VoxelGNNGenerator(cfg, 17, 12), VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(og, T_max=cfg.EPOCHS)
    return Trainer(G, D, loaders, og, od, sched, cfg, log_dir=None if log_dir is None else str(log_dir))


def _ref_metrics(cfg, records):
    """trainer.py:497-519 / :553-576 reductions of sklearn's per-batch scores."""
    f1s, per_graph, precs, recs, accs = [], [], [], [], []
    for vox, hard in records:
        f1, pg, prec, rec, acc = R.metrics(cfg, vox, hard.unsqueeze(0) if hard.dim() == 2 else hard)
        f1s.append(f1)
        per_graph.extend(pg)
        precs.append(prec)
        recs.append(rec)
        accs.append(acc)
    mean = lambda v: torch.tensor(v).mean().item()  # noqa: E731
    return mean(f1s), min(per_graph), mean(precs), mean(recs), mean(accs)


def test_train_epochs_figures_match_reference_reductions(cuda, tmp_path):
    store = write_store(str(tmp_path / "store"), SyntheticDataset(16, seed=9))
    cfg = _cfg(cuda, epochs=3)
    torch.manual_seed(cfg.SEED)
    loaders = GraphDataLoaders(cfg, store, device=cuda, resident_eval=True)
    assert len(loaders.train_dataloader) == 3 and len(loaders.validation_dataloader) == 1
    tr = _trainer(cfg, loaders, tmp_path / "run")
    train_rec, eval_rec = [], []
    tr.eval_record = eval_rec
    orig = tr._train_batch

    def rec(loc, vox):
        out = orig(loc, vox)
        train_rec.append((vox, out["label_hard"].squeeze(0).clone(), out["d_losses"].clone(), out["g_loss"].clone()))
        return out

    tr._train_batch = rec
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        history = tr.train()
    # FlatAdam's update is the caller's optimizer.step(): no scheduler-order warning
    assert not [w for w in caught if "lr_scheduler.step()" in str(w.message)]
    assert [h["epoch"] for h in history] == [1, 2, 3]
    for e, h in enumerate(history):
        batches = train_rec[3 * e:3 * e + 3]
        f1, f1_min, prec, rec_, acc = _ref_metrics(cfg, [(v, l) for v, l, _, _ in batches])
        assert h["f1_score_train"] == pytest.approx(f1, abs=1e-7)
        assert h["f1_score_min_train"] == f1_min
        assert (h["precision_score_train"], h["recall_score_train"], h["accuracy_score_train"]) == \
            pytest.approx((prec, rec_, acc), abs=1e-7)
        d_ref = torch.tensor([float(v) for _, _, d, _ in batches for v in d.cpu()]).mean().item()
        g_ref = torch.tensor([float(g) for _, _, _, g in batches]).mean().item()
        assert h["d_loss_train"] == pytest.approx(d_ref, rel=1e-6) and h["g_loss_train"] == pytest.approx(g_ref, rel=1e-6)
        vf1, vmin, vprec, vrec, vacc = _ref_metrics(cfg, eval_rec[e:e + 1])
        assert h["f1_score_validation"] == pytest.approx(vf1, abs=1e-7) and h["f1_score_min_validation"] == vmin
        assert (h["precision_score_validation"], h["recall_score_validation"], h["accuracy_score_validation"]) == \
            pytest.approx((vprec, vrec, vacc), abs=1e-7)
        assert h["f1_score_min_weightedsum"] == pytest.approx(
            h["f1_score_min_train"] * cfg.F1_SCORE_TRAIN_WEIGHT + vmin * cfg.F1_SCORE_VALIDATION_WEIGHT)
    # the resident validation batch: eager (epoch 1), captured (2), replayed (3)
    vox_val = eval_rec[0][0]
    assert eval_rec[1][0] is vox_val and eval_rec[2][0] is vox_val
    assert isinstance(vox_val.derived(f"{tr._graph_key}:eval:1"), tuple)
    assert int(tr.adam_d.step_t.item()) == 3 * 3 * cfg.N_CRITIC and int(tr.adam_g.step_t.item()) == 9
    assert tr.scheduler_generator.last_epoch == 3
    states = torch.load(os.path.join(tr.log_dir, "states.pt"), weights_only=True)
    best = max(history, key=lambda h: h["f1_score_min_weightedsum"])
    assert states["best_f1_score"] == pytest.approx(best["f1_score_min_weightedsum"])
    assert states["epoch_start"] == 3  # bumped by every later non-best epoch, as trainer.py:742-745
    test = tr.test()
    assert set(test) == {"f1_score_test", "f1_score_min_test", "precision_score_test", "recall_score_test",
                         "accuracy_score_test"}
    assert 0.0 <= test["f1_score_test"] <= 1.0


def test_resume_continues_bitwise(cuda, tmp_path):
    cfg = _cfg(cuda, epochs=5)
    loc, vox = SyntheticDataset(16, seed=4).batch(range(4))
    loc, vox = loc.to(cuda), vox.to(cuda)
    a = _trainer(cfg, log_dir=tmp_path)
    for _ in range(2):
        a.step_graphed(loc, vox)
    a.scheduler_generator.step()
    a.save_checkpoint(2, 0.5)
    a.step_graphed(loc, vox)
    torch.cuda.synchronize()
    b = _trainer(cfg, log_dir=tmp_path, seed=99)  # resumes from states.pt
    b.step_graphed(loc, vox)
    torch.cuda.synchronize()
    for x, y in ((a.flat_g.param, b.flat_g.param), (a.flat_d.param, b.flat_d.param),
                 (a.adam_g.exp_avg_sq, b.adam_g.exp_avg_sq), (a.adam_d.exp_avg, b.adam_d.exp_avg)):
        assert torch.equal(x, y)
    assert int(b.adam_g.step_t.item()) == 3 and b.optimizer_generator.param_groups[0]["lr"] == \
        a.optimizer_generator.param_groups[0]["lr"]


def test_step_fresh_matches_eager_step(cuda):
    """step_fresh (the critic iteration recorded once per batch, replayed
    N_CRITIC times; labels and generator eager) against the eager step from
    the same state and device-RNG stream, over two new batches (the second
    capture reuses the graph pool and skips the warm-up)."""
    cfg = _cfg(cuda)
    a, b = _trainer(cfg), _trainer(cfg)
    ds = SyntheticDataset(16, seed=4)
    for k in range(2):
        loc, vox = ds.batch(range(4 * k, 4 * k + 4))
        loc, vox = loc.to(cuda), vox.to(cuda)
        oa = a.step(loc, vox)
        ob = b.step_fresh(loc, vox)
        torch.cuda.synchronize()
        da, db = oa["d_losses"].cpu(), ob["d_losses"].cpu()
        print(f"batch {k}: d_losses eager {da.tolist()} fresh {db.tolist()}; "
              f"max |param diff| G {float((a.flat_g.param - b.flat_g.param).abs().max()):.2e} "
              f"D {float((a.flat_d.param - b.flat_d.param).abs().max()):.2e}")
        assert torch.allclose(da, db, rtol=1e-4, atol=1e-5)
        assert abs(float(oa["g_loss"]) - float(ob["g_loss"])) <= 1e-4 * max(1.0, abs(float(oa["g_loss"])))
        # Adam moves near-zero gradient elements by +-lr either way: a handful of
        # sign flips at most, every other parameter equal to rounding
        for x, y in ((a.flat_g.param, b.flat_g.param), (a.flat_d.param, b.flat_d.param)):
            d = (x - y).abs()
            assert float(d.max()) <= 5e-4 and float((d > 1e-6).float().mean()) < 2e-3
        for x, y in ((a, b),):
            assert int(x.adam_d.step_t.item()) == int(y.adam_d.step_t.item()) == (k + 1) * cfg.N_CRITIC
        with torch.no_grad():  # continue from identical state
            for x, y in zip(a._state_tensors(), b._state_tensors()):
                y.copy_(x)


def test_step_fresh_back_to_back_without_sync(cuda):
    """Six new batches through step_fresh with no host synchronisation between
    them (the host records and updates batch k+1's critic graph while batch
    k's replays may still be queued) against the same six batches with a
    device synchronisation after every step: losses, parameters, Adam state
    and RNG counters bit-identical.  An executable graph updated under its own
    queued launches would hand those launches the next batch's arguments."""
    cfg = _cfg(cuda)
    a, b = _trainer(cfg), _trainer(cfg)
    ds = SyntheticDataset(32, seed=11)
    batches = []
    for k in range(6):
        loc, vox = ds.batch(range(4 * k, 4 * k + 4 + (k % 3)))  # sizes vary: updates and re-instantiations
        batches.append((loc.to(cuda), vox.to(cuda)))
    torch.cuda.synchronize()
    outs_a = [a.step_fresh(loc, vox) for loc, vox in batches]  # no sync in between
    outs_b = []
    for loc, vox in batches:
        outs_b.append(b.step_fresh(loc, vox))
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    for k, (oa, ob) in enumerate(zip(outs_a, outs_b)):
        assert torch.equal(oa["d_losses"], ob["d_losses"]), k
        assert torch.equal(oa["g_loss"], ob["g_loss"]), k
    for x, y in zip(a._state_tensors(), b._state_tensors()):
        assert torch.equal(x, y)


def _run_worker(args, timeout=300):
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, PKG_ROOT, os.path.dirname(__file__)]))
    proc = subprocess.run([sys.executable, "-u", os.path.join(os.path.dirname(__file__), "dist_gpu_worker.py")]
                          + args, env=env, capture_output=True, text=True, timeout=timeout)
    print(proc.stdout[-3000:], proc.stderr[-3000:])
    assert proc.returncode == 0, proc.stderr[-3000:]
    return proc.stdout


def test_rccl_all_reduce_recorded_in_step_graphs(cuda):
    """One rank over RCCL with the gradient sync forced on: the all-reduce is
    recorded inside the critic and generator graphs, and the trajectory is
    bit-identical to the single-process step (a one-rank sum is exact) --
    for replays of a cached batch and for three new batches through
    step_fresh (the collective recorded per batch, the executable graph
    updated in place)."""
    out = _run_worker(["rccl1"])
    assert "RCCL_GRAPH_OK" in out


def test_gloo_two_ranks_full_steps_identical_parameters(cuda):
    """Two ranks (gloo, sharing the one GPU) each train on their own batch:
    2 eager steps + 1 graphed step.  Parameters stay bit-identical across
    ranks (averaged gradients, identical Adam), the losses differ (different
    buildings and draws)."""
    out = _run_worker(["gloo2"])
    # the two ranks share one stdout: a line may land inside the other's
    import re

    lines = re.findall(r"RANK \d+ \S+ \S+ \S+ \d+", out)
    assert len(lines) == 2, out
    r0, r1 = (l.split() for l in sorted(lines))
    assert r0[2] == r1[2] and r0[3] == r1[3]  # parameter digests (G, D)
    assert r0[4] != r1[4]  # d_loss of the last step: own batch, own draws
    assert r0[5] != r1[5]  # device RNG seeds
