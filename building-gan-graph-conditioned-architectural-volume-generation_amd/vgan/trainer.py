"""Trainer with the reference surface plus an explicit, sync-free ``step``.

Mirrors ``building_gan/src/trainer.py``:

* ``Trainer(generator, discriminator, dataloaders, optimizer_generator,
  optimizer_discriminator, scheduler_generator, configuration, log_dir=None)``
  (``trainer.py:581-591``), ``.train()`` (``:641``), ``.test(n)`` (``:750``);
* ``_compute_gradient_penalty`` / ``_compute_discriminator_loss`` /
  ``_compute_generator_loss`` / ``_compute_metrics`` with the reference's
  arithmetic (``:291-443``);
* ``step(local_graph, voxel_graph)`` is the loop body of ``_train_each_epoch``
  (``:461-502``) factored out: N_CRITIC x {no-grad G forward, D zero_grad,
  WGAN-GP D loss, backward, Adam} then {G forward, G zero_grad, G loss,
  backward, Adam}.  It performs no host synchronisation: losses stay on the
  device until the caller reads them.

Differences that do not change results:

* parameters live in flat buffers, Adam is one kernel (``vgan.flat``); the
  caller's optimizers are the hyper-parameter source (a scheduler on them keeps
  working);
* in the generator iteration the discriminator's parameter gradients are not
  formed: the reference computes them at ``:492`` and discards them (the next
  critic iteration zeroes them at ``:475`` before any use);
* with more than one rank the flat gradients are averaged over RCCL after
  every backward (``vgan.dist``).
"""
from __future__ import annotations

import datetime
import itertools
import os
import time
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import data as vdata
from . import metrics as vmetrics
from . import ops
from ._lib import gemm_precision_scope
from .critic import CriticEngine
from .dist import GradSync
from .flat import FlatAdam, FlatParams
from .rng import RNG

_TRAINER_IDS = itertools.count()


class Trainer:
    def __init__(self, generator, discriminator, dataloaders, optimizer_generator, optimizer_discriminator,
                 scheduler_generator, configuration, log_dir: Optional[str] = None):
        self.generator = generator
        self.discriminator = discriminator
        self.dataloaders = dataloaders
        self.optimizer_generator = optimizer_generator
        self.optimizer_discriminator = optimizer_discriminator
        self.scheduler_generator = scheduler_generator
        self.configuration = configuration
        self.sanity_checking = getattr(configuration, "SANITY_CHECKING", False)
        self.log_dir = log_dir or os.path.join(configuration.LOG_DIR,
                                               datetime.datetime.now().strftime("%m-%d-%Y__%H-%M-%S"))
        runtime = getattr(configuration, "runtime", {})
        # data-parallel rank: the process group's when one is initialised (every
        # rank builds its models after the same torch.manual_seed, so the rank
        # term is what gives ranks different z / dropout / Gumbel / eps draws)
        rank = int(runtime.get("rank", 0))
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            rank = torch.distributed.get_rank()
        self.rank = rank
        self.rng = RNG(runtime.get("rng", "device"), seed=torch.initial_seed() + 7919 * rank)
        generator.rng = self.rng
        discriminator.rng = self.rng
        self.flat_g = FlatParams(generator)
        self.flat_d = FlatParams(discriminator)
        self.adam_g = FlatAdam.from_optimizer(self.flat_g, optimizer_generator)
        self.adam_d = FlatAdam.from_optimizer(self.flat_d, optimizer_discriminator)
        self.sync = GradSync()
        self.sync.broadcast_params(self.flat_g)
        self.sync.broadcast_params(self.flat_d)
        self.skip_dead_d_grads = runtime.get("skip_dead_d_grads", True)
        # critic iterations: the explicit four-pass engine (vgan/critic.py) or
        # autograd double backward through the differentiable HIP ops
        # (vg_gp_head holds a row's classes in registers: K <= 32)
        use_engine = (runtime.get("critic", "engine") == "engine" and getattr(configuration, "USE_WGANGP", True)
                      and int(configuration.NUM_CLASSES) <= 32)
        self.critic = CriticEngine(discriminator, configuration) if use_engine else None
        self.states = {"epoch_start": 1, "best_f1_score": 0.0}
        # captured step graphs are cached on the batch, per trainer (two
        # trainers -- e.g. f32 and bf16 -- may step the same batch)
        self._graph_key = f"step_graphs:{next(_TRAINER_IDS)}"
        # operand precision of the dense products: "f32" (configs[1], the
        # reference's) or "bf16" (configs[2]: bf16 operands, f32 accumulate)
        self.precision = runtime.get("precision", "f32")
        if self.precision not in ("f32", "bf16"):
            raise ValueError(f"runtime['precision'] must be 'f32' or 'bf16', not {self.precision!r}")

    def _critic_loss_backward(self, local_graph, voxel_graph, label_hard, label_soft) -> torch.Tensor:
        """d_loss of trainer.py:476-479 with D's gradients accumulated into .grad."""
        if self.critic is not None:
            return self.critic.loss_and_grad(local_graph, voxel_graph, label_hard, label_soft, self.rng)
        d_loss = self._compute_discriminator_loss(local_graph, voxel_graph, label_hard, label_soft)
        d_loss.backward()
        return d_loss

    # ------------------------------------------------------------- losses
    def _compute_gradient_penalty(self, local_graph, voxel_graph, label_soft):
        """trainer.py:291-316."""
        cfg = self.configuration
        prep = vdata.prepared(local_graph, voxel_graph, cfg.NUM_CLASSES)
        n = prep.onehot_f.shape[0]
        eps = self.rng.uniform((n, 1), label_soft.device)
        mix = (eps * prep.onehot_f + (1 - eps) * label_soft.squeeze(0)).requires_grad_(True)
        score = self.discriminator(local_graph, voxel_graph, mix.unsqueeze(0))
        (grad,) = torch.autograd.grad(score, mix, torch.ones_like(score), create_graph=True, only_inputs=True)
        return ((grad.norm(dim=1) - 1) ** 2).mean() * cfg.LAMBDA_GP

    def _compute_discriminator_loss(self, local_graph, voxel_graph, label_hard, label_soft):
        """trainer.py:318-332."""
        prep = vdata.prepared(local_graph, voxel_graph, self.configuration.NUM_CLASSES)
        d_real = self.discriminator(local_graph, voxel_graph, prep.onehot_f.unsqueeze(0))
        d_fake = self.discriminator(local_graph, voxel_graph, label_hard)
        if self.configuration.USE_WGANGP:
            d_loss = d_fake.mean() - d_real.mean()
            return d_loss + self._compute_gradient_penalty(local_graph, voxel_graph, label_soft)
        return (F.binary_cross_entropy(d_fake, torch.zeros_like(d_fake))
                + F.binary_cross_entropy(d_real, torch.ones_like(d_real)))

    def _compute_generator_loss(self, local_graph, voxel_graph, logits, label_hard):
        """trainer.py:334-385 (the per-building FAR loop is one kernel)."""
        cfg = self.configuration
        prep = vdata.prepared(local_graph, voxel_graph, cfg.NUM_CLASSES)
        d_fake = self.discriminator(local_graph, voxel_graph, label_hard)
        hard = label_hard.squeeze(0)
        if cfg.USE_WGANGP and cfg.NUM_CLASSES > 2:  # fused loss head: same terms, same order
            far_gen, far_ref = ops.far_per_graph(prep.voxel_x, hard, voxel_graph.ptr, voxel_graph.site_area,
                                                 far_col=9, dy_col=4, dx_col=5,
                                                 dim_scale=float(cfg.NORMALIZATION_FACTOR_DIMENSION),
                                                 void_class=cfg.VOID)
            return ops.gen_loss_head(d_fake, hard, logits, prep.onehot_f, voxel_graph.type, far_gen, far_ref,
                                     (cfg.LAMBDA_ADV, cfg.LAMBDA_LABEL, cfg.LAMBDA_RATIO, cfg.LAMBDA_RATIO_VOID,
                                      cfg.LAMBDA_FAR))
        if cfg.USE_WGANGP:
            adv = -d_fake.mean()
        else:
            adv = F.binary_cross_entropy(d_fake, torch.ones_like(d_fake))
        adv = adv * cfg.LAMBDA_ADV
        ce = F.cross_entropy(logits, voxel_graph.type) * cfg.LAMBDA_LABEL
        n = prep.onehot_f.shape[0]
        ratio_gen = hard.sum(dim=0) / n
        ratio_ref = prep.onehot_f.sum(dim=0) / n
        ratio = F.mse_loss(ratio_gen[:-2], ratio_ref[:-2]) * cfg.LAMBDA_RATIO
        ratio_void = F.mse_loss(ratio_gen[-2:], ratio_ref[-2:]) * cfg.LAMBDA_RATIO_VOID
        far_gen, far_ref = ops.far_per_graph(prep.voxel_x, hard, voxel_graph.ptr, voxel_graph.site_area,
                                             far_col=9, dy_col=4, dx_col=5,
                                             dim_scale=float(cfg.NORMALIZATION_FACTOR_DIMENSION),
                                             void_class=cfg.VOID)
        far = F.mse_loss(far_gen, far_ref) * cfg.LAMBDA_FAR  # no gradient, as at trainer.py:380
        return adv + ratio + ce + ratio_void + far

    def _compute_metrics(self, voxel_graph, label_hard):
        """trainer.py:387-443 via device confusion matrices (one D2H copy)."""
        conf, conf_all = ops.confusion(voxel_graph.type, label_hard.squeeze(0), voxel_graph.ptr)
        return vmetrics.batch_metrics(conf.cpu().numpy(), conf_all.cpu().numpy())

    # --------------------------------------------------------------- step
    def _generate(self, local_graph, voxel_graph):
        z = self.rng.normal((1, voxel_graph.num_nodes, self.configuration.Z_DIM), voxel_graph.x.device)
        logits, hard, soft = self.generator(local_graph, voxel_graph, z)
        return logits, hard.unsqueeze(0), soft.unsqueeze(0)

    def _stacked_labels(self) -> bool:
        """Generate all N_CRITIC critic-iteration labels in one stacked G
        forward?  G is not updated during the critic iterations
        (trainer.py:466-481), so the N_CRITIC no-grad forwards differ only in
        their random draws; with device RNG they run as one forward over
        N_CRITIC stacked copies.  Host / fixed RNG keep the reference's
        per-iteration draw order."""
        return (self.rng.mode == "device" and self.configuration.N_CRITIC > 1
                and getattr(self.configuration, "runtime", {}).get("stack_critic_g", True))

    def _critic_labels(self, local_graph, voxel_graph):
        """[N_CRITIC, N, 7] (hard, soft) from one stacked no-grad G forward."""
        self.rng.reset()
        z = self.rng.normal((self.configuration.N_CRITIC, voxel_graph.num_nodes, self.configuration.Z_DIM),
                            voxel_graph.x.device)
        with torch.no_grad():
            _, hard, soft = self.generator(local_graph, voxel_graph, z)
        return hard, soft

    def _critic_iteration(self, local_graph, voxel_graph, labels, i: int) -> torch.Tensor:
        self.rng.reset()
        if labels is not None:
            hard, soft = labels[0][i:i + 1], labels[1][i:i + 1]
        else:
            with torch.no_grad():
                _, hard, soft = self._generate(local_graph, voxel_graph)
        self.adam_d.zero_grad()
        return self._critic_loss_backward(local_graph, voxel_graph, hard, soft)

    def _gen_iteration(self, local_graph, voxel_graph):
        self.rng.reset()
        logits, hard, _ = self._generate(local_graph, voxel_graph)
        self.adam_g.zero_grad()
        d_params = list(self.discriminator.parameters())
        if self.skip_dead_d_grads:
            for p in d_params:
                p.requires_grad_(False)
        try:
            g_loss = self._compute_generator_loss(local_graph, voxel_graph, logits, hard)
            with ops.direct_param_grads(), ops.deferred_param_folds(g_loss.device):
                g_loss.backward()
        finally:
            if self.skip_dead_d_grads:
                for p in d_params:
                    p.requires_grad_(True)
        return g_loss, hard

    def step(self, local_graph, voxel_graph) -> Dict[str, torch.Tensor]:
        """One full G+D step (trainer.py:466-495); returns device tensors."""
        with gemm_precision_scope(self.precision):
            return self._step(local_graph, voxel_graph)

    def _step(self, local_graph, voxel_graph) -> Dict[str, torch.Tensor]:
        cfg = self.configuration
        labels = self._critic_labels(local_graph, voxel_graph) if self._stacked_labels() else None
        d_losses: List[torch.Tensor] = []
        for i in range(cfg.N_CRITIC):
            d_loss = self._critic_iteration(local_graph, voxel_graph, labels, i)
            d_losses.append(d_loss.detach())
            self.sync.all_reduce_grad(self.flat_d)
            self.adam_d.step()
        g_loss, hard = self._gen_iteration(local_graph, voxel_graph)
        self.sync.all_reduce_grad(self.flat_g)
        self.adam_g.step()
        return {"d_losses": torch.stack(d_losses), "g_loss": g_loss.detach(), "label_hard": hard.detach()}

    # ------------------------------------------------- hipGraph-captured step
    def _critic_body(self, local_graph, voxel_graph, acc, with_adam: bool, labels=None, i: int = 0):
        d_loss = self._critic_iteration(local_graph, voxel_graph, labels, i)
        acc[0].add_(d_loss.detach())
        if with_adam:
            self.adam_d.step()

    def _gen_body(self, local_graph, voxel_graph, acc, with_adam: bool):
        g_loss, hard = self._gen_iteration(local_graph, voxel_graph)
        acc[1].copy_(g_loss.detach())
        if with_adam:
            self.adam_g.step()
        return hard.detach()

    def _snapshot(self):
        return [t.clone() for t in (self.flat_g.param, self.flat_d.param, self.adam_g.exp_avg, self.adam_g.exp_avg_sq,
                                    self.adam_d.exp_avg, self.adam_d.exp_avg_sq, self.adam_g.step_t,
                                    self.adam_d.step_t)]

    def _restore(self, snap):
        dst = (self.flat_g.param, self.flat_d.param, self.adam_g.exp_avg, self.adam_g.exp_avg_sq,
               self.adam_d.exp_avg, self.adam_d.exp_avg_sq, self.adam_g.step_t, self.adam_d.step_t)
        for d, s_ in zip(dst, snap):
            d.copy_(s_)

    def capture(self, local_graph, voxel_graph):
        with gemm_precision_scope(self.precision):
            return self._capture(local_graph, voxel_graph)

    def _capture(self, local_graph, voxel_graph):
        """Record the step of this (static) batch as hipGraphs.

        * stacked labels (device RNG): one graph for the stacked critic-label
          G forward, one per critic iteration (each reads its own label slice)
          and one for the generator iteration;
        * otherwise: one critic-iteration graph replayed N_CRITIC times and the
          generator graph.
        RNG counters, parameters and Adam state advance in place on the device.
        With several ranks the RCCL all-reduce and Adam run eagerly between
        replays.  Needs device-side randomness (device or fixed RNG)."""
        if self.rng.mode == "host":
            raise RuntimeError("graph capture needs device-side randomness (runtime['rng'] 'device')")
        dev = voxel_graph.x.device
        n_critic = self.configuration.N_CRITIC
        with_adam = not self.sync.active
        stacked = self._stacked_labels()
        acc = torch.zeros(2, dtype=torch.float32, device=dev)
        vdata.prepared(local_graph, voxel_graph, self.configuration.NUM_CLASSES)  # CSR etc. before capture
        self.adam_g.sync_lr()
        self.adam_d.sync_lr()
        snap = self._snapshot()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up (lazy init) on a side stream, then undo it
            labels = self._critic_labels(local_graph, voxel_graph) if stacked else None
            self._critic_body(local_graph, voxel_graph, acc, with_adam, labels, 0)
            self._gen_body(local_graph, voxel_graph, acc, with_adam)
        torch.cuda.current_stream(dev).wait_stream(side)
        self._restore(snap)
        pool = getattr(self, "_graph_pool", None)
        if pool is None:
            pool = self._graph_pool = torch.cuda.graph_pool_handle()
        g_labels, labels = None, None
        if stacked:
            g_labels = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_labels, pool=pool):
                labels = self._critic_labels(local_graph, voxel_graph)
        critic = []
        for i in range(n_critic if stacked else 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                self._critic_body(local_graph, voxel_graph, acc, with_adam, labels, i)
            critic.append(g)
        g_gen = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_gen, pool=pool):
            hard = self._gen_body(local_graph, voxel_graph, acc, with_adam)
        self._restore(snap)
        graphs = {"labels": g_labels, "label_tensors": labels, "critic": critic, "gen": g_gen, "acc": acc,
                  "hard": hard, "with_adam": with_adam}
        voxel_graph.set_derived(self._graph_key, graphs)
        return graphs

    def step_graphed(self, local_graph, voxel_graph) -> Dict[str, torch.Tensor]:
        """``step`` replayed from hipGraphs (captured on first use per batch)."""
        graphs = voxel_graph.derived(self._graph_key) if callable(getattr(voxel_graph, "derived", None)) else None
        if graphs is None:
            graphs = self.capture(local_graph, voxel_graph)
        self.adam_g.sync_lr()
        self.adam_d.sync_lr()
        acc = graphs["acc"]
        acc.zero_()
        if graphs["labels"] is not None:
            graphs["labels"].replay()
        critic = graphs["critic"]
        for i in range(self.configuration.N_CRITIC):
            critic[i if len(critic) > 1 else 0].replay()
            if not graphs["with_adam"]:
                self.sync.all_reduce_grad(self.flat_d)
                self.adam_d.step()
        graphs["gen"].replay()
        if not graphs["with_adam"]:
            self.sync.all_reduce_grad(self.flat_g)
            self.adam_g.step()
        return {"d_loss_mean": acc[0] / self.configuration.N_CRITIC, "g_loss": acc[1], "label_hard": graphs["hard"]}

    # ------------------------------------------------------ orchestration
    def _train_each_epoch(self):
        start = time.time()
        g_losses, d_losses, f1s, f1_graphs, precs, recs, accs = [], [], [], [], [], [], []
        for local_graph, voxel_graph in self.dataloaders.train_dataloader:
            local_graph = local_graph.to(self.configuration.DEVICE)
            voxel_graph = voxel_graph.to(self.configuration.DEVICE)
            assert [set(d) for d in local_graph.data_number] == [set(d) for d in voxel_graph.data_number]
            out = self.step(local_graph, voxel_graph)
            d_losses.append(out["d_losses"])
            g_losses.append(out["g_loss"])
            f1, per_graph, prec, rec, acc = self._compute_metrics(voxel_graph, out["label_hard"])
            f1s.append(f1)
            f1_graphs.extend(per_graph)
            precs.append(prec)
            recs.append(rec)
            accs.append(acc)
        # epoch means of the losses averaged over the data-parallel ranks (one
        # collective per epoch); the F1 / precision / recall are this rank's
        means = self.sync.all_reduce_scalars(torch.stack([torch.stack(g_losses).mean(), torch.cat(d_losses).mean()]))
        g_mean, d_mean = (float(v) for v in means.tolist())
        print(f"The function _train_each_epoch took {time.time() - start} seconds to run.")
        return (g_mean, d_mean, float(np.mean(f1s)), min(f1_graphs), float(np.mean(precs)), float(np.mean(recs)),
                float(np.mean(accs)))

    @torch.no_grad()
    def _validate_each_epoch(self):
        if self.sanity_checking or getattr(self.dataloaders, "validation_dataloader", None) is None:
            return 0.0, 0.0, 0.0, 0.0, 0.0, 0.0
        self.generator.eval()
        self.discriminator.eval()
        g_losses, f1s, f1_graphs, precs, recs, accs = [], [], [], [], [], []
        for local_graph, voxel_graph in self.dataloaders.validation_dataloader:
            local_graph = local_graph.to(self.configuration.DEVICE)
            voxel_graph = voxel_graph.to(self.configuration.DEVICE)
            with gemm_precision_scope(self.precision):
                logits, hard, _ = self._generate(local_graph, voxel_graph)
            g_losses.append(self._compute_generator_loss(local_graph, voxel_graph, logits, hard))
            f1, per_graph, prec, rec, acc = self._compute_metrics(voxel_graph, hard)
            f1s.append(f1)
            f1_graphs.extend(per_graph)
            precs.append(prec)
            recs.append(rec)
            accs.append(acc)
        self.generator.train()
        self.discriminator.train()
        return (torch.stack(g_losses).mean().item(), float(np.mean(f1s)), min(f1_graphs), float(np.mean(precs)),
                float(np.mean(recs)), float(np.mean(accs)))

    def train(self):
        """Epoch loop of trainer.py:641-747 (metrics printed; checkpoint on best
        weighted min-F1 with the reference's states.pt keys)."""
        cfg = self.configuration
        best = self.states["best_f1_score"]
        for epoch in range(self.states["epoch_start"], cfg.EPOCHS + 1):
            tr = self._train_each_epoch()
            va = self._validate_each_epoch()
            score = tr[3] * cfg.F1_SCORE_TRAIN_WEIGHT + va[2] * cfg.F1_SCORE_VALIDATION_WEIGHT
            print(f"epoch {epoch}: g_loss {tr[0]:.5f} d_loss {tr[1]:.5f} f1 {tr[2]:.4f} f1_val {va[1]:.4f}")
            if best < score:
                best = score
                if not self.sanity_checking:
                    self.save_checkpoint(epoch, best)
            if self.scheduler_generator is not None:
                self.scheduler_generator.step()

    def save_checkpoint(self, epoch: int, best: float) -> str:
        os.makedirs(self.log_dir, exist_ok=True)
        path = os.path.join(self.log_dir, "states.pt")
        torch.save({
            "epoch_start": epoch,
            "epoch_end": self.configuration.EPOCHS + 1,
            "best_f1_score": best,
            "generator": self.generator.state_dict(),
            "discriminator": self.discriminator.state_dict(),
            "optimizer_generator_flat": self.adam_g.state_dict_flat(),
            "optimizer_discriminator_flat": self.adam_d.state_dict_flat(),
        }, path)
        return path

    @torch.no_grad()
    def test(self, num_samples_to_viz: int = 0):
        """trainer.py:749-795 metrics (visualisation is out of scope)."""
        self.generator.eval()
        self.discriminator.eval()
        f1s, f1_graphs, precs, recs, accs = [], [], [], [], []
        for local_graph, voxel_graph in self.dataloaders.test_dataloader:
            local_graph = local_graph.to(self.configuration.DEVICE)
            voxel_graph = voxel_graph.to(self.configuration.DEVICE)
            with gemm_precision_scope(self.precision):
                _, hard, _ = self._generate(local_graph, voxel_graph)
            f1, per_graph, prec, rec, acc = self._compute_metrics(voxel_graph, hard)
            f1s.append(f1)
            f1_graphs.extend(per_graph)
            precs.append(prec)
            recs.append(rec)
            accs.append(acc)
        self.generator.train()
        self.discriminator.train()
        result = {"f1_score_test": float(np.mean(f1s)), "f1_score_min_test": min(f1_graphs),
                  "precision_score_test": float(np.mean(precs)), "recall_score_test": float(np.mean(recs)),
                  "accuracy_score_test": float(np.mean(accs))}
        print(result)
        return result
