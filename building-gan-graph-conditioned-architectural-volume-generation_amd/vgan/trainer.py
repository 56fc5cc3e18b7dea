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

import ctypes
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
from ._lib import LIB, check, gemm_precision_scope, ptr, stream_handle
from .critic import CriticEngine
from .dist import GradSync
from .flat import FlatAdam, FlatParams
from .gcscope import gc_frozen
from .genstep import GeneratorEngine
from .rng import RNG

_TRAINER_IDS = itertools.count()
# VGAN_FRESH_UPDATE=0: instantiate every fresh batch's critic graph (A/B knob)
_FRESH_UPDATE = os.environ.get("VGAN_FRESH_UPDATE", "1") == "1"
# step_graphed: the whole step (stacked labels, N_CRITIC critic iterations,
# generator iteration) recorded as ONE graph when Adam and the all-reduce are
# in the graphs; "parts": one graph per piece, replayed back to back (each
# graph launch boundary left the GPU idle ~8.7 us)
_STEP_GRAPH = os.environ.get("VGAN_STEP_GRAPH", "whole")
_FRESH_KEEP = int(os.environ.get("VGAN_FRESH_KEEP", "256"))  # recorded graphs released per batch


def _loss_slots(n: int, dev) -> torch.Tensor:
    """The step's loss slots [n] as column 0 of an [n, 2] buffer: slot i and
    the float after it (column 1) are the two floats the native critic
    engine writes (d_loss, penalty), so iteration i's loss lands in its slot
    with no copy launch (one ~4.6 us blit per critic iteration)."""
    return torch.zeros(n, 2, dtype=torch.float32, device=dev)[:, 0]


def _loss_pair(acc: torch.Tensor, i: int):
    """Slot i's (d_loss, penalty) pair of ``_loss_slots``, or None."""
    base = acc._base
    if base is None or base.dim() != 2 or base.shape[1] != 2 or acc.stride(0) != 2:
        return None
    return base[i]


class _StepOut(dict):
    """step_graphed's result: "d_loss_mean" is formed when first read (an
    eager reduction launch per step otherwise, whether read or not); ``in``,
    ``get`` and ``keys()`` see it like any other key.

    The tensors ALIAS the captured graphs' persistent slots: the next
    ``step_graphed`` replay of the same batch overwrites them (clone to keep),
    and a "d_loss_mean" first read after that replay is the later step's."""

    _LAZY = ("d_loss_mean",)

    def __missing__(self, key):
        if key not in self._LAZY:
            raise KeyError(key)
        v = self[key] = self["d_losses"].mean()
        return v

    def __contains__(self, key):
        return key in self._LAZY or dict.__contains__(self, key)

    def get(self, key, default=None):
        return self[key] if key in self else default

    def keys(self):
        return list(dict.keys(self)) + [k for k in self._LAZY if not dict.__contains__(self, k)]


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
        self.phase_hook = None  # callable(name) marking host-side phase ends (profiling only)
        # critic iterations: the explicit four-pass engine (vgan/critic.py) or
        # autograd double backward through the differentiable HIP ops
        # (vg_gp_head holds a row's classes in registers: K <= 32)
        use_engine = (runtime.get("critic", "engine") == "engine" and getattr(configuration, "USE_WGANGP", True)
                      and int(configuration.NUM_CLASSES) <= 32)
        self.critic = CriticEngine(discriminator, configuration) if use_engine else None
        # generator iteration: the explicit schedule (vgan/genstep.py) or
        # autograd through the differentiable HIP ops
        gen = GeneratorEngine(generator, discriminator, configuration) \
            if runtime.get("gen", os.environ.get("VGAN_GEN", "engine")) == "engine" else None
        self.gen_engine = gen if gen is not None and gen.supported else None
        self.states = {"epoch_start": 1, "epoch_end": int(configuration.EPOCHS) + 1, "best_f1_score": 0}
        # resume (trainer.py:628-636): a states.pt in log_dir -- written by this
        # trainer or by the reference's -- restores models, optimizers, scheduler
        if os.path.exists(self._states_path()):
            self.load_states(torch.load(self._states_path(), map_location="cpu", weights_only=True))
            if self.rank == 0:
                print(f"Loaded states from {self.log_dir}")
            self.sync.broadcast_params(self.flat_g)
            self.sync.broadcast_params(self.flat_d)
        # captured step graphs are cached on the batch, per trainer (two
        # trainers -- e.g. f32 and bf16 -- may step the same batch)
        self._graph_key = f"step_graphs:{next(_TRAINER_IDS)}"
        # operand precision of the dense products: "f32" (configs[1], the
        # reference's) or "bf16" (configs[2]: bf16 operands, f32 accumulate)
        self.precision = runtime.get("precision", "f32")
        if self.precision not in ("f32", "bf16"):
            raise ValueError(f"runtime['precision'] must be 'f32' or 'bf16', not {self.precision!r}")

    def _critic_loss_backward(self, local_graph, voxel_graph, label_hard, label_soft, out=None) -> torch.Tensor:
        """d_loss of trainer.py:476-479 with D's gradients accumulated into .grad.
        ``out``: two floats the native critic engine may write (d_loss, penalty)."""
        if self.critic is not None:
            return self.critic.loss_and_grad(local_graph, voxel_graph, label_hard, label_soft, self.rng, out=out)
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

    def _iter_begin(self, adam: FlatAdam) -> None:
        """Open an iteration whose update ``adam`` makes: RNG.reset(),
        adam.zero_grad() and the step count optimizer.step() increments, as
        ONE launch (vg_iter_begin) instead of three; the iteration's update
        then runs ``adam.step(counted=True)``.  The gradient is zeroed before
        the no-grad generator forward instead of after it (trainer.py:474-475),
        which that forward never reads."""
        ctrs = self.rng.reset(defer=True)
        for t in ctrs[1:]:  # counters on other devices (not the path's single-device case)
            t.add_(1)
        flat = adam.flat
        flat.zero_grad(device=False)
        check(LIB.vg_iter_begin(ptr(ctrs[0]) if ctrs else None, ptr(adam.step_t), ptr(flat.grad),
                                flat.grad.numel(), stream_handle(flat.grad.device)), "vg_iter_begin")

    def _critic_iteration(self, local_graph, voxel_graph, labels, i: int, out=None) -> torch.Tensor:
        """trainer.py:470-479 up to backward(); the update (adam_d.step(counted=True)) is the caller's."""
        self._iter_begin(self.adam_d)
        if labels is not None:
            hard, soft = labels[0][i:i + 1], labels[1][i:i + 1]
        else:
            with torch.no_grad():
                _, hard, soft = self._generate(local_graph, voxel_graph)
        return self._critic_loss_backward(local_graph, voxel_graph, hard, soft, out=out)

    def _gen_iteration(self, local_graph, voxel_graph, early=None):
        """trainer.py:483-492 up to backward(); the update (adam_g.step(counted=True)) is the caller's."""
        self._iter_begin(self.adam_g)
        if self.gen_engine is not None and self.skip_dead_d_grads:
            return self.gen_engine.loss_and_grad(local_graph, voxel_graph, self.rng, early=early)
        # the autograd path forms every gradient in one backward: an early
        # bucket would be all-reduced before it holds anything
        assert early is None, "early all-reduce needs the explicit generator schedule (gen_engine)"
        logits, hard, _ = self._generate(local_graph, voxel_graph)
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

    def _overlap_ready(self) -> bool:
        """Overlap the generator's all-reduce with its backward: RCCL ranks
        (capturable, stream-ordered collectives), the explicit generator
        schedule, runtime['overlap_allreduce'] (default OFF).  Measured on one
        GPU with the collectives recorded (tools/dp_overlap_probe.py,
        profiles/r04_dp_overlap.jsonl): the side-stream branch in the captured
        step costs 0.86-0.88 ms per replayed step (8.55 vs 7.69 ms), against
        the ~12-20 us an 8-rank all-reduce of the 1.1 MB bucket takes over
        xGMI -- graph branches on this stack cost more than any overlap they
        buy."""
        return (self.sync.active and self.sync.capturable and self.gen_engine is not None
                and self.skip_dead_d_grads and getattr(self.configuration, "runtime", {}).get("overlap_allreduce", False))

    def _gen_iteration_synced(self, local_graph, voxel_graph):
        """The generator iteration with its flat gradient averaged over the
        ranks.  With RCCL the gradient goes in two buckets: the decoder's
        (the last parameters of the flat buffer, models.py:92-113), reduced on
        a side stream as soon as the decoder's backward has formed it, while
        the GAT encoder and MLP backward run; then the rest.  (north_star:
        "RCCL gradient all-reduce over xGMI overlapped with backward"; inside
        a captured graph the side stream is a parallel branch.)"""
        if not self._overlap_ready():
            out = self._gen_iteration(local_graph, voxel_graph)
            self.sync.all_reduce_grad(self.flat_g)
            return out
        flat = self.flat_g
        lo = self.__dict__.get("_dec_offset")
        if lo is None:
            lo = self._dec_offset = min(flat._offset(p) for p in self.generator.decoder.parameters())
        cur = torch.cuda.current_stream(flat.grad.device)
        side = self.__dict__.get("_ar_stream")
        if side is None:
            side = self._ar_stream = torch.cuda.Stream(flat.grad.device)

        def early():
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self.sync.all_reduce_tensor(flat.grad[lo:])

        out = self._gen_iteration(local_graph, voxel_graph, early=early)
        self.sync.all_reduce_tensor(flat.grad[:lo])
        cur.wait_stream(side)
        return out

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
            self.adam_d.step(counted=True)
        g_loss, hard = self._gen_iteration_synced(local_graph, voxel_graph)
        self.adam_g.step(counted=True)
        return {"d_losses": torch.stack(d_losses), "g_loss": g_loss.detach(), "label_hard": hard.detach()}

    # ------------------------------------------------- hipGraph-captured step
    def _critic_body(self, local_graph, voxel_graph, acc, with_adam: bool, labels=None, i: int = 0,
                     sync: bool = False):
        """One critic iteration; its loss goes to acc[i].  ``sync``: the flat
        D gradient is averaged over the ranks (RCCL, recorded in the graph)
        before Adam."""
        pair = _loss_pair(acc, i)
        d_loss = self._critic_iteration(local_graph, voxel_graph, labels, i, out=pair)
        if d_loss.data_ptr() != acc[i].data_ptr():  # the native engine wrote it in place
            acc[i].copy_(d_loss.detach())
        if sync:
            self.sync.all_reduce_grad(self.flat_d)
        if with_adam:
            self.adam_d.step(counted=True)

    def _gen_body(self, local_graph, voxel_graph, acc, with_adam: bool, sync: bool = False):
        """The generator iteration; its loss goes to acc[-1]."""
        if sync:
            g_loss, hard = self._gen_iteration_synced(local_graph, voxel_graph)
        else:
            g_loss, hard = self._gen_iteration(local_graph, voxel_graph)
        acc[-1].copy_(g_loss.detach())
        if with_adam:
            self.adam_g.step(counted=True)
        return hard.detach()

    def _state_tensors(self):
        """Everything a step advances in place: parameters, Adam state and the
        device RNG's iteration counters."""
        return [self.flat_g.param, self.flat_d.param, self.adam_g.exp_avg, self.adam_g.exp_avg_sq,
                self.adam_d.exp_avg, self.adam_d.exp_avg_sq, self.adam_g.step_t, self.adam_d.step_t,
                *getattr(self.rng, "_iters", {}).values()]

    def _snapshot(self):
        return [t.clone() for t in self._state_tensors()]

    def _restore(self, snap):
        """Undo a capture's warm-up: the captured step then draws exactly what
        the eager step would from the same state."""
        for d, s_ in zip(self._state_tensors(), snap):
            d.copy_(s_)

    def capture(self, local_graph, voxel_graph, whole: Optional[bool] = None):
        """``whole`` (default VGAN_STEP_GRAPH): the step as one graph where
        it can be (stacked labels, Adam in the graphs); False: one graph per
        piece (the per-iteration graphs the parity tests replay one by one)."""
        with gemm_precision_scope(self.precision):
            return self._capture(local_graph, voxel_graph, _STEP_GRAPH == "whole" if whole is None else whole)

    def _capture(self, local_graph, voxel_graph, whole: bool = False):
        """Record the step of this (static) batch as hipGraphs.

        * stacked labels (device RNG): one graph for the stacked critic-label
          G forward, one per critic iteration (each reads its own label slice)
          and one for the generator iteration;
        * otherwise: one critic-iteration graph replayed N_CRITIC times and the
          generator graph.
        RNG counters, parameters and Adam state advance in place on the device.
        With several ranks over RCCL the flat-gradient all-reduce is recorded
        in each iteration's graph between its backward and its Adam step (no
        host round trip between replays); over gloo (host collectives, the CPU
        tests) the all-reduce and Adam run eagerly between replays.  Needs
        device-side randomness (device or fixed RNG)."""
        if self.rng.mode == "host":
            raise RuntimeError("graph capture needs device-side randomness (runtime['rng'] 'device')")
        dev = voxel_graph.x.device
        n_critic = self.configuration.N_CRITIC
        sync = self.sync.active and self.sync.capturable
        with_adam = not self.sync.active or sync
        stacked = self._stacked_labels()
        acc = _loss_slots(n_critic + 1, dev)
        vdata.prepared(local_graph, voxel_graph, self.configuration.NUM_CLASSES)  # CSR etc. before capture
        self.adam_g.sync_lr()
        self.adam_d.sync_lr()
        if callable(getattr(self.rng, "_iter", None)):
            self.rng._iter(dev)  # the counter exists before the snapshot
        snap = self._snapshot()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up (lazy init) on a side stream, then undo it
            labels = self._critic_labels(local_graph, voxel_graph) if stacked else None
            self._critic_body(local_graph, voxel_graph, acc, with_adam, labels, 0, sync)
            self._gen_body(local_graph, voxel_graph, acc, with_adam, sync)
        torch.cuda.current_stream(dev).wait_stream(side)
        self._restore(snap)
        pool = getattr(self, "_graph_pool", None)
        if pool is None:
            pool = self._graph_pool = torch.cuda.graph_pool_handle()
        g_labels, labels = None, None
        if whole and stacked and with_adam:  # the whole step, one graph
            g_all = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_all, pool=pool, capture_error_mode="thread_local"):
                labels = self._critic_labels(local_graph, voxel_graph)
                for i in range(n_critic):
                    self._critic_body(local_graph, voxel_graph, acc, with_adam, labels, i, sync)
                hard = self._gen_body(local_graph, voxel_graph, acc, with_adam, sync)
            self._restore(snap)
            graphs = {"whole": g_all, "labels": None, "label_tensors": labels, "critic": [], "gen": None, "acc": acc,
                      "hard": hard, "with_adam": with_adam, "sync_in_graph": sync}
            voxel_graph.set_derived(self._graph_key, graphs)
            return graphs
        if stacked:
            g_labels = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_labels, pool=pool, capture_error_mode="thread_local"):
                labels = self._critic_labels(local_graph, voxel_graph)
        critic = []
        for i in range(n_critic if stacked else 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                self._critic_body(local_graph, voxel_graph, acc, with_adam, labels, i, sync)
            critic.append(g)
        g_gen = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_gen, pool=pool, capture_error_mode="thread_local"):
            hard = self._gen_body(local_graph, voxel_graph, acc, with_adam, sync)
        self._restore(snap)
        graphs = {"labels": g_labels, "label_tensors": labels, "critic": critic, "gen": g_gen, "acc": acc,
                  "hard": hard, "with_adam": with_adam, "sync_in_graph": sync}
        voxel_graph.set_derived(self._graph_key, graphs)
        return graphs

    def step_graphed(self, local_graph, voxel_graph) -> Dict[str, torch.Tensor]:
        """``step`` replayed from hipGraphs (captured on first use per batch).
        The returned tensors are the graphs' static outputs: valid until the
        next replay of this batch (clone to keep)."""
        graphs = voxel_graph.derived(self._graph_key) if callable(getattr(voxel_graph, "derived", None)) else None
        if graphs is None:
            graphs = self.capture(local_graph, voxel_graph)
        self.adam_g.sync_lr()
        self.adam_d.sync_lr()
        acc = graphs["acc"]
        n_critic = self.configuration.N_CRITIC
        if graphs.get("whole") is not None:
            graphs["whole"].replay()
            return _StepOut(d_losses=acc[:n_critic], g_loss=acc[n_critic], label_hard=graphs["hard"])
        if graphs["labels"] is not None:
            graphs["labels"].replay()
        critic = graphs["critic"]
        single = len(critic) == 1 and n_critic > 1  # one graph replayed: its loss slot is acc[0]
        for i in range(n_critic):
            critic[0 if single else i].replay()
            if single:  # iteration 0's loss waits in the generator's slot
                (acc[n_critic] if i == 0 else acc[i]).copy_(acc[0])
            if not graphs["with_adam"]:
                self.sync.all_reduce_grad(self.flat_d)
                self.adam_d.step(counted=True)
        if single:
            acc[0].copy_(acc[n_critic])
        graphs["gen"].replay()
        if not graphs["with_adam"]:
            self.sync.all_reduce_grad(self.flat_g)
            self.adam_g.step(counted=True)
        return _StepOut(d_losses=acc[:n_critic], g_loss=acc[n_critic], label_hard=graphs["hard"])

    # ------------------------------------------------ a batch seen once
    def step_fresh(self, local_graph, voxel_graph) -> Dict[str, torch.Tensor]:
        """``step`` for a batch the trainer sees once (every batch of
        ``Trainer.train``'s shuffled loader).  The N_CRITIC critic iterations
        of a step issue the same launches on the same batch, so the critic
        iteration is recorded ONCE per batch as a hipGraph that reads its
        labels from a static slot, and replayed N_CRITIC times (the labels of
        iteration i copied into the slot before each replay); the stacked
        critic-label forward and the generator iteration run once per step
        either way and run eagerly.  The host then pays one critic body per
        step instead of N_CRITIC -- the eager step is host-bound.  Same
        arithmetic and draws as ``step`` (device RNG: each replay advances the
        counter like an eager iteration).  Host / fixed RNG or one critic
        iteration: ``step``."""
        if self.rng.mode != "device" or not self._stacked_labels():
            return self.step(local_graph, voxel_graph)
        with gemm_precision_scope(self.precision):
            return self._step_fresh(local_graph, voxel_graph)

    def _fresh_record(self, fn):
        """(recorded graph, fn's result): fn's launches recorded -- not run --
        on the fresh path's side stream into its memory pool.
        torch.cuda.graph() would synchronise the device, collect garbage and
        empty the allocator cache on every capture: the low-level calls
        record without any of that.  Thread-local capture mode: the loader's
        thread keeps collating into pinned buffers and uploading meanwhile."""
        dev = torch.cuda.current_device()
        pool = getattr(self, "_fresh_pool", None)
        if pool is None:
            pool = self._fresh_pool = torch.cuda.graph_pool_handle()
        side = getattr(self, "_fresh_stream", None)
        if side is None:
            side = self._fresh_stream = torch.cuda.Stream(dev)
        # No stream waits around the recording: it enqueues no device work,
        # so neither side.wait_stream(cur) nor cur.wait_stream(side) would
        # order anything -- and each costs the device a drain of its queue
        # (a cross-queue barrier): 8.30-8.46 vs 7.71-7.72 ms per fresh step
        # with them (profiles/r04_record_waits_ab.txt).
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.stream(side):
            g.capture_begin(pool=pool, capture_error_mode="thread_local")
            try:
                out = fn()
            finally:
                g.capture_end()
        return g, out

    def _fresh_exec(self, kind: str, g) -> ctypes.c_void_p:
        """The executable graph that replays recording ``g`` of graph kind
        ``kind`` (step_fresh: "critic").  Two executable graphs per kind,
        used by alternate batches, are updated in place from each new
        recording (vg_graph_exec_update) -- instantiating a graph per batch
        and destroying the previous one cost ~3 ms of host time per step.  An
        update rewrites an executable graph's kernel arguments, and HIP does
        not promise that launches of it already queued keep the old ones, so
        an executable graph is updated only after its last launches -- two
        batches back -- have finished (a host wait on the event recorded
        behind them by _fresh_done; the device is normally less than one
        batch behind the host, so the wait rarely stalls)."""
        st = self.__dict__.setdefault("_fresh_state", {})
        k = st.setdefault(kind, {"owners": [None, None], "events": [None, None], "parity": 1})
        j = k["parity"] = (k["parity"] + 1) % 2
        owner = k["owners"][j]
        if k["events"][j] is not None:
            k["events"][j].synchronize()
        if owner is None or not _FRESH_UPDATE or \
                LIB.vg_graph_exec_update(ctypes.c_void_p(owner.raw_cuda_graph_exec()),
                                         ctypes.c_void_p(g.raw_cuda_graph())) != 0:
            g.instantiate()  # first batches, or a launch sequence of another shape
            if owner is not None:
                self.__dict__.setdefault("_fresh_dead", []).append(owner)
            owner = k["owners"][j] = g
        elif g is not owner:
            self.__dict__.setdefault("_fresh_dead", []).append(g)
        return ctypes.c_void_p(owner.raw_cuda_graph_exec())

    def _fresh_done(self, kind: str, stream) -> None:
        """Record the event behind the last launch of ``kind``'s current
        executable graph (see _fresh_exec)."""
        k = self._fresh_state[kind]
        ev = k["events"][k["parity"]] = torch.cuda.Event()
        ev.record(stream)

    def _step_fresh(self, local_graph, voxel_graph) -> Dict[str, torch.Tensor]:
        cfg = self.configuration
        dev = voxel_graph.x.device
        n_critic = cfg.N_CRITIC
        sync = self.sync.active and self.sync.capturable
        with_adam = not self.sync.active or sync
        mark = self.phase_hook or (lambda name: None)  # host-time probes (tools/host_profile.py)
        prep = vdata.prepared(local_graph, voxel_graph, cfg.NUM_CLASSES)
        # the critic's per-batch structures (stacked real / fake / mix graph,
        # its padded columns, the adjoint seeds) before the capture: built
        # inside it, their ~25 small launches would be recorded and replayed by
        # every critic iteration
        if self.critic is not None:
            self.critic.prepare_batch(prep)
        self.adam_g.sync_lr()
        self.adam_d.sync_lr()
        acc = _loss_slots(n_critic + 1, dev)
        cur = torch.cuda.current_stream(dev)
        st = stream_handle(dev)
        warm = getattr(self, "_fresh_warm", False)
        mark("prepare")
        # the label forward and the generator iteration run eagerly: each runs
        # once per batch, so recording them costs the host what launching
        # them does -- measured no faster recorded
        hard_all, soft_all = self._critic_labels(local_graph, voxel_graph)
        mark("labels")
        slot = (torch.empty_like(hard_all[0:1]), torch.empty_like(soft_all[0:1]))
        if not warm:
            # first capture of this trainer: run the body once outside any
            # capture (lazy initialisation, constant buffers), then undo it
            self.rng._iter(dev)
            snap = self._snapshot()
            slot[0].copy_(hard_all[0:1])
            slot[1].copy_(soft_all[0:1])
            self._critic_body(local_graph, voxel_graph, acc, with_adam, slot, 0, sync)
            self._restore(snap)
            self._fresh_warm = True
        g_crit, _ = self._fresh_record(
            lambda: self._critic_body(local_graph, voxel_graph, acc, with_adam, slot, 0, sync))
        exec_ = self._fresh_exec("critic", g_crit)
        mark("capture")
        d_losses = torch.empty(n_critic, dtype=torch.float32, device=dev)
        for i in range(n_critic):
            slot[0].copy_(hard_all[i:i + 1])
            slot[1].copy_(soft_all[i:i + 1])
            check(LIB.vg_graph_launch(exec_, st), "vg_graph_launch")
            d_losses[i:i + 1].copy_(acc[0:1])
            if not with_adam:
                self.sync.all_reduce_grad(self.flat_d)
                self.adam_d.step(counted=True)
        self._fresh_done("critic", cur)
        mark("replays")
        g_loss, hard = self._gen_iteration_synced(local_graph, voxel_graph)
        self.adam_g.step(counted=True)
        mark("gen")
        # Recorded graphs are released in batches: destroying one while the
        # device is busy blocks the runtime (every thread's launches) for ~8 ms
        # (tools/graph_destroy_probe.py; ~0.3 ms on an idle device), so they
        # are kept until _FRESH_KEEP have gathered and destroyed after one
        # device synchronisation
        dead = self.__dict__.setdefault("_fresh_dead", [])
        if len(dead) >= _FRESH_KEEP:
            torch.cuda.synchronize(dev)
            dead.clear()
        mark("release")
        return {"d_losses": d_losses, "g_loss": g_loss.detach(), "label_hard": hard.detach()}

    # ------------------------------------------------------ orchestration
    # The epoch loop of trainer.py:445-520 (train), :522-577 (validation),
    # :641-747 (epochs, checkpoint) and :749-806 (test).  Per batch only device
    # work is enqueued -- the step, the confusion counts, the losses -- and the
    # figures are read back once per epoch, so the host keeps queueing ahead of
    # the GPU.  With several ranks every epoch figure is reduced over the ranks
    # (sums and minima), so all ranks report, and decide on, the same numbers.

    def _train_mode(self) -> str:
        """runtime['train_step']: "eager" (``step``), "fresh" (``step_fresh``:
        the critic iteration captured once per batch, replayed N_CRITIC times),
        "graphed" (``step_graphed``: the whole step captured per batch) or
        "auto" (default: ``step_fresh`` on a batch seen for the first time,
        ``step_graphed`` when a batch object comes back -- a resident dataset
        -- captured on its second visit and replayed from then on)."""
        mode = getattr(self.configuration, "runtime", {}).get("train_step", "auto")
        if mode not in ("eager", "fresh", "graphed", "auto"):
            raise ValueError(f"runtime['train_step'] must be 'eager', 'fresh', 'graphed' or 'auto', not {mode!r}")
        return "eager" if self.rng.mode == "host" else mode  # host draws cannot be replayed

    def _train_batch(self, local_graph, voxel_graph) -> Dict[str, torch.Tensor]:
        """One step on a batch, by ``_train_mode``; the returned losses are
        this step's own (clones of a replay's static outputs)."""
        mode = self._train_mode()
        getter = getattr(voxel_graph, "derived", None)
        if mode == "auto":
            mode = "fresh"
            if callable(getter) and voxel_graph.x.is_cuda:
                seen_key = self._graph_key + ":seen"
                if getter(self._graph_key) is not None or getter(seen_key):
                    mode = "graphed"
                else:
                    voxel_graph.set_derived(seen_key, True)
        if mode == "graphed" and callable(getter):
            out = self.step_graphed(local_graph, voxel_graph)
            return {"d_losses": out["d_losses"].clone(), "g_loss": out["g_loss"].clone(),
                    "label_hard": out["label_hard"]}
        if mode == "fresh":
            return self.step_fresh(local_graph, voxel_graph)
        return self.step(local_graph, voxel_graph)

    def _to_device(self, local_graph, voxel_graph):
        local_graph = local_graph.to(self.configuration.DEVICE)
        voxel_graph = voxel_graph.to(self.configuration.DEVICE)
        assert [set(d) for d in local_graph.data_number] == [set(d) for d in voxel_graph.data_number]
        return local_graph, voxel_graph

    @staticmethod
    def _read_confusions(confs):
        """One device-to-host copy for an epoch's confusion counts: per batch
        (per-building [G, K, K], whole batch [K, K]) -> the metric tuples of
        trainer.py:443."""
        if not confs:
            return []
        sizes = [c.shape[0] for c, _ in confs]
        per_graph = torch.cat([c for c, _ in confs]).cpu().numpy()
        whole = torch.stack([a for _, a in confs]).cpu().numpy()
        out, lo = [], 0
        for b, g in enumerate(sizes):
            out.append(vmetrics.batch_metrics(per_graph[lo:lo + g], whole[b]))
            lo += g
        return out

    def _epoch_figures(self, metrics, losses):
        """Means over the epoch's batches (losses over every recorded value) and
        the minimum per-building F1.  One rank: the reference's own reductions
        (``torch.tensor(list).mean().item()`` -- float32 -- and ``min``).
        Several ranks: float64 sums and counts reduced over the ranks, and the
        minimum reduced with MIN, so every rank gets the global figures."""
        f1s = [m[0] for m in metrics]
        per_graph = [v for m in metrics for v in m[1]]
        cols = [f1s, [m[2] for m in metrics], [m[3] for m in metrics], [m[4] for m in metrics]]
        if not self.sync.active:
            mean = lambda v: torch.tensor(v).mean().item() if len(v) else 0.0  # noqa: E731
            loss_means = [torch.cat([t.reshape(-1) for t in l]).mean().item() if l else 0.0 for l in losses]
            return loss_means, [mean(c) for c in cols], (min(per_graph) if per_graph else 0.0)
        flat_losses = [torch.cat([t.reshape(-1) for t in l]).double().cpu() if l else torch.zeros(0, dtype=torch.float64)
                       for l in losses]
        sums = self.sync.reduce_host([float(v.sum()) for v in flat_losses] + [float(v.numel()) for v in flat_losses]
                                     + [float(sum(c)) for c in cols] + [float(len(f1s))])
        nl = len(losses)
        loss_means = [s / c if c else 0.0 for s, c in zip(sums[:nl], sums[nl:2 * nl])]
        nb = sums[-1]
        means = [s / nb if nb else 0.0 for s in sums[2 * nl:2 * nl + len(cols)]]
        lo = self.sync.reduce_host([min(per_graph) if per_graph else float("inf")], op="min")[0]
        return loss_means, means, (lo if lo != float("inf") else 0.0)

    def _train_each_epoch(self):
        """trainer.py:445-520 -> (g_loss, d_loss, f1, min per-building f1,
        precision, recall, accuracy)."""
        start = time.time()
        g_losses, d_losses, confs = [], [], []
        with gc_frozen():  # the batch loop's GC passes skip everything alive before it (vgan/gcscope.py)
            for local_graph, voxel_graph in self.dataloaders.train_dataloader:
                local_graph, voxel_graph = self._to_device(local_graph, voxel_graph)
                out = self._train_batch(local_graph, voxel_graph)
                d_losses.append(out["d_losses"])
                g_losses.append(out["g_loss"])
                confs.append(ops.confusion(voxel_graph.type, out["label_hard"].squeeze(0), voxel_graph.ptr))
        metrics = self._read_confusions(confs)
        (g_mean, d_mean), (f1, prec, rec, acc), f1_min = self._epoch_figures(metrics, [g_losses, d_losses])
        print(f"The function _train_each_epoch took {time.time() - start} seconds to run.")
        return g_mean, d_mean, f1, f1_min, prec, rec, acc

    # ------------------------------------------------------ evaluation
    def _eval_forward(self):
        fwd = getattr(self, "_eval_sweep", None)
        if fwd is None:
            from .infer import InferenceSweep

            fwd = self._eval_sweep = InferenceSweep(self.generator, [float(self.generator.tau)])
        return fwd

    def _eval_body(self, local_graph, voxel_graph, with_loss: bool):
        """Generator sample + (optionally) its generator loss + confusion
        counts of one evaluation batch (trainer.py:545-553 / :769-774): the
        no-grad stacked forward of the inference sweep (vgan.infer)."""
        logits, hard = self._eval_forward().generate(local_graph, voxel_graph)
        loss = self._compute_generator_loss(local_graph, voxel_graph, logits, hard.unsqueeze(0)) if with_loss \
            else torch.zeros((), device=logits.device)
        conf, conf_all = ops.confusion(voxel_graph.type, hard, voxel_graph.ptr)
        return loss, conf, conf_all, hard

    def _eval_batch(self, local_graph, voxel_graph, with_loss: bool):
        """``_eval_body``, eager on a batch's first visit; a batch object that
        comes back (a resident evaluation set: every epoch's validation) is
        captured as one hipGraph on its second visit and replayed from then
        on.  Returns (loss, conf, conf_all) owned by the caller;
        ``self.eval_record`` (a list, tests) also receives (voxel_graph, a copy
        of the sampled labels)."""
        out = self._eval_outputs(local_graph, voxel_graph, with_loss)
        if getattr(self, "eval_record", None) is not None:
            self.eval_record.append((voxel_graph, out[3].clone()))
        return out[:3]

    def _eval_outputs(self, local_graph, voxel_graph, with_loss: bool):
        getter = getattr(voxel_graph, "derived", None)
        if self.rng.mode == "host" or not callable(getter) or not voxel_graph.x.is_cuda:
            return self._eval_body(local_graph, voxel_graph, with_loss)
        key = f"{self._graph_key}:eval:{int(with_loss)}"
        cached = getter(key)
        if cached is None:
            voxel_graph.set_derived(key, "seen")
            return self._eval_body(local_graph, voxel_graph, with_loss)
        if cached == "seen":
            dev = voxel_graph.x.device
            pool = getattr(self, "_eval_pool", None)
            if pool is None:
                pool = self._eval_pool = torch.cuda.graph_pool_handle()
            # the warm-up draws like a visit (its RNG reset advances the device
            # counter): undo that, so the draw stream does not depend on which
            # epoch captured the batch (a resumed run captures at another one)
            if callable(getattr(self.rng, "_iter", None)):
                self.rng._iter(dev)
            iters = {d: t.clone() for d, t in getattr(self.rng, "_iters", {}).items()}
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):  # lazy allocations outside the capture
                self._eval_body(local_graph, voxel_graph, with_loss)
            torch.cuda.current_stream(dev).wait_stream(side)
            for d, t in iters.items():
                self.rng._iters[d].copy_(t)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                outs = self._eval_body(local_graph, voxel_graph, with_loss)
            cached = (g, outs)
            voxel_graph.set_derived(key, cached)
        cached[0].replay()
        loss, conf, conf_all, hard = cached[1]
        return loss.clone(), conf.clone(), conf_all.clone(), hard  # hard: valid until the next replay

    def _evaluate(self, loader, with_loss: bool):
        losses, confs = [], []
        self.generator.eval()
        self.discriminator.eval()
        try:
            with torch.no_grad(), gemm_precision_scope(self.precision):
                for local_graph, voxel_graph in loader:
                    local_graph, voxel_graph = self._to_device(local_graph, voxel_graph)
                    loss, conf, conf_all = self._eval_batch(local_graph, voxel_graph, with_loss)
                    losses.append(loss)
                    confs.append((conf, conf_all))
        finally:
            self.generator.train()
            self.discriminator.train()
        metrics = self._read_confusions(confs)
        return self._epoch_figures(metrics, [losses] if with_loss else [])

    def _validate_each_epoch(self):
        """trainer.py:522-577 -> (g_loss, f1, min per-building f1, precision,
        recall, accuracy).  Sanity mode returns six zeros (the reference returns
        five and then fails to unpack them, trainer.py:526,666-673)."""
        if self.sanity_checking or getattr(self.dataloaders, "validation_dataloader", None) is None:
            return 0.0, 0.0, 0.0, 0.0, 0.0, 0.0
        start = time.time()
        (g_mean,), (f1, prec, rec, acc), f1_min = self._evaluate(self.dataloaders.validation_dataloader, True)
        print(f"The function _validate_each_epoch took {time.time() - start} seconds to run.")
        return g_mean, f1, f1_min, prec, rec, acc

    def test(self, num_samples_to_viz: int = 0):
        """trainer.py:749-795: test-split metrics (the qualitative figures of
        :797-803 are out of scope)."""
        _, (f1, prec, rec, acc), f1_min = self._evaluate(self.dataloaders.test_dataloader, False)
        result = {"f1_score_test": f1, "f1_score_min_test": f1_min, "precision_score_test": prec,
                  "recall_score_test": rec, "accuracy_score_test": acc}
        if self.rank == 0:
            print("\n".join(f"{k}: {v}" for k, v in result.items()))
        return result

    # ------------------------------------------------------ epochs, checkpoint
    def _set_epoch(self, epoch: int) -> None:
        """Per-epoch shuffle of a data-parallel loader (like
        DistributedSampler.set_epoch): a resumed run continues the epochs'
        shuffles instead of repeating epoch 0's."""
        for name in ("train_dataloader", "validation_dataloader", "test_dataloader"):
            ld = getattr(self.dataloaders, name, None)
            if ld is not None and callable(getattr(ld, "set_epoch", None)):
                ld.set_epoch(epoch)

    def train(self):
        """trainer.py:641-747: per epoch train + validate, the weighted min-F1
        score, a checkpoint (states.pt, the reference's keys) on a new best and
        an epoch_start bump otherwise, then the scheduler step.  Returns the
        per-epoch figures."""
        cfg = self.configuration
        epoch_start = int(self.states["epoch_start"])
        epoch_end = int(cfg.EPOCHS) + 1
        best = float(self.states["best_f1_score"])
        history = []
        for epoch in range(epoch_start, epoch_end):
            self._set_epoch(epoch)
            tr = self._train_each_epoch()
            va = self._validate_each_epoch()
            score = tr[3] * cfg.F1_SCORE_TRAIN_WEIGHT + va[2] * cfg.F1_SCORE_VALIDATION_WEIGHT
            figures = {"epoch": epoch, "g_loss_train": tr[0], "d_loss_train": tr[1], "f1_score_train": tr[2],
                       "f1_score_min_train": tr[3], "precision_score_train": tr[4], "recall_score_train": tr[5],
                       "accuracy_score_train": tr[6], "g_loss_validation": va[0], "f1_score_validation": va[1],
                       "f1_score_min_validation": va[2], "precision_score_validation": va[3],
                       "recall_score_validation": va[4], "accuracy_score_validation": va[5],
                       "f1_score_min_weightedsum": score}
            history.append(figures)
            if self.rank == 0:
                print(f"epoch {epoch}: g_loss {tr[0]:.5f} d_loss {tr[1]:.5f} f1 {tr[2]:.4f} "
                      f"f1_val {va[1]:.4f} score {score:.4f}")
            if best < score:
                if self.rank == 0:
                    print(f"Best f1 score updated: {best} -> {score}")
                best = score
                if not self.sanity_checking:
                    self.save_checkpoint(epoch, best, figures)
            elif not self.sanity_checking:
                self._bump_epoch_start(epoch)
            if self.scheduler_generator is not None:
                self.scheduler_generator.step()
        return history

    def _states_path(self) -> str:
        return os.path.join(self.log_dir, "states.pt")

    def checkpoint_states(self, epoch: int, best: float, figures: Optional[Dict[str, float]] = None) -> Dict:
        """The states.pt dictionary of trainer.py:715-736: the reference's keys,
        the models' state_dicts and torch.optim.Adam / scheduler state_dicts
        (the flat Adam moments written back into the caller's optimizers), so
        the reference trainer resumes from it and vice versa."""
        figures = figures or {}
        self.adam_g.export_to(self.optimizer_generator)
        self.adam_d.export_to(self.optimizer_discriminator)
        opt_g = self.optimizer_generator if self.optimizer_generator is not None else self.adam_g
        opt_d = self.optimizer_discriminator if self.optimizer_discriminator is not None else self.adam_d
        states = {"epoch_start": epoch, "epoch_end": int(self.configuration.EPOCHS) + 1, "best_f1_score": best}
        for key in ("f1_score_train", "f1_score_validation", "f1_score_min_train", "f1_score_min_validation",
                    "f1_score_min_weightedsum", "recall_score_train", "recall_score_validation",
                    "accuracy_score_train", "accuracy_score_validation"):
            states[key] = figures.get(key, 0)
        states.update({
            "generator": self.generator.state_dict(),
            "discriminator": self.discriminator.state_dict(),
            "optimizer_generator": opt_g.state_dict(),
            "optimizer_discriminator": opt_d.state_dict(),
            "scheduler_generator": self.scheduler_generator.state_dict() if self.scheduler_generator is not None
            else None,
        })
        # not a reference key (its loader ignores it): the device draw stream,
        # with the rank term taken out of the seed, so a resumed run continues it
        rng = self.rng.state_dict()
        rng["seed"] -= 7919 * self.rank
        states["vgan_rng"] = rng
        return states

    def save_checkpoint(self, epoch: int, best: float, figures: Optional[Dict[str, float]] = None) -> str:
        """Write states.pt (rank 0 only; the ranks hold identical parameters)."""
        path = self._states_path()
        states = self.checkpoint_states(epoch, best, figures)
        if self.rank == 0:
            os.makedirs(self.log_dir, exist_ok=True)
            torch.save(states, path)
        self.states = states
        return path

    def _bump_epoch_start(self, epoch: int) -> None:
        """trainer.py:742-745: a non-best epoch only moves states.pt's
        epoch_start (no file yet: nothing to move, where the reference raises)."""
        path = self._states_path()
        if self.rank == 0 and os.path.exists(path):
            states = torch.load(path, map_location="cpu", weights_only=True)
            states["epoch_start"] = epoch
            torch.save(states, path)

    def load_states(self, states: Dict) -> None:
        """Resume from a states.pt dictionary (trainer.py:628-636): models,
        optimizers (into the flat Adam state) and scheduler."""
        self.generator.load_state_dict(states["generator"])
        self.discriminator.load_state_dict(states["discriminator"])
        for opt, flat, key in ((self.optimizer_generator, self.adam_g, "optimizer_generator"),
                               (self.optimizer_discriminator, self.adam_d, "optimizer_discriminator")):
            if states.get(key) is None:
                continue
            (opt if opt is not None else flat).load_state_dict(states[key])
            if opt is not None:
                flat.import_from(opt)
        if self.scheduler_generator is not None and states.get("scheduler_generator") is not None:
            self.scheduler_generator.load_state_dict(states["scheduler_generator"])
        rng = states.get("vgan_rng")
        if isinstance(rng, dict):
            self.rng.load_state_dict(dict(rng, seed=int(rng["seed"]) + 7919 * self.rank))
        self.states = dict(states)
