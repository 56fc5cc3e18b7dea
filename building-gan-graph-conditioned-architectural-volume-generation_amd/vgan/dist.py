"""Data parallelism: one process per GPU, RCCL all-reduce of flat gradients.

The reference is single-GPU (``train.py:5``).  Here every rank trains on its
own mini-batch of 32 buildings (GraphNorm with batch=None and the type-matched
mean are batch-global, so per-rank semantics stay exactly the reference's at
batch 32) and the gradients are averaged once per backward:

* 5 x D gradient (15,665 floats, 63 KB) per step -- the critic updates;
* 1 x G gradient (274,185 floats, 1.10 MB) per step.

Both are single flat buffers (``vgan.flat``).  Over xGMI (point-to-point
links, ~153 GB/s each) a ring all-reduce of 1.1 MB at 8 ranks is ~12 us,
latency-dominated: D's gradient is one bucket per critic iteration (its
parameter gradients are all formed by the backward's final fold batch), G's
two -- the decoder's, reduced on a side stream while the encoders' backward
runs, then the rest (Trainer._gen_iteration_synced).  RCCL averages in the
collective (ReduceOp.AVG): no scale launch.  ``torch.distributed`` backend "nccl" is RCCL on ROCm; "gloo" is used
for the CPU multi-process tests.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist


def env_world() -> tuple:
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def init(backend: Optional[str] = None, configuration=None) -> tuple:
    """Initialise the default process group from torchrun env vars (no-op at 1
    rank) and record the layout in ``configuration.runtime`` (``rank``,
    ``world_size``), which the Trainer's per-rank RNG seed reads."""
    rank, world, local = env_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    if configuration is not None:
        runtime = getattr(configuration, "runtime", None)
        if runtime is None:
            runtime = configuration.runtime = {}
        runtime["rank"], runtime["world_size"] = rank, world
    return rank, world, local


class GradSync:
    """Averages a flat gradient across ranks; broadcasts initial parameters.

    ``force=True`` makes a one-rank group active (the collectives become
    identities): the tests use it to capture RCCL calls in the step graphs on a
    one-GPU box."""

    def __init__(self, group=None, force: bool = False):
        self.group = group
        up = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if up else 1
        self.force = bool(force) and up
        self.backend = dist.get_backend(group) if up else None

    @property
    def active(self) -> bool:
        return self.world > 1 or self.force

    @property
    def capturable(self) -> bool:
        """The collectives can be recorded inside a hipGraph: RCCL ("nccl") is
        stream-ordered device work; gloo runs on the host."""
        return self.backend == "nccl"

    def broadcast_params(self, flat) -> None:
        if self.active:
            dist.broadcast(flat.param, src=0, group=self.group)

    @property
    def avg_op(self) -> bool:
        """RCCL averages in the collective itself (ncclAvg): no separate scale
        launch after every all-reduce -- six fewer dependent launches per step
        (and per captured graph).  gloo has no AVG: sum, then scale."""
        return self.backend == "nccl" and hasattr(dist.ReduceOp, "AVG")

    def all_reduce_grad(self, flat) -> None:
        if self.active:
            if self.avg_op:
                dist.all_reduce(flat.grad, op=dist.ReduceOp.AVG, group=self.group)
            else:
                dist.all_reduce(flat.grad, op=dist.ReduceOp.SUM, group=self.group)
                flat.grad.mul_(1.0 / self.world)

    def all_reduce_tensor(self, t: torch.Tensor) -> None:
        """Average a (contiguous) gradient bucket in place over the ranks."""
        if self.active:
            if self.avg_op:
                dist.all_reduce(t, op=dist.ReduceOp.AVG, group=self.group)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
                t.mul_(1.0 / self.world)

    def all_reduce_scalars(self, t: torch.Tensor) -> torch.Tensor:
        if self.active:
            t = t.clone()
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            t.mul_(1.0 / self.world)
        return t

    def reduce_host(self, values, op: str = "sum"):
        """All-reduce a list of Python floats (epoch metric sums, minima) over
        the ranks: one small collective, on the device for RCCL."""
        if not self.active:
            return [float(v) for v in values]
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MIN, group=self.group)
        return [float(v) for v in t.cpu().tolist()]
