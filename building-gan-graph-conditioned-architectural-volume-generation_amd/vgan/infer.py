"""Generator-only inference sweep (BASELINE.json configs[4]): many buildings,
a Gumbel temperature schedule, hipGraph replay.

The reference samples layouts in ``Trainer.test`` (``trainer.py:749-806``): per
test batch one ``generator(local_graph, voxel_graph, z)`` forward in eval mode
(``models.py:119-155``; ``F.gumbel_softmax`` at tau = 1) and argmax labels.
``InferenceSweep`` runs that forward for a whole schedule of temperatures at
once: one STACKED forward per batch over ``len(taus)`` copies (z [k, N, Z], each
copy normalised on its own -- GraphNorm segments -- exactly as k separate
forwards), and the Gumbel head reads copy c's temperature from a device
vector (``vg_gumbel_fwd_dev``), so a captured hipGraph follows a new schedule
without re-capture.  Per batch the result is the predicted type of every voxel
for every temperature, [k, N] int8.

``graphed=True`` captures the stacked forward of a batch on first use and
replays it afterwards (the batch object caches its graph, as the training
step does); a one-pass sweep over batches seen once runs eagerly.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Dict, Iterable, List, Optional, Sequence

import torch

from . import data as vdata
from .gcscope import gc_frozen


# run_stream launches each batch's forward eagerly; VGAN_SWEEP_STREAM=record
# records it and updates an executable graph instead (run_fresh).  Eager
# measured faster: recording costs the host what launching does, and the
# update, the graph launch and its event come on top -- f16 147-204k vs
# 129-167k samples/s, alternated (profiles/r04_sweep_eager_ab.txt)
_STREAM = os.environ.get("VGAN_SWEEP_STREAM", "eager")
# the f16 sweep's forward of a batch as one native call (vg_hgen_sweep, csrc/
# hgen_engine.hip) instead of ~70 launches issued from Python; 0: the Python path
_NATIVE = os.environ.get("VGAN_HGEN_NATIVE", "1") == "1"


def geometric_taus(t0: float = 1.0, t1: float = 0.1, steps: int = 10) -> List[float]:
    """Annealing schedule tau_i = t0 (t1/t0)^(i/(steps-1)) (cfg #5)."""
    if steps <= 1:
        return [float(t0)]
    r = math.log(t1 / t0) / (steps - 1)
    return [float(t0 * math.exp(r * i)) for i in range(steps)]


class InferenceSweep:
    """``dtype="f16"`` runs the forward on the f16 kernels (``vgan.half``,
    configs[4]'s precision); "f32" on the training path's kernels."""

    def __init__(self, generator, taus: Sequence[float], graphed: bool = False, dtype: str = "f32"):
        if dtype not in ("f32", "f16"):
            raise ValueError(f"dtype {dtype!r}: f32 or f16")
        self.G = generator
        self.taus = [float(t) for t in taus]
        self.graphed = graphed
        self.dtype = dtype
        self.half = None
        if dtype == "f16":
            from .half import HalfGenerator

            self.half = HalfGenerator(generator)
        dev = next(generator.parameters()).device
        self.tau_t = torch.tensor(self.taus, dtype=torch.float32, device=dev)
        # one memory pool for every batch's graph: replays are sequential and
        # only each graph's output stays referenced, so intermediates are shared
        self._pool = torch.cuda.graph_pool_handle() if graphed else None

    def set_taus(self, taus: Sequence[float]) -> None:
        """New schedule of the same length: captured graphs keep working."""
        if len(taus) != len(self.taus):
            raise ValueError("a captured sweep keeps its number of temperatures")
        self.taus = [float(t) for t in taus]
        self.tau_t.copy_(torch.tensor(self.taus, dtype=torch.float32))

    @contextlib.contextmanager
    def _eval(self):
        """The generator in eval mode for the body, its mode restored after.
        Module.train() / eval() walk the whole module tree (~0.45 ms of host
        time each for the generator): a generator already in eval mode -- the
        sweeps below set it once for the whole loop -- is left alone."""
        was = self.G.training
        if was:
            self.G.eval()
        try:
            yield
        finally:
            if was:
                self.G.train()

    def _forward(self, local_graph, voxel_graph) -> torch.Tensor:
        G = self.G
        k = len(self.taus)
        if self.half is not None and _NATIVE and getattr(G.rng, "mode", None) == "device":
            # the whole batch in one native call (vg_hgen_sweep): bit-identical labels
            return self.half.sweep_labels(local_graph, voxel_graph, k, self.tau_t)
        n = voxel_graph.num_nodes
        G.rng.reset()  # advance the device counter: every (replayed) batch draws fresh z and noise
        z = G.rng.normal((k, n, G.configuration.Z_DIM), voxel_graph.x.device)
        if self.half is not None:
            _, hard, _ = self.half(local_graph, voxel_graph, z, tau=self.tau_t)
            return hard.reshape(k, n, -1).argmax(-1).to(torch.int8)
        saved = G.tau
        G.tau = self.tau_t
        try:
            _, hard, _ = G(local_graph, voxel_graph, z)
        finally:
            G.tau = saved
        return hard.reshape(k, n, -1).argmax(-1).to(torch.int8)

    @torch.no_grad()
    def generate(self, local_graph, voxel_graph):
        """(logits [N, K], label_hard [N, K]) of one sample per voxel at the
        schedule's single temperature: the evaluation forward of
        ``Trainer._validate_each_epoch`` / ``test`` (``trainer.py:545-548,
        769-772``), on the sweep's no-grad path (multi-source first layers, no
        concatenation).  Eval mode is the caller's."""
        if len(self.taus) != 1 or self.half is not None:
            raise ValueError("generate() is the one-temperature f32 forward")
        G = self.G
        G.rng.reset()
        z = G.rng.normal((1, voxel_graph.num_nodes, G.configuration.Z_DIM), voxel_graph.x.device)
        saved = G.tau
        G.tau = self.taus[0]
        try:
            logits, hard, _ = G(local_graph, voxel_graph, z, stacked=True)
        finally:
            G.tau = saved
        return logits.reshape(-1, logits.shape[-1]), hard.reshape(-1, hard.shape[-1])

    @torch.no_grad()
    def run_batch(self, local_graph, voxel_graph) -> torch.Tensor:
        """[len(taus), N] int8 predicted voxel types (device tensor)."""
        with self._eval():
            vdata.prepared(local_graph, voxel_graph, self.G.configuration.NUM_CLASSES)
            if not self.graphed:
                return self._forward(local_graph, voxel_graph)
            cached = voxel_graph.derived("sweep_graph")
            if cached is None or cached[0] is not self:
                dev = voxel_graph.x.device
                side = torch.cuda.Stream(dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):  # warm-up (lazy allocations) outside the capture
                    self._forward(local_graph, voxel_graph)
                torch.cuda.current_stream(dev).wait_stream(side)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self._pool, capture_error_mode="thread_local"):
                    out = self._forward(local_graph, voxel_graph)
                cached = (self, g, out)
                voxel_graph.set_derived("sweep_graph", cached)
            cached[1].replay()
            return cached[2]

    @torch.no_grad()
    def run_fresh(self, local_graph, voxel_graph) -> torch.Tensor:
        """``run_batch`` for a batch seen once (a stream of distinct
        buildings): the stacked forward is RECORDED as a hipGraph and two
        executable graphs, used by alternate batches, are updated in place
        with its kernel parameters (vg_graph_exec_update) -- no instantiation
        per batch; a recording of another launch shape (the f16 kernels pick
        their shapes from the sizes) instantiates a new one.  An executable
        graph is updated only after its previous launch finished (the event
        recorded behind it, two batches back).  Returns [len(taus), N] int8,
        valid until the next call (clone to keep)."""
        import ctypes

        from ._lib import LIB, check, stream_handle

        with self._eval():
            prep = vdata.prepared(local_graph, voxel_graph, self.G.configuration.NUM_CLASSES)
            k = len(self.taus)
            if k > 1:  # the stacked graph (and its padded columns) before the recording
                prep.csr.stacked(k).ell()
            dev = voxel_graph.x.device
            cur = torch.cuda.current_stream(dev)
            st = self.__dict__.setdefault("_stream_state", {"owners": [None, None], "events": [None, None],
                                                            "parity": 1, "dead": [], "side": None,
                                                            "out": None, "warm": False})
            if self._pool is None:
                self._pool = torch.cuda.graph_pool_handle()
            if st["side"] is None:
                st["side"] = torch.cuda.Stream(dev)
                st["out"] = torch.empty(0, dtype=torch.int8, device=dev)
            side = st["side"]
            if not st["warm"]:  # lazy initialisation outside any recording; its draws undone
                ctr = self.G.rng._iter(dev) if callable(getattr(self.G.rng, "_iter", None)) else None
                keep = ctr.clone() if ctr is not None else None
                self._forward(local_graph, voxel_graph)
                if ctr is not None:
                    ctr.copy_(keep)
                st["warm"] = True
            # recorded on the side stream with no stream waits around it: a
            # recording enqueues no device work, and each cross-stream wait
            # costs the device a queue drain
            g = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.stream(side):
                g.capture_begin(pool=self._pool, capture_error_mode="thread_local")
                try:
                    out = self._forward(local_graph, voxel_graph)
                finally:
                    g.capture_end()
            j = st["parity"] = (st["parity"] + 1) % 2
            owner = st["owners"][j]
            if st["events"][j] is not None:
                st["events"][j].synchronize()
            if owner is None or LIB.vg_graph_exec_update(ctypes.c_void_p(owner.raw_cuda_graph_exec()),
                                                         ctypes.c_void_p(g.raw_cuda_graph())) != 0:
                g.instantiate()
                if owner is not None:
                    st["dead"].append(owner)
                owner = st["owners"][j] = g
            check(LIB.vg_graph_launch(ctypes.c_void_p(owner.raw_cuda_graph_exec()), stream_handle(dev)),
                  "vg_graph_launch")
            if st["out"].shape != out.shape:
                st["out"] = torch.empty_like(out)
            res = st["out"]
            res.copy_(out)  # out lives in the recording's pool, reused by the next batch
            ev = st["events"][j] = torch.cuda.Event()
            ev.record(cur)
            if g is not owner:
                st["dead"].append(g)
            if len(st["dead"]) >= 64:  # graphs released in batches, on an idle device
                torch.cuda.synchronize(dev)
                st["dead"].clear()
            return res

    def run_stream(self, batches: Iterable, collect: bool = False) -> Dict[str, object]:
        """Sweep a stream of batches each seen once (each batch's forward
        launched eagerly, or recorded with ``run_fresh`` under
        VGAN_SWEEP_STREAM=record): counts and, with ``collect``, every
        batch's [k, N] predictions."""
        outs: List[torch.Tensor] = []
        graphs = samples = nb = 0
        eager = _STREAM == "eager" and not self.graphed
        with self._eval(), gc_frozen():  # vgan/gcscope.py
            for local_graph, voxel_graph in batches:
                pred = self.run_batch(local_graph, voxel_graph) if eager else self.run_fresh(local_graph, voxel_graph)
                graphs += voxel_graph.num_graphs
                samples += voxel_graph.num_graphs * len(self.taus)
                nb += 1
                if collect:
                    outs.append(pred.clone())
        res: Dict[str, object] = {"graphs": graphs, "samples": samples, "batches": nb}
        if collect:
            res["predictions"] = [o.cpu() for o in outs]
        return res

    def run(self, batches: Iterable, collect: bool = False) -> Dict[str, object]:
        """Sweep every (local_graph, voxel_graph) batch; returns counts and,
        with ``collect``, the per-batch [k, N] predictions (copied to the host
        once at the end)."""
        outs: List[torch.Tensor] = []
        graphs = samples = 0
        with self._eval(), gc_frozen():  # vgan/gcscope.py
            for local_graph, voxel_graph in batches:
                pred = self.run_batch(local_graph, voxel_graph)
                graphs += voxel_graph.num_graphs
                samples += voxel_graph.num_graphs * len(self.taus)
                if collect:
                    outs.append(pred.clone() if self.graphed else pred)
        res: Dict[str, object] = {"graphs": graphs, "samples": samples}
        if collect:
            res["predictions"] = [o.cpu() for o in outs]
        return res


def sweep(generator, batches, taus: Optional[Sequence[float]] = None, graphed: bool = False,
          collect: bool = False, dtype: str = "f32") -> Dict[str, object]:
    return InferenceSweep(generator, taus or geometric_taus(), graphed, dtype).run(batches, collect)
