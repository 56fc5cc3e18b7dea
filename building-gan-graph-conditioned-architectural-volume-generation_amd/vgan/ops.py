"""Differentiable operators over the HIP C ABI.

Fast path
    ``gat_conv``             one fused kernel forward (attention projections,
                             logits, segment softmax, weighted gather-sum, bias),
                             three kernels for the first-order backward (no atomics).
    ``graphnorm_relu_dropout`` stats + apply forward, partial/final/apply backward.
    ``gumbel_head``          row kernel forward/backward.

Twice-differentiable path (WGAN-GP, ``trainer.py:306-312`` with
``create_graph=True``).  When autograd asks for a graph of the backward
(``torch.is_grad_enabled()`` inside ``backward``), the GAT and GraphNorm
backward re-express the forward through the closed primitive set

    spmm <-> spmm_t, sddmm, gather(src|dst) <-> scatter_src / seg_sum

whose adjoints are each other (all HIP kernels), so any order of derivative is
available and every derivative runs through the same C ABI.
"""
from __future__ import annotations

import os
import weakref
from typing import Optional, Tuple

import torch
from torch.autograd import Function

from . import _lib
from ._lib import LIB, FoldCollector, dense, check, ptr, require_cuda, stream_handle, sync_counter

NEG_SLOPE = 0.2
SOFTMAX_EPS = 1e-16
# VGAN_ELL=0: the aggregation reads its sources through row_ptr -> col only
# (A/B knob for the padded column array, CSR.ell)
_ELL = os.environ.get("VGAN_ELL", "1") == "1"
ELL_WIDTHS = (8, 16, 32)
# Large graphs aggregate on the wave-specialised LDS ring (vg_gat_aggregate_fwd_ring
# and its _gnp form) when the graph has at least
# VGAN_RING_MIN_ROWS rows and its tile plan stages at least VGAN_RING_MIN_STAGED
# of the 64-row tiles (voxels numbered in lattice blocks, vgan.locality.blocked;
# the reference's row-major numbering stages almost none and keeps the register
# gather).  VGAN_RING=0: never.
_RING = os.environ.get("VGAN_RING", "1") == "1"
RING_MIN_ROWS = int(os.environ.get("VGAN_RING_MIN_ROWS", "131072"))
RING_MIN_STAGED = float(os.environ.get("VGAN_RING_MIN_STAGED", "0.9"))
RING_TILE_ROWS = int(LIB.vg_gat_ring_tile_rows())
# Ring layers form no GraphNorm partials by default: the GraphNorm reads its
# input for the statistics (one pass over the output, ~40 us at 400k x 128),
# which measured faster than the ring's _gnp form -- the configs[3] G forward
# 7.45 vs 7.56 ms (register gather 8.00).  VGAN_RING_GNP=1:
# vg_gat_aggregate_fwd_ring_gnp (the loaders form the partials).
_RING_GNP = os.environ.get("VGAN_RING_GNP", "0") == "1"


# --------------------------------------------------------------------- CSR
class CSR:
    """Destination CSR with self loops + its source CSC, built on the device once
    per mini-batch (replaces remove_self_loops/add_self_loops in every layer)."""

    def __init__(self, edge_index: torch.Tensor, num_nodes: int):
        if not edge_index.is_cuda:
            raise RuntimeError("vgan HIP ops require tensors on a ROCm device (no CPU fallback)")
        if edge_index.dtype != torch.long or edge_index.dim() != 2 or edge_index.shape[0] != 2:
            raise ValueError("edge_index must be int64 [2, E]")
        dev = edge_index.device
        n = int(num_nodes)
        e = int(edge_index.shape[1])
        ei = edge_index.contiguous()
        i32 = dict(dtype=torch.int32, device=dev)
        row_ptr = torch.empty(n + 1, **i32)
        col = torch.empty(e + n, **i32)
        csc_ptr = torch.empty(n + 1, **i32)
        csc_slot = torch.empty(e + n, **i32)
        csc_dst = torch.empty(e + n, **i32)
        ws = torch.empty(int(LIB.vg_csr_ws_ints(e, n)), **i32)
        status = torch.zeros(2, **i32)
        check(LIB.vg_csr_build(ptr(ei), e, n, ptr(row_ptr), ptr(col), ptr(csc_ptr), ptr(csc_slot),
                               ptr(csc_dst), ptr(ws), ptr(status), stream_handle(dev)), "vg_csr_build")
        st = status.cpu()  # one host sync per mini-batch (sizes the edge arrays)
        if int(st[1]) != 0:
            raise ValueError("edge_index contains node ids outside [0, num_nodes)")
        ep = int(st[0])
        self.num_nodes, self.num_edges = n, ep
        self.row_ptr, self.col = row_ptr, col[:ep]
        self.csc_ptr, self.csc_slot, self.csc_dst = csc_ptr, csc_slot[:ep], csc_dst[:ep]
        self.device = dev

    @classmethod
    def from_arrays(cls, row_ptr: torch.Tensor, col: torch.Tensor, csc_ptr: torch.Tensor, csc_slot: torch.Tensor,
                    csc_dst: torch.Tensor, max_degree: Optional[int] = None) -> "CSR":
        """The same structure from arrays built elsewhere -- the host collate of
        ``vgan.store`` emits them in csr.hip's order -- with no device build and
        no host sync.  ``max_degree`` (the largest row length, known to the
        host collate) sizes the padded column array (``ell``) without reading
        row_ptr back."""
        for t in (row_ptr, col, csc_ptr, csc_slot, csc_dst):
            if not t.is_cuda or t.dtype != torch.int32 or t.dim() != 1:
                raise ValueError("CSR arrays must be int32 vectors on a ROCm device")
        n, ep = row_ptr.numel() - 1, col.numel()
        if csc_ptr.numel() != n + 1 or csc_slot.numel() != ep or csc_dst.numel() != ep or n <= 0:
            raise ValueError("inconsistent CSR / CSC array sizes")
        self = cls.__new__(cls)
        self.num_nodes, self.num_edges = n, ep
        self.row_ptr, self.col = row_ptr, col
        self.csc_ptr, self.csc_slot, self.csc_dst = csc_ptr, csc_slot, csc_dst
        self.device = row_ptr.device
        if max_degree is not None:
            self._ell_w = next((x for x in ELL_WIDTHS if int(max_degree) <= x), 0)
        return self

    def stream(self):
        return stream_handle(self.device)

    def stacked(self, copies: int) -> "CSR":
        """Block-diagonal CSR/CSC of ``copies`` copies of this graph (node ids and
        edge slots offset per copy): several forwards over the same batch run
        as one (the critic engine's real / fake / mix discriminator passes).
        Cached; built with a few device ops, no host sync."""
        if copies == 1:
            return self
        cache = self.__dict__.setdefault("_stacked", {})
        if copies in cache:
            return cache[copies]
        n, e = self.num_nodes, self.num_edges
        k = torch.arange(copies, device=self.device, dtype=torch.int32)

        def tile(a, step):
            return (a.unsqueeze(0) + (k * step).unsqueeze(1)).reshape(-1).contiguous()

        out = CSR.__new__(CSR)
        out.num_nodes, out.num_edges, out.device = n * copies, e * copies, self.device
        tail = torch.full((1,), e * copies, dtype=torch.int32, device=self.device)
        out.row_ptr = torch.cat([tile(self.row_ptr[:-1], e), tail])
        out.csc_ptr = torch.cat([tile(self.csc_ptr[:-1], e), tail])
        out.col = tile(self.col, n)
        out.csc_slot = tile(self.csc_slot, e)
        out.csc_dst = tile(self.csc_dst, n)
        if "_ell_w" in self.__dict__:  # same degrees: no host sync for the copies' width
            out._ell_w = self._ell_w
        out._seg_rows = n
        cache[copies] = out
        return out

    @property
    def seg_rows(self) -> int:
        """Rows per stacked copy (``stacked``): the GraphNorm segment a
        forward over this graph normalises separately."""
        return self.__dict__.get("_seg_rows", self.num_nodes)

    def ell(self):
        """(ell, width): the destination rows' sources padded to a fixed width
        (vg_csr_ell: [N][width] int32, -1 past the degree; width the smallest
        of 8 / 16 / 32 that holds the largest degree), so the aggregation
        loads a row's sources without waiting for row_ptr.  (None, 0) when
        the largest degree exceeds 32 or VGAN_ELL=0.  Built once and cached;
        the width costs one host sync per graph (inherited by stacked()
        copies), taken by data.prepared before any capture."""
        cached = self.__dict__.get("_ell")
        if cached is not None:
            return cached
        if not _ELL:
            return None, 0
        w = self.__dict__.get("_ell_w")
        if w is None:
            maxdeg = int((self.row_ptr[1:] - self.row_ptr[:-1]).max().item()) if self.num_nodes else 0
            w = next((x for x in ELL_WIDTHS if maxdeg <= x), 0)
            self._ell_w = w
        if w == 0:
            self._ell = (None, 0)
            return self._ell
        t = torch.empty(self.num_nodes * w, dtype=torch.int32, device=self.device)
        check(LIB.vg_csr_ell(ptr(self.row_ptr), ptr(self.col), self.num_nodes, w, ptr(t), self.stream()),
              "vg_csr_ell")
        self._ell = (t, w)
        return self._ell

    def tile_plan(self) -> torch.Tensor:
        """The LDS tile plan of this graph (vg_gat_tile_plan: per 16-row tile
        the distinct sources and every edge's slot among them), built once and
        cached; consumed by aggregate_lds."""
        plan = self.__dict__.get("_tile_plan")
        if plan is None:
            n_ints = int(LIB.vg_gat_tile_plan_ints(self.num_nodes, self.num_edges))
            plan = torch.empty(n_ints, dtype=torch.int32, device=self.device)
            check(LIB.vg_gat_tile_plan(ptr(self.row_ptr), ptr(self.col), self.num_nodes, self.num_edges, ptr(plan),
                                       self.stream()), "vg_gat_tile_plan")
            tiles = (self.num_nodes + 15) // 16
            # the LDS image is sized to the largest tile (one host sync, once per graph)
            self._tile_umax = max(1, int(plan[:tiles].max().item()))
            self._tile_plan = plan
        return plan


    def stage_plan(self) -> torch.Tensor:
        """The staged-tile plan of this graph (vg_gat_stage_plan: per 64-row
        tile the distinct sources and every edge's LDS slot), built once and
        cached; consumed by aggregate_staged."""
        plan = self.__dict__.get("_stage_plan")
        if plan is None:
            n_ints = int(LIB.vg_gat_stage_plan_ints(self.num_nodes, self.num_edges))
            plan = torch.empty(n_ints, dtype=torch.int32, device=self.device)
            check(LIB.vg_gat_stage_plan(ptr(self.row_ptr), ptr(self.col), self.num_nodes, self.num_edges,
                                        ptr(plan), self.stream()), "vg_gat_stage_plan")
            self._stage_plan = plan
        return plan

    def stage_tiles(self) -> int:
        return (self.num_nodes + 63) // 64

    def ring_plan(self) -> torch.Tensor:
        """The ring aggregation's tile plan (vg_gat_ring_plan: per
        RING_TILE_ROWS-row tile the distinct sources -- -1 for a tile left to
        global memory -- and every edge's LDS slot), built once and cached;
        consumed by vg_gat_aggregate_fwd_ring."""
        plan = self.__dict__.get("_ring_plan")
        if plan is None:
            n_ints = int(LIB.vg_gat_ring_plan_ints(self.num_nodes, self.num_edges))
            plan = torch.empty(n_ints, dtype=torch.int32, device=self.device)
            check(LIB.vg_gat_ring_plan(ptr(self.row_ptr), ptr(self.col), self.num_nodes, self.num_edges, ptr(plan),
                                       self.stream()), "vg_gat_ring_plan")
            self._ring_plan = plan
        return plan


    def ring_staged(self) -> float:
        """Fraction of the ring plan's tiles staged through LDS (built once,
        one host sync per graph; taken by data.prepared before any capture)."""
        frac = self.__dict__.get("_ring_staged")
        if frac is None:
            tiles = -(-self.num_nodes // RING_TILE_ROWS)
            frac = float((self.ring_plan()[:tiles] > 0).sum().item()) / tiles
            self._ring_err = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._ring_staged = frac
        return frac

    def ring_on(self, c: int) -> bool:
        """True when the aggregation over this graph at ``c`` channels runs on
        the LDS ring (vg_gat_aggregate_fwd_ring[_gnp]): C = 64 / 128, at least
        RING_MIN_ROWS rows, GraphNorm segments of whole tiles, and a plan that
        stages at least RING_MIN_STAGED of the tiles.  A graph whose plan has
        not been measured yet is measured now -- outside a stream capture; a
        capture keeps the register gather for it."""
        if not _RING or c not in (64, 128) or self.num_nodes < RING_MIN_ROWS:
            return False
        if self.seg_rows != self.num_nodes and self.seg_rows % RING_TILE_ROWS:
            return False  # stacked segments must be whole tiles
        if "_ring_staged" not in self.__dict__ and torch.cuda.is_current_stream_capturing():
            return False
        return self.ring_staged() >= RING_MIN_STAGED

    def ring_check(self) -> None:
        """Raise if a ring aggregation over this graph expired a hand-over wait
        (its output is then invalid; one host sync).  GATEncoder.forward calls
        it after a forward that dispatched the ring, outside captures."""
        err = self.__dict__.get("_ring_err")
        if err is not None and int(err.item()) != 0:
            raise RuntimeError("vg_gat_aggregate_fwd_ring: a hand-over wait expired (output invalid)")


def aggregate_fwd_raw(csr: "CSR", c: int, h, a_src, a_dst, bias, slope: float, out, alpha, stream,
                      gnp=None) -> None:
    """vg_gat_aggregate_fwd over raw device pointers (ctypes), through the
    padded column array when the graph has one (vg_gat_aggregate_fwd_ell);
    bit-identical either way.  gnp (``gnp_buffer``): also the following
    GraphNorm's column partials (vg_gat_aggregate_fwd_gnp).  Large graphs
    whose plan stages most tiles (CSR.ring_on) run the LDS ring instead
    (vg_gat_aggregate_fwd_ring, bit-identical output and alpha; with gnp its
    _gnp form, whose partials cover 64-row tiles -- gnp_buffer sized them)."""
    if csr.ring_on(c):
        if (h | out | bias) & 15:
            if gnp is not None:  # the buffer holds 64-row partials: no other kernel may fill it
                raise ValueError("ring aggregation: h, out and bias must be 16-byte aligned")
        else:
            if gnp is not None:
                check(LIB.vg_gat_aggregate_fwd_ring_gnp(ptr(csr.row_ptr), ptr(csr.col), csr.num_nodes, c, h, a_src,
                                                        a_dst, bias, float(slope), out, alpha, ptr(csr.ring_plan()),
                                                        csr.seg_rows, ptr(gnp), ptr(csr._ring_err), stream),
                      "vg_gat_aggregate_fwd_ring_gnp")
            else:
                check(LIB.vg_gat_aggregate_fwd_ring(ptr(csr.row_ptr), ptr(csr.col), csr.num_nodes, c, h, a_src, a_dst,
                                                    bias, float(slope), out, alpha, ptr(csr.ring_plan()),
                                                    ptr(csr._ring_err), stream), "vg_gat_aggregate_fwd_ring")
            csr._ring_used = True
            global RING_DISPATCHES
            RING_DISPATCHES += 1
            return
    ell, w = csr.ell()
    if gnp is not None:
        check(LIB.vg_gat_aggregate_fwd_gnp(ptr(csr.row_ptr), ptr(csr.col), ptr(ell) if ell is not None else None,
                                           w if ell is not None else 0, csr.num_nodes, c, h, a_src, a_dst, bias,
                                           float(slope), out, alpha, csr.seg_rows, ptr(gnp), stream),
              "vg_gat_aggregate_fwd_gnp")
    elif ell is not None:
        check(LIB.vg_gat_aggregate_fwd_ell(ptr(csr.row_ptr), ptr(csr.col), ptr(ell), w, csr.num_nodes, c, h, a_src,
                                           a_dst, bias, float(slope), out, alpha, stream), "vg_gat_aggregate_fwd_ell")
    else:
        check(LIB.vg_gat_aggregate_fwd(ptr(csr.row_ptr), ptr(csr.col), csr.num_nodes, c, h, a_src, a_dst, bias,
                                       float(slope), out, alpha, stream), "vg_gat_aggregate_fwd")


# GraphNorm statistics from the GAT aggregation's epilogue: every GATConv is
# followed by a GraphNorm (models.py:73-75,193-195), whose column statistics
# pass (k_stats_partial) re-read the aggregation's output.  The aggregation
# writes per-workgroup Welford partials instead (vg_gat_aggregate_fwd_gnp) and
# the GraphNorm folds them (vg_graphnorm_fwd_gnp): one launch and one pass over
# the layer's output fewer per GraphNorm.  VGAN_GN_FWD_FUSE=0: off.
_GN_FWD_FUSE = os.environ.get("VGAN_GN_FWD_FUSE", "1") == "1"


# ring aggregations dispatched by aggregate_fwd_raw (tests assert the model path takes it)
RING_DISPATCHES = 0


def gnp_buffer(csr: "CSR", c: int, device):
    """(gnp, rows per partial) for an aggregation over ``csr`` at ``c``
    channels, or (None, 0) when its workgroups would span more than two
    GraphNorm segments.  On the LDS ring (CSR.ring_on): (None, 0) -- the
    GraphNorm forms its statistics -- or, with VGAN_RING_GNP=1, partials over
    its 64-row tiles (vg_gat_ring_gnp_floats)."""
    if not _GN_FWD_FUSE:
        return None, 0
    if csr.ring_on(c):
        if not _RING_GNP:
            return None, 0
        return torch.empty(int(LIB.vg_gat_ring_gnp_floats(csr.num_nodes, c)), dtype=torch.float32,
                           device=device), RING_TILE_ROWS
    g = int(LIB.vg_gat_gnp_rows(csr.num_nodes, c))
    if g <= 0 or csr.seg_rows < g or csr.num_nodes % csr.seg_rows:
        return None, 0
    return torch.empty(int(LIB.vg_gat_gnp_floats(csr.num_nodes, c)), dtype=torch.float32, device=device), g


class _GnpHint:
    """The partials of the last GAT aggregation, for the GraphNorm that
    consumes exactly its output tensor (same object, not modified since)."""
    __slots__ = ("ref", "version", "gnp", "rows", "seg_rows")

    def __init__(self, out, gnp, rows, seg_rows):
        self.ref, self.version = weakref.ref(out), out._version
        self.gnp, self.rows, self.seg_rows = gnp, rows, seg_rows


_GNP_LAST: Optional[_GnpHint] = None


def _take_gnp(x: torch.Tensor, seg_rows: int):
    """(gnp, rows) left by the aggregation that produced ``x``, or (None, 0)."""
    global _GNP_LAST
    h, _GNP_LAST = _GNP_LAST, None
    if h is None or h.ref() is not x or x._version != h.version or h.seg_rows != seg_rows:
        return None, 0
    return h.gnp, h.rows


def aggregate_lds(csr: "CSR", h: torch.Tensor, a_src: torch.Tensor, a_dst: torch.Tensor, bias: torch.Tensor,
                  slope: float = 0.2):
    """(out, alpha) of vg_gat_aggregate_fwd_lds: GATConv's edge softmax and
    gather-sum with every 16-row tile's distinct source rows staged in LDS
    (large graphs; C a multiple of 64).  Bit-identical to the register-gather
    kernel."""
    h = _f32(h)
    require_cuda(h, a_src, a_dst, bias)
    n, c = h.shape
    if n != csr.num_nodes or c % 64:
        raise ValueError("aggregate_lds: h must be [num_nodes, 64k]")
    out = torch.empty_like(h)
    alpha = torch.empty(csr.num_edges, dtype=torch.float32, device=h.device)
    check(LIB.vg_gat_aggregate_fwd_lds(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(_f32(a_src)),
                                       ptr(_f32(a_dst)), ptr(_f32(bias)), float(slope), ptr(out), ptr(alpha),
                                       ptr(csr.tile_plan()), csr._tile_umax, csr.stream()), "vg_gat_aggregate_fwd_lds")
    return out, alpha


def aggregate_staged(csr: "CSR", h: torch.Tensor, a_src: torch.Tensor, a_dst: torch.Tensor, bias: torch.Tensor,
                     slope: float = 0.2, out: Optional[torch.Tensor] = None, alpha: Optional[torch.Tensor] = None):
    """(out, alpha) of vg_gat_aggregate_fwd_staged: GATConv's edge softmax and
    gather-sum by the persistent kernel that stages each 64-row tile's
    distinct source rows in LDS (large graphs, C = 64 or 128).  Bit-identical
    to the register-gather kernel."""
    h = _f32(h)
    require_cuda(h, a_src, a_dst, bias)
    n, c = h.shape
    if n != csr.num_nodes or c not in (64, 128):
        raise ValueError("aggregate_staged: h must be [num_nodes, 64 or 128]")
    out = torch.empty_like(h) if out is None else out
    alpha = torch.empty(csr.num_edges, dtype=torch.float32, device=h.device) if alpha is None else alpha
    check(LIB.vg_gat_aggregate_fwd_staged(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(_f32(a_src)),
                                          ptr(_f32(a_dst)), ptr(_f32(bias)), float(slope), ptr(out), ptr(alpha),
                                          ptr(csr.stage_plan()), csr.stream()), "vg_gat_aggregate_fwd_staged")
    return out, alpha


def _f32(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"expected float32, got {t.dtype}")
    return t.contiguous()


# ------------------------------------------------ direct parameter gradients
_DIRECT_GRADS = False


class direct_param_grads:
    """Within this context a first-order ``backward()`` through the fused ops
    accumulates parameter gradients straight into ``param.grad`` (views into
    the flat gradient buffer) with the kernels' accumulate flag, and hands
    autograd ``None`` for them -- no per-parameter AccumulateGrad ``add_``
    launch.  Only for ``loss.backward()`` into existing ``.grad`` tensors (the
    trainer's step), not for ``torch.autograd.grad``."""

    def __enter__(self):
        global _DIRECT_GRADS
        self._prev, _DIRECT_GRADS = _DIRECT_GRADS, True
        return self

    def __exit__(self, *exc):
        global _DIRECT_GRADS
        _DIRECT_GRADS = self._prev
        return False


_FOLDS = None  # active FoldCollector of deferred_param_folds()


class deferred_param_folds:
    """Within this context the direct parameter-gradient paths (``gemm_tn_into``
    and the GATConv backward under ``direct_param_grads``) leave their partial
    folds to ONE ``vg_fold_batch`` launch enqueued when the context exits --
    the optimizer step is their only consumer."""

    def __init__(self, device=None):
        self.device = device

    def __enter__(self):
        global _FOLDS
        self._prev, _FOLDS = _FOLDS, FoldCollector()
        return self

    def __exit__(self, exc_type, *exc):
        global _FOLDS
        col, _FOLDS = _FOLDS, self._prev
        if exc_type is None and col.folds:
            dev = self.device if self.device is not None else col.keep[0].device
            col.flush(stream_handle(dev))
        return False


def _direct(*params) -> bool:
    """All params take direct accumulation (flag on, leaf, fp32 contiguous .grad)."""
    if not _DIRECT_GRADS:
        return False
    for p in params:
        if p is None:
            continue
        g = p.grad
        if not p.requires_grad or g is None or g.dtype != torch.float32 or not g.is_contiguous():
            return False
    return True


# ----------------------------------------------------- sparse primitives
def _empty_like_rows(csr: CSR, c: Optional[int], like: torch.Tensor) -> torch.Tensor:
    shape = (csr.num_nodes,) if c is None else (csr.num_nodes, c)
    return torch.empty(shape, dtype=torch.float32, device=like.device)


def _spmm_raw(csr: CSR, w: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    w, x = _f32(w), _f32(x)
    require_cuda(w, x)
    y = _empty_like_rows(csr, x.shape[1], x)
    check(LIB.vg_spmm(ptr(csr.row_ptr), ptr(csr.col), csr.num_nodes, x.shape[1], ptr(w), ptr(x), ptr(y),
                      csr.stream()), "vg_spmm")
    return y


def _spmm_t_raw(csr: CSR, w: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    w, g = _f32(w), _f32(g)
    require_cuda(w, g)
    z = _empty_like_rows(csr, g.shape[1], g)
    check(LIB.vg_spmm_t(ptr(csr.csc_ptr), ptr(csr.csc_slot), ptr(csr.csc_dst), csr.num_nodes, g.shape[1],
                        ptr(w), ptr(g), ptr(z), csr.stream()), "vg_spmm_t")
    return z


def _sddmm_raw(csr: CSR, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    a, b = _f32(a), _f32(b)
    require_cuda(a, b)
    e = torch.empty(csr.num_edges, dtype=torch.float32, device=a.device)
    check(LIB.vg_sddmm(ptr(csr.row_ptr), ptr(csr.col), csr.num_nodes, a.shape[1], ptr(a), ptr(b), ptr(e),
                       csr.stream()), "vg_sddmm")
    return e


def _gather_raw(csr: CSR, v: torch.Tensor, by_src: bool) -> torch.Tensor:
    v = _f32(v)
    require_cuda(v)
    e = torch.empty(csr.num_edges, dtype=torch.float32, device=v.device)
    check(LIB.vg_gather(ptr(csr.row_ptr), ptr(csr.col), csr.num_nodes, 1 if by_src else 0, ptr(v), ptr(e),
                        csr.stream()), "vg_gather")
    return e


def _seg_sum_raw(csr: CSR, x: torch.Tensor) -> torch.Tensor:
    x = _f32(x)
    require_cuda(x)
    s = _empty_like_rows(csr, None, x)
    check(LIB.vg_seg_sum(ptr(csr.row_ptr), csr.num_nodes, ptr(x), ptr(s), csr.stream()), "vg_seg_sum")
    return s


def _seg_max_raw(csr: CSR, x: torch.Tensor) -> torch.Tensor:
    x = _f32(x)
    require_cuda(x)
    m = _empty_like_rows(csr, None, x)
    check(LIB.vg_seg_max(ptr(csr.row_ptr), csr.num_nodes, ptr(x), ptr(m), csr.stream()), "vg_seg_max")
    return m


def _scatter_src_raw(csr: CSR, x: torch.Tensor) -> torch.Tensor:
    x = _f32(x)
    require_cuda(x)
    s = _empty_like_rows(csr, None, x)
    check(LIB.vg_scatter_src(ptr(csr.csc_ptr), ptr(csr.csc_slot), csr.num_nodes, ptr(x), ptr(s), csr.stream()),
          "vg_scatter_src")
    return s


class _SpMM(Function):
    @staticmethod
    def forward(ctx, w, x, csr):
        ctx.csr = csr
        ctx.save_for_backward(w, x)
        return _spmm_raw(csr, w, x)

    @staticmethod
    def backward(ctx, gy):
        w, x = ctx.saved_tensors
        gw = sddmm(ctx.csr, gy, x) if ctx.needs_input_grad[0] else None
        gx = spmm_t(ctx.csr, w, gy) if ctx.needs_input_grad[1] else None
        return gw, gx, None


class _SpMMT(Function):
    @staticmethod
    def forward(ctx, w, g, csr):
        ctx.csr = csr
        ctx.save_for_backward(w, g)
        return _spmm_t_raw(csr, w, g)

    @staticmethod
    def backward(ctx, gz):
        w, g = ctx.saved_tensors
        gw = sddmm(ctx.csr, g, gz) if ctx.needs_input_grad[0] else None
        gg = spmm(ctx.csr, w, gz) if ctx.needs_input_grad[1] else None
        return gw, gg, None


class _SDDMM(Function):
    @staticmethod
    def forward(ctx, a, b, csr):
        ctx.csr = csr
        ctx.save_for_backward(a, b)
        return _sddmm_raw(csr, a, b)

    @staticmethod
    def backward(ctx, ge):
        a, b = ctx.saved_tensors
        ga = spmm(ctx.csr, ge, b) if ctx.needs_input_grad[0] else None
        gb = spmm_t(ctx.csr, ge, a) if ctx.needs_input_grad[1] else None
        return ga, gb, None


class _Gather(Function):
    @staticmethod
    def forward(ctx, v, csr, by_src):
        ctx.csr, ctx.by_src = csr, by_src
        return _gather_raw(csr, v, by_src)

    @staticmethod
    def backward(ctx, ge):
        gv = scatter_src(ctx.csr, ge) if ctx.by_src else seg_sum(ctx.csr, ge)
        return gv, None, None


class _SegSum(Function):
    @staticmethod
    def forward(ctx, x, csr):
        ctx.csr = csr
        return _seg_sum_raw(csr, x)

    @staticmethod
    def backward(ctx, gs):
        return gather(ctx.csr, gs, by_src=False), None


class _ScatterSrc(Function):
    @staticmethod
    def forward(ctx, x, csr):
        ctx.csr = csr
        return _scatter_src_raw(csr, x)

    @staticmethod
    def backward(ctx, gs):
        return gather(ctx.csr, gs, by_src=True), None


def spmm(csr: CSR, w: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """Y_i = sum_{k in row i} w_k X[col_k]."""
    return _SpMM.apply(w, x, csr)


def spmm_t(csr: CSR, w: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """Z_j = sum_{k: col_k = j} w_k G[dst_k]."""
    return _SpMMT.apply(w, g, csr)


def sddmm(csr: CSR, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """e_k = <A[dst_k], B[col_k]>."""
    return _SDDMM.apply(a, b, csr)


def gather(csr: CSR, v: torch.Tensor, by_src: bool) -> torch.Tensor:
    return _Gather.apply(v, csr, by_src)


def seg_sum(csr: CSR, x: torch.Tensor) -> torch.Tensor:
    return _SegSum.apply(x, csr)


def seg_max(csr: CSR, x: torch.Tensor) -> torch.Tensor:
    """Non-differentiable (used on detached logits, like utils/_softmax.py)."""
    return _seg_max_raw(csr, x.detach())


def scatter_src(csr: CSR, x: torch.Tensor) -> torch.Tensor:
    return _ScatterSrc.apply(x, csr)


def edge_softmax_composed(csr: CSR, a_src: torch.Tensor, a_dst: torch.Tensor, slope: float) -> torch.Tensor:
    """utils/_softmax.py (index branch) over GATConv logits, from primitives."""
    pre = gather(csr, a_src, by_src=True) + gather(csr, a_dst, by_src=False)
    e = torch.nn.functional.leaky_relu(pre, slope)
    m = seg_max(csr, e)
    p = torch.exp(e - _gather_raw(csr, m, by_src=False))
    s = seg_sum(csr, p) + SOFTMAX_EPS
    return p / gather(csr, s, by_src=False)


def _gat_backward_composed(csr, h, a_src, a_dst, g_out, slope: float):
    """d(out)/d(h, a_src, a_dst) applied to g_out, from differentiable primitives:
        ga_k = <g_out[dst_k], h[src_k]>            (sddmm)
        g_h  = spmm_t(alpha, g_out)
        ge_k = alpha_k (ga_k - sum_{row} alpha ga)  (segment-softmax adjoint)
        gp_k = ge_k * lrelu'(pre_k)
        g_a_src = scatter_src(gp), g_a_dst = seg_sum(gp)."""
    alpha = edge_softmax_composed(csr, a_src, a_dst, slope)
    ga = sddmm(csr, g_out, h)
    g_h = spmm_t(csr, alpha, g_out)
    t = seg_sum(csr, alpha * ga)
    ge = alpha * (ga - gather(csr, t, by_src=False))
    pre = _gather_raw(csr, a_src.detach(), True) + _gather_raw(csr, a_dst.detach(), False)
    gp = ge * torch.where(pre > 0, torch.ones_like(pre), torch.full_like(pre, slope))
    return g_h, scatter_src(csr, gp), seg_sum(csr, gp)


def gat_aggregate_composed(csr, h, a_src, a_dst, bias, slope: float = NEG_SLOPE):
    alpha = edge_softmax_composed(csr, a_src, a_dst, slope)
    out = spmm(csr, alpha, h)
    return out + bias if bias is not None else out


# --------------------------------------------------------- fused GATConv
def gat_conv_composed(csr, h, att_src, att_dst, bias, slope: float = NEG_SLOPE):
    """GATConv after the projection, from differentiable primitives only."""
    a_src = (h * att_src.view(1, -1)).sum(1)
    a_dst = (h * att_dst.view(1, -1)).sum(1)
    return gat_aggregate_composed(csr, h, a_src, a_dst, bias, slope)


class _GATConv(Function):
    @staticmethod
    def forward(ctx, h, att_src, att_dst, bias, csr, slope, pre=None):
        h = _f32(h)
        vs, vd, b = _f32(att_src.reshape(-1)), _f32(att_dst.reshape(-1)), _f32(bias)
        require_cuda(h, vs, vd, b)
        n, c = h.shape
        if n != csr.num_nodes or vs.numel() != c or vd.numel() != c or b.numel() != c:
            raise ValueError("gat_conv: inconsistent shapes")
        dev = h.device
        out = torch.empty_like(h)
        alpha = torch.empty(csr.num_edges, dtype=torch.float32, device=dev)
        if pre is not None:  # projections from the projection GEMM's epilogue (lin_att)
            a_src, a_dst = pre
            require_cuda(a_src, a_dst)
            if a_src.numel() != n or a_dst.numel() != n:
                raise ValueError("gat_conv: inconsistent projection shapes")
            gnp, g = gnp_buffer(csr, c, dev)
            aggregate_fwd_raw(csr, c, ptr(h), ptr(a_src), ptr(a_dst), ptr(b), slope, ptr(out), ptr(alpha),
                              csr.stream(), gnp)
            if gnp is not None:
                global _GNP_LAST
                _GNP_LAST = _GnpHint(out, gnp, g, csr.seg_rows)
        else:
            a_src = torch.empty(n, dtype=torch.float32, device=dev)
            a_dst = torch.empty(n, dtype=torch.float32, device=dev)
            check(LIB.vg_gat_fwd(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(vs), ptr(vd), ptr(b),
                                 float(slope), ptr(out), ptr(alpha), ptr(a_src), ptr(a_dst), csr.stream()),
                  "vg_gat_fwd")
        ctx.csr, ctx.slope = csr, slope
        ctx.params = (att_src, att_dst, bias)
        ctx.save_for_backward(h, att_src, att_dst, bias, alpha, a_src, a_dst)
        return out

    @staticmethod
    def backward(ctx, g_out):
        h, att_src, att_dst, bias, alpha, a_src, a_dst = ctx.saved_tensors
        csr = ctx.csr
        if torch.is_grad_enabled():
            # create_graph=True: the backward formulas of vg_gat_bwd written with
            # differentiable primitives on the saved inputs, so the returned
            # gradients carry their own graph (WGAN-GP second order).
            vs, vd = att_src.reshape(1, -1), att_dst.reshape(1, -1)
            a_s = (h * vs).sum(1)
            a_d = (h * vd).sum(1)
            g_h, g_as, g_ad = _gat_backward_composed(csr, h, a_s, a_d, g_out, ctx.slope)
            g_h = g_h + g_as.unsqueeze(1) * vs + g_ad.unsqueeze(1) * vd
            g_vs = (h * g_as.unsqueeze(1)).sum(0).view_as(att_src)
            g_vd = (h * g_ad.unsqueeze(1)).sum(0).view_as(att_dst)
            return g_h, g_vs, g_vd, g_out.sum(0), None, None, None
        g_out = _f32(g_out)
        n, c = h.shape
        dev = h.device
        g_h = torch.empty_like(h)
        p_s, p_d, p_b = ctx.params
        direct = _direct(p_s, p_d, p_b)
        want_p = any(ctx.needs_input_grad[1:4])
        if direct:
            g_vs, g_vd, g_b = p_s.grad, p_d.grad, p_b.grad
        elif not want_p:  # e.g. the frozen discriminator in the generator iteration: g_h only
            g_vs = g_vd = g_b = None
        else:
            g_vs = torch.empty(c, dtype=torch.float32, device=dev)
            g_vd = torch.empty_like(g_vs)
            g_b = torch.empty_like(g_vs)
        ws = torch.empty(int(LIB.vg_gat_bwd_ws_floats(n, csr.num_edges, c)), dtype=torch.float32, device=dev)
        args = (ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot), ptr(csr.csc_dst), n,
                csr.num_edges, c, ptr(h), ptr(_f32(att_src.reshape(-1))), ptr(_f32(att_dst.reshape(-1))), ptr(a_src),
                ptr(a_dst), ptr(alpha), ptr(g_out), float(ctx.slope), ptr(g_h), ptr(g_vs), ptr(g_vd), ptr(g_b),
                1 if direct else 0, None, 0, ptr(ws))
        if direct and _FOLDS is not None:  # parameter-gradient fold deferred to the context's batch
            _FOLDS.call(LIB.vg_gat_bwd_deferred, args, csr.stream(), keep=(ws,), name="vg_gat_bwd_deferred")
        else:
            check(LIB.vg_gat_bwd_ex(*args, csr.stream()), "vg_gat_bwd_ex")
        if direct or not want_p:
            return g_h, None, None, None, None, None, None
        return g_h, g_vs.view_as(att_src), g_vd.view_as(att_dst), g_b, None, None, None


def gat_conv(csr: CSR, h, att_src, att_dst, bias, slope: float = NEG_SLOPE, pre=None) -> torch.Tensor:
    """GATConv (heads=1) after the projection h = x W^T: attention projections,
    segment softmax, aggregation and bias (``vg_gat_fwd``).  ``pre`` = (h .
    att_src, h . att_dst) already computed (``lin_att``): then only the edge
    softmax + gather-sum kernel runs (``vg_gat_aggregate_fwd``).  The
    projections' dependence on h / att is part of this op's backward, so
    ``pre`` carries no gradient."""
    return _GATConv.apply(h, att_src, att_dst, bias, csr, slope, pre)


# ------------------------------------------ GraphNorm + ReLU + Dropout
def graphnorm_relu_dropout_torch(x, weight, bias, mean_scale, keep, eps):
    """torch expression of the fused op (used only to build the create_graph
    backward; same formula as torch_geometric GraphNorm, batch=None)."""
    centred = x - x.mean(dim=0, keepdim=True) * mean_scale
    z = weight * centred / (centred.pow(2).mean(dim=0, keepdim=True) + eps).sqrt() + bias
    y = torch.relu(z)
    return y * keep if keep is not None else y


# The GraphNorm backward's column partials from the epilogue of the GEMM that
# produces its g_y (vg_gemm_gn_bwd, as the critic engine does): a GraphNorm
# forward whose output feeds a linear layer leaves a hint keyed by that output
# (address, shape); the linear backward finds it for its input and forms
# g_x = g_h W with the partials; the GraphNorm backward folds them
# (vg_graphnorm_bwd_seg_tiles) when its g_y IS that GEMM output -- a second
# consumer of y would make autograd sum into a new tensor, and the hint holds
# the GEMM output, so the sum cannot land in place.  VGAN_GN_EPI=0: off.
_GN_EPI = os.environ.get("VGAN_GN_EPI", "1") == "1"
_GN_HINTS = {}
_STORE_NOGRAD_KEEP = os.environ.get("VGAN_STORE_NOGRAD_KEEP", "0") == "1"


class _GnHint:
    __slots__ = ("x", "keep", "stats", "weight", "bias", "mean_scale", "eps", "segments", "seg_rows", "tp", "gx")

    def __init__(self, **kw):
        for k in self.__slots__:
            setattr(self, k, kw.get(k))


def gn_hint_for(x: torch.Tensor):
    """The GraphNorm hint of a linear layer's input, or None."""
    if not _GN_HINTS:
        return None
    return _GN_HINTS.get((x.data_ptr(), tuple(x.shape)))


def gemm_gn_bwd(gy: torch.Tensor, weight: torch.Tensor, hint: "_GnHint") -> torch.Tensor:
    """g_x = g_y W (the linear backward's input gradient, = g_y of the
    GraphNorm in ``hint``) with that GraphNorm backward's column partials
    left on the hint."""
    gy, w = _f32(gy), _f32(weight)
    n, k = gy.shape
    m = w.shape[1]
    gx = torch.empty(n, m, dtype=torch.float32, device=gy.device)
    tp = torch.empty(int(LIB.vg_gemm_gn_tpart_floats(n, m)), dtype=torch.float32, device=gy.device)
    check(dense("vg_gemm_gn_bwd")(ptr(gy), k, ptr(w), m, n, m, k, ptr(gx), m, ptr(hint.x), ptr(hint.keep),
                                  hint.seg_rows, ptr(hint.weight), ptr(hint.bias), ptr(hint.mean_scale),
                                  float(hint.eps), ptr(hint.stats), ptr(tp), stream_handle(gy.device)),
          "vg_gemm_gn_bwd")
    hint.tp, hint.gx = tp, gx
    return gx


class _GraphNormReLUDropout(Function):
    """GraphNorm(batch=None) + ReLU + Dropout; ``segments`` > 1 normalises that
    many equal row blocks independently (stacked forwards of one batch)."""

    @staticmethod
    def forward(ctx, x, weight, bias, mean_scale, keep, eps, spec, segments, grad=True):
        # grad: grad mode at the call (a backward will follow): leave the
        # GEMM-epilogue hint; store a dropout mask drawn in-kernel
        x = _f32(x)
        w, b, ms = _f32(weight), _f32(bias), _f32(mean_scale)
        kp = _f32(keep) if keep is not None else None
        require_cuda(x, w, b, ms, kp)
        rows, c = x.shape
        S = int(segments)
        if S < 1 or rows % S:
            raise ValueError("graphnorm: rows must split into equal segments")
        n = rows // S
        if w.numel() != c or b.numel() != c or ms.numel() != c or (kp is not None and kp.shape != x.shape):
            raise ValueError("graphnorm: inconsistent shapes")
        y = torch.empty_like(x)
        stats = torch.empty(S * 2 * c, dtype=torch.float32, device=x.device)
        gnp, g = _take_gnp(x, n)
        ws = None if gnp is not None else \
            torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(S, n, c)), dtype=torch.float32, device=x.device)
        if spec is not None and tuple(spec.shape) != tuple(x.shape):
            raise ValueError("graphnorm: dropout spec shape differs from x")
        if gnp is not None:  # column statistics from the aggregation's partials
            if spec is not None:
                kp = torch.empty_like(x) if grad or _STORE_NOGRAD_KEEP else None
                args = (None, float(spec.p), int(spec.seed), ptr(spec.iter), int(spec.salt) & 0xFFFFFFFF)
            else:
                args = (ptr(kp), 0.0, 0, None, 0)
            check(LIB.vg_graphnorm_fwd_gnp(ptr(x), S, n, c, ptr(w), ptr(b), ptr(ms), *args, float(eps), ptr(y),
                                           ptr(kp) if spec is not None else None, ptr(stats), ptr(gnp), g,
                                           stream_handle(x.device)), "vg_graphnorm_fwd_gnp")
        elif spec is not None:  # dropout drawn in-kernel (device RNG)
            # no backward: apply the mask, do not store it (VGAN_STORE_NOGRAD_KEEP=1: store, A/B knob)
            kp = torch.empty_like(x) if grad or _STORE_NOGRAD_KEEP else None
            check(LIB.vg_graphnorm_fwd_drop(ptr(x), S, n, c, ptr(w), ptr(b), ptr(ms), float(spec.p), int(spec.seed),
                                            ptr(spec.iter), int(spec.salt) & 0xFFFFFFFF, float(eps), ptr(y), ptr(kp),
                                            ptr(stats), ptr(ws), sync_counter(x.device), stream_handle(x.device)),
                  "vg_graphnorm_fwd_drop")
        else:
            check(LIB.vg_graphnorm_fwd_seg(ptr(x), S, n, c, ptr(w), ptr(b), ptr(ms), ptr(kp), float(eps), ptr(y),
                                           ptr(stats), ptr(ws), sync_counter(x.device), stream_handle(x.device)),
                  "vg_graphnorm_fwd_seg")
        ctx.eps, ctx.has_keep, ctx.segments = eps, kp is not None, S
        ctx.params = (weight, bias, mean_scale)
        ctx.save_for_backward(x, weight, bias, mean_scale, kp if kp is not None else x.new_empty(0), stats)
        ctx.hint_key = None
        if _GN_EPI and grad and n >= 64 and c % 4 == 0 and any(ctx.needs_input_grad[:4]):
            if len(_GN_HINTS) > 256:  # forwards whose backward never ran
                _GN_HINTS.clear()
            ctx.hint_key = (y.data_ptr(), tuple(y.shape))
            _GN_HINTS[ctx.hint_key] = _GnHint(x=x, keep=kp, stats=stats, weight=w, bias=b, mean_scale=ms, eps=eps,
                                              segments=S, seg_rows=n)
        return y

    @staticmethod
    def backward(ctx, g_y):
        x, w, b, ms, keep, stats = ctx.saved_tensors
        kp = keep if ctx.has_keep else None
        S = ctx.segments
        if torch.is_grad_enabled():
            ins = [x, w, b, ms]
            with torch.enable_grad():
                parts = zip(x.chunk(S), kp.chunk(S) if kp is not None else [None] * S)
                y = torch.cat([graphnorm_relu_dropout_torch(xs, w, b, ms, ks, ctx.eps) for xs, ks in parts])
                need = [t for t in ins if t.requires_grad]
                grads = torch.autograd.grad(y, need, g_y, create_graph=True, allow_unused=True)
            it = iter(grads)
            res = [next(it) if t.requires_grad else None for t in ins]
            return res[0], res[1], res[2], res[3], None, None, None, None, None
        g_y = _f32(g_y)
        rows, c = x.shape
        n = rows // S
        g_x = torch.empty_like(x)
        pw, pb, pms = ctx.params
        direct = _direct(pw, pb, pms)
        if direct:
            g_w, g_b, g_ms = pw.grad, pb.grad, pms.grad
        else:
            g_w = torch.empty(c, dtype=torch.float32, device=x.device)
            g_b = torch.empty_like(g_w)
            g_ms = torch.empty_like(g_w)
        ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(S, n, c)), dtype=torch.float32, device=x.device)
        hint = _GN_HINTS.pop(ctx.hint_key, None) if ctx.hint_key is not None else None
        if hint is not None and hint.tp is not None and hint.gx is not None and \
                g_y.data_ptr() == hint.gx.data_ptr() and g_y.shape == hint.gx.shape:
            check(LIB.vg_graphnorm_bwd_seg_tiles(ptr(x), S, n, c, ptr(w), ptr(b), ptr(ms), ptr(kp), float(ctx.eps),
                                                 ptr(stats), ptr(g_y), ptr(hint.tp), ptr(g_x), ptr(g_w), ptr(g_b),
                                                 ptr(g_ms), 1 if direct else 0, None, 0, ptr(ws),
                                                 stream_handle(x.device)), "vg_graphnorm_bwd_seg_tiles")
        else:
            check(LIB.vg_graphnorm_bwd_seg(ptr(x), S, n, c, ptr(w), ptr(b), ptr(ms), ptr(kp), float(ctx.eps),
                                           ptr(stats), ptr(g_y), ptr(g_x), ptr(g_w), ptr(g_b), ptr(g_ms),
                                           1 if direct else 0, None, 0, ptr(ws), sync_counter(x.device),
                                           stream_handle(x.device)), "vg_graphnorm_bwd_seg")
        if hint is not None:
            hint.tp = hint.gx = None
        if direct:
            return g_x, None, None, None, None, None, None, None, None
        return g_x, g_w, g_b, g_ms, None, None, None, None, None


def graphnorm_relu_dropout(x, weight, bias, mean_scale, keep, eps: float = 1e-5, segments: int = 1):
    """keep: dropout multipliers [N, C], a ``vgan.rng.DropSpec`` (drawn in-kernel) or None."""
    grad = torch.is_grad_enabled()  # a backward may follow (the GEMM-epilogue hint, the stored mask)
    if keep is not None and not isinstance(keep, torch.Tensor):
        return _GraphNormReLUDropout.apply(x, weight, bias, mean_scale, None, eps, keep, segments, grad)
    return _GraphNormReLUDropout.apply(x, weight, bias, mean_scale, keep, eps, None, segments, grad)


# ------------------------------------------------------ type-matched mean
def type_mean(local_x: torch.Tensor, local_type: torch.Tensor, voxel_type: torch.Tensor, n_types: int,
              out: Optional[torch.Tensor] = None, col0: int = 0) -> torch.Tensor:
    """models.py:122-129 without host syncs (data only, no gradient)."""
    lx = _f32(local_x)
    require_cuda(lx, local_type, voxel_type)
    if local_type.dtype != torch.long or voxel_type.dtype != torch.long:
        raise TypeError("type tensors must be int64")
    nl, f = lx.shape
    nv = voxel_type.numel()
    if out is None:
        out = torch.empty(nv, f, dtype=torch.float32, device=lx.device)
        col0 = 0
    ws = torch.empty(n_types * (f + 1), dtype=torch.float32, device=lx.device)
    lt, vt = local_type.contiguous(), voxel_type.contiguous()  # bound: the kernel reads them after this line
    check(LIB.vg_type_mean(ptr(lx), ptr(lt), nl, f, ptr(vt), nv,
                           int(n_types), ptr(out), out.shape[1], int(col0), ptr(ws), stream_handle(lx.device)),
          "vg_type_mean")
    return out


# ------------------------------------------------------------ Gumbel head
class _GumbelHead(Function):
    @staticmethod
    def forward(ctx, logits, noise, tau):
        lg, nz = _f32(logits), _f32(noise)
        require_cuda(lg, nz)
        if lg.shape != nz.shape or lg.dim() != 2:
            raise ValueError("gumbel_head: logits and noise must be [N, K]")
        soft = torch.empty_like(lg)
        hard = torch.empty_like(lg)
        if isinstance(tau, torch.Tensor):  # per-copy temperatures on the device (inference sweep)
            tt = _f32(tau.reshape(-1))
            require_cuda(tt)
            if lg.shape[0] % tt.numel():
                raise ValueError("gumbel_head: rows must split evenly over the temperatures")
            check(LIB.vg_gumbel_fwd_dev(ptr(lg), ptr(nz), lg.shape[0], lg.shape[1], ptr(tt), lg.shape[0] // tt.numel(),
                                        ptr(soft), ptr(hard), None, stream_handle(lg.device)), "vg_gumbel_fwd_dev")
            ctx.mark_non_differentiable(hard, soft)  # inference only
        else:
            check(LIB.vg_gumbel_fwd(ptr(lg), ptr(nz), lg.shape[0], lg.shape[1], float(tau), ptr(soft), ptr(hard),
                                    None, stream_handle(lg.device)), "vg_gumbel_fwd")
        ctx.tau = tau
        ctx.save_for_backward(soft)
        ctx.set_materialize_grads(False)  # an unused output's gradient stays None (no zero fill launch)
        return hard, soft

    @staticmethod
    def backward(ctx, g_hard, g_soft):
        (soft,) = ctx.saved_tensors
        g_logits = torch.empty_like(soft)
        gh = _f32(g_hard) if g_hard is not None else None
        gs = _f32(g_soft) if g_soft is not None else None
        check(LIB.vg_gumbel_bwd(ptr(soft), ptr(gh), ptr(gs), soft.shape[0], soft.shape[1], float(ctx.tau),
                                ptr(g_logits), stream_handle(soft.device)), "vg_gumbel_bwd")
        return g_logits, None, None


def gumbel_head(logits: torch.Tensor, noise: torch.Tensor, tau: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor]:
    """(label_hard, label_soft) of models.py:150-153 given Exp(1) noise."""
    return _GumbelHead.apply(logits, noise, tau)


# ------------------------------------------------------- per-building work
def far_per_graph(x, label, ptr_, site_area, far_col=9, dy_col=4, dx_col=5, dim_scale=11.0, void_class=6):
    require_cuda(x, label, ptr_, site_area)
    g = ptr_.numel() - 1
    gen = torch.empty(g, dtype=torch.float32, device=x.device)
    ref = torch.empty_like(gen)
    lbl = _f32(label.detach())
    xc, pc, sa = _f32(x), ptr_.contiguous(), _f32(site_area)
    check(LIB.vg_far_per_graph(ptr(xc), xc.shape[1], ptr(lbl), lbl.shape[1], ptr(pc), g,
                               ptr(sa), far_col, dy_col, dx_col, float(dim_scale), void_class,
                               ptr(gen), ptr(ref), stream_handle(x.device)), "vg_far_per_graph")
    return gen, ref


class _GenLossHead(Function):
    """The WGAN-GP generator loss (trainer.py:334-385) as two launches forward
    and one backward (vg_gen_loss_fwd / _bwd) instead of ~40 small torch
    kernels.  The FAR term enters the value only (no gradient, :380); the
    label cross-entropy's gradient is returned only when its weight is not 0
    (0 x a finite gradient is exactly 0)."""

    @staticmethod
    def forward(ctx, d_fake, hard, logits, onehot, vtype, far_gen, far_ref, lambdas):
        df, hd, lg, oh = (_f32(t.reshape(t.shape[-2], -1) if t.dim() > 2 else t) for t in (d_fake, hard, logits, onehot))
        df = df.reshape(-1).contiguous()
        require_cuda(df, hd, lg, oh, vtype, far_gen, far_ref)
        n, k = hd.shape
        if df.numel() != n or lg.shape != (n, k) or oh.shape != (n, k) or vtype.numel() != n:
            raise ValueError("gen_loss_head: inconsistent shapes")
        dev = hd.device
        out = torch.empty(k + 3, dtype=torch.float32, device=dev)
        ws = torch.empty(int(LIB.vg_gen_loss_ws_floats(n, k)), dtype=torch.float32, device=dev)
        l_adv, l_label, l_ratio, l_void, l_far = (float(v) for v in lambdas)
        check(LIB.vg_gen_loss_fwd(ptr(df), ptr(hd), ptr(lg), ptr(oh), ptr(vtype), n, k, ptr(_f32(far_gen)),
                                  ptr(_f32(far_ref)), far_gen.numel(), l_adv, l_label, l_ratio, l_void, l_far,
                                  ptr(out), ptr(ws), stream_handle(dev)), "vg_gen_loss_fwd")
        ctx.l_label = l_label
        ctx.shapes = (d_fake.shape, hard.shape, logits.shape)
        ctx.save_for_backward(out, lg, vtype)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        out, lg, vtype = ctx.saved_tensors
        n, k = lg.shape
        dev = lg.device
        g = _f32(g.reshape(1))
        need_d, need_h, need_l = ctx.needs_input_grad[:3]
        need_l = need_l and ctx.l_label != 0.0
        g_d = torch.empty(n, dtype=torch.float32, device=dev) if need_d else None
        g_h = torch.empty(n, k, dtype=torch.float32, device=dev) if need_h else None
        g_l = torch.empty(n, k, dtype=torch.float32, device=dev) if need_l else None
        check(LIB.vg_gen_loss_bwd(ptr(g), ptr(out), ptr(lg), ptr(vtype), n, k, ptr(g_d), ptr(g_h), ptr(g_l),
                                  stream_handle(dev)), "vg_gen_loss_bwd")
        sd, sh, sl = ctx.shapes
        return (g_d.view(sd) if g_d is not None else None, g_h.view(sh) if g_h is not None else None,
                g_l.view(sl) if g_l is not None else None, None, None, None, None, None)


def gen_loss_head(d_fake, hard, logits, onehot, vtype, far_gen, far_ref, lambdas) -> torch.Tensor:
    """WGAN-GP generator loss (device scalar); lambdas = (adv, label, ratio, ratio_void, far)."""
    return _GenLossHead.apply(d_fake, hard, logits, onehot, vtype, far_gen, far_ref, tuple(lambdas))


def confusion(truth, label, ptr_):
    require_cuda(truth, label, ptr_)
    g = ptr_.numel() - 1
    k = label.shape[1]
    conf = torch.empty(g, k, k, dtype=torch.int32, device=label.device)
    conf_all = torch.empty(k, k, dtype=torch.int32, device=label.device)
    lbl = _f32(label.detach())
    tc, pc = truth.contiguous(), ptr_.contiguous()
    check(LIB.vg_confusion(ptr(tc), ptr(lbl), k, ptr(pc), g, ptr(conf), ptr(conf_all),
                           stream_handle(label.device)), "vg_confusion")
    return conf, conf_all


# --------------------------------------------------------------- dense GEMMs
ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2


class _LNAct(Function):
    """leaky_relu(LayerNorm(x)) in one kernel (vg_ln_act_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, slope):
        x, g, b = _f32(x), _f32(gamma), _f32(beta)
        require_cuda(x, g, b)
        n, c = x.shape
        if g.numel() != c or b.numel() != c:
            raise ValueError("ln_act: inconsistent shapes")
        y = torch.empty_like(x)
        save = any(ctx.needs_input_grad[:3])  # (grad mode is off inside Function.forward)
        mean = torch.empty(n, dtype=torch.float32, device=x.device) if save else None
        rstd = torch.empty(n, dtype=torch.float32, device=x.device) if save else None
        check(LIB.vg_ln_act_fwd(ptr(x), n, c, ptr(g), ptr(b), float(eps), float(slope), ptr(y), ptr(mean), ptr(rstd),
                                stream_handle(x.device)), "vg_ln_act_fwd")
        ctx.eps, ctx.slope = eps, slope
        ctx.params = (gamma, beta)
        if save:
            ctx.save_for_backward(x, gamma, beta, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, g_y):
        x, gamma, beta, mean, rstd = ctx.saved_tensors
        n, c = x.shape
        if torch.is_grad_enabled():  # create_graph: differentiable torch restatement
            leaves = [t.detach().requires_grad_(t.requires_grad) for t in (x, gamma, beta)]
            with torch.enable_grad():
                y = torch.nn.functional.leaky_relu(
                    torch.nn.functional.layer_norm(leaves[0], (c,), leaves[1], leaves[2], ctx.eps), ctx.slope)
                need = [t for t in leaves if t.requires_grad]
                grads = iter(torch.autograd.grad(y, need, g_y, create_graph=True))
            res = [next(grads) if t.requires_grad else None for t in leaves]
            return res[0], res[1], res[2], None, None
        g_y = _f32(g_y)
        g_x = torch.empty_like(x)
        pg, pb = ctx.params
        direct = _direct(pg, pb)
        if direct:
            g_g, g_b = pg.grad, pb.grad
        else:
            g_g = torch.empty(c, dtype=torch.float32, device=x.device)
            g_b = torch.empty_like(g_g)
        ws = torch.empty(int(LIB.vg_ln_act_bwd_ws_floats(c)), dtype=torch.float32, device=x.device)
        check(LIB.vg_ln_act_bwd(ptr(x), n, c, ptr(gamma), ptr(beta), float(ctx.slope), ptr(mean), ptr(rstd), ptr(g_y),
                                ptr(g_x), ptr(g_g), ptr(g_b), 1 if direct else 0, ptr(ws), stream_handle(x.device)),
              "vg_ln_act_bwd")
        if direct:
            return g_x, None, None, None, None
        return g_x, g_g, g_b, None, None


def ln_act_backward(x, gamma, beta, eps, slope, mean, rstd, g_y, params, want_params: bool = True):
    """First-order backward of leaky_relu(LayerNorm(x)) (vg_ln_act_bwd) from the
    saved row statistics: (g_x, g_gamma, g_beta); the parameter gradients are
    accumulated straight into ``params``' .grad under direct_param_grads (then
    returned as None)."""
    del eps  # mean / rstd already carry it
    g_y = _f32(g_y)
    n, c = x.shape
    g_x = torch.empty_like(x)
    pg, pb = params
    direct = want_params and _direct(pg, pb)
    if direct:
        g_g, g_b = pg.grad, pb.grad
    else:
        g_g = torch.empty(c, dtype=torch.float32, device=x.device)
        g_b = torch.empty_like(g_g)
    ws = torch.empty(int(LIB.vg_ln_act_bwd_ws_floats(c)), dtype=torch.float32, device=x.device)
    args = (ptr(x), n, c, ptr(gamma), ptr(beta), float(slope), ptr(mean), ptr(rstd), ptr(g_y), ptr(g_x), ptr(g_g),
            ptr(g_b), 1 if direct else 0, ptr(ws))
    if direct and _FOLDS is not None:  # gamma / beta fold deferred to the context's batch
        _FOLDS.call(LIB.vg_ln_act_bwd_deferred, args, stream_handle(x.device), keep=(ws,),
                    name="vg_ln_act_bwd_deferred")
    else:
        check(LIB.vg_ln_act_bwd(*args, stream_handle(x.device)), "vg_ln_act_bwd")
    if direct or not want_params:
        return g_x, None, None
    return g_x, g_g, g_b


def ln_act(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-5, slope: float = 0.2):
    """nn.LayerNorm(C) followed by nn.LeakyReLU(slope) (models.py:33-113)."""
    return _LNAct.apply(x, gamma, beta, eps, slope)


def gemm(a: torch.Tensor, b: torch.Tensor, b_trans: bool, bias: Optional[torch.Tensor] = None,
         act: int = ACT_NONE) -> torch.Tensor:
    """C = a . (b^T if b_trans else b) (+ bias) (+ act), f32 MFMA (vg_gemm)."""
    a, b = _f32(a), _f32(b)
    bb = _f32(bias) if bias is not None else None
    require_cuda(a, b, bb)
    n, k = a.shape
    m = b.shape[0] if b_trans else b.shape[1]
    if (b.shape[1] if b_trans else b.shape[0]) != k:
        raise ValueError("gemm: inner dimensions differ")
    c = torch.empty(n, m, dtype=torch.float32, device=a.device)
    check(dense("vg_gemm")(ptr(a), k, ptr(b), b.shape[1], 1 if b_trans else 0, ptr(bb), int(act), None, 0, ptr(c), m, n,
                      m, k, stream_handle(a.device)), "vg_gemm")
    return c


def lin_att(x: torch.Tensor, w: torch.Tensor, att_src: torch.Tensor, att_dst: torch.Tensor):
    """(h = x w^T, h . att_src, h . att_dst) from one launch (vg_gat_lin_att):
    GATConv.lin plus the attention projections, the latter in the GEMM's
    epilogue."""
    x, w = _f32(x), _f32(w)
    vs, vd = _f32(att_src.reshape(-1)), _f32(att_dst.reshape(-1))
    require_cuda(x, w, vs, vd)
    n, k = x.shape
    c = w.shape[0]
    if w.shape[1] != k or vs.numel() != c or vd.numel() != c:
        raise ValueError("lin_att: inconsistent shapes")
    h = torch.empty(n, c, dtype=torch.float32, device=x.device)
    a_s = torch.empty(n, dtype=torch.float32, device=x.device)
    a_d = torch.empty(n, dtype=torch.float32, device=x.device)
    check(dense("vg_gat_lin_att")(ptr(x), k, ptr(w), n, k, c, ptr(vs), ptr(vd), ptr(h), ptr(a_s), ptr(a_d),
                             stream_handle(x.device)), "vg_gat_lin_att")
    return h, a_s, a_d


def gemm_tn(a: torch.Tensor, b: torch.Tensor, want_colsum: bool = True):
    """(a^T . b, column sums of a): the weight / bias gradient of nn.Linear."""
    a, b = _f32(a), _f32(b)
    require_cuda(a, b)
    n, m = a.shape
    k = b.shape[1]
    if b.shape[0] != n:
        raise ValueError("gemm_tn: row counts differ")
    c = torch.empty(m, k, dtype=torch.float32, device=a.device)
    db = torch.empty(m, dtype=torch.float32, device=a.device) if want_colsum else None
    ws = torch.empty(max(1, int(LIB.vg_gemm_tn_ws_floats(n, m, k))), dtype=torch.float32, device=a.device)
    check(dense("vg_gemm_tn")(ptr(a), m, ptr(b), k, n, m, k, ptr(c), k, ptr(db), 0, ptr(ws), stream_handle(a.device)),
          "vg_gemm_tn")
    return c, db


def gemm_tn_into(a: torch.Tensor, b: torch.Tensor, c_out: torch.Tensor, db_out: Optional[torch.Tensor]) -> None:
    """c_out += a^T b and db_out += column sums of a (accumulating vg_gemm_tn)."""
    a, b = _f32(a), _f32(b)
    require_cuda(a, b, c_out, db_out)
    n, m = a.shape
    k = b.shape[1]
    if b.shape[0] != n or tuple(c_out.shape) != (m, k):
        raise ValueError("gemm_tn_into: inconsistent shapes")
    ws = torch.empty(max(1, int(LIB.vg_gemm_tn_ws_floats(n, m, k))), dtype=torch.float32, device=a.device)
    if _FOLDS is not None and n > 0:  # fold deferred to the context's batch
        _FOLDS.tn((ptr(a), m, ptr(b), k, n, m, k, ptr(c_out), k, ptr(db_out), n, 1, ptr(ws)),
                  stream_handle(a.device), keep=(ws, a, b))
        return
    check(dense("vg_gemm_tn")(ptr(a), m, ptr(b), k, n, m, k, ptr(c_out), k, ptr(db_out), 1, ptr(ws),
                         stream_handle(a.device)), "vg_gemm_tn")


def adam_flat_dev(param, grad, exp_avg, exp_avg_sq, beta1, beta2, eps, weight_decay, lr_t, step_t):
    """vg_adam_dev: lr (float64 [1]) and the incremented step (int32 [1]) on the device."""
    require_cuda(param, grad, exp_avg, exp_avg_sq, lr_t, step_t)
    check(LIB.vg_adam_dev(ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), param.numel(), float(beta1),
                          float(beta2), float(eps), float(weight_decay), ptr(lr_t), ptr(step_t),
                          stream_handle(param.device)), "vg_adam_dev")


def adam_flat(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step: int):
    require_cuda(param, grad, exp_avg, exp_avg_sq)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    check(LIB.vg_adam(ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), param.numel(), float(beta2),
                      float(1.0 - beta1), float(1.0 - beta2), float(eps), float(weight_decay), float(lr / bc1),
                      float(bc2 ** 0.5), stream_handle(param.device)), "vg_adam")


__all__ = [
    "CSR", "gat_conv", "gat_conv_composed", "gat_aggregate_composed", "graphnorm_relu_dropout", "type_mean", "gumbel_head",
    "spmm", "spmm_t", "sddmm", "gather", "seg_sum", "seg_max", "scatter_src", "far_per_graph", "confusion",
    "adam_flat", "_lib",
]
