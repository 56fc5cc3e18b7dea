"""VoxelGNNGenerator / VoxelGNNDiscriminator on the HIP message-passing core.

Drop-in for ``building_gan/src/models.py``:

* constructor signatures ``(configuration, local_graph_dim, voxel_graph_dim)``
  and ``forward`` signatures/returns are the reference's (``models.py:15,119,
  159,229``);
* parameter names are the reference state_dict keys
  (``matched_features_encoder.{i}``, ``mlp_encoder.{i}``,
  ``encoder.module_{i}.{lin.weight,att_src,att_dst,bias | weight,bias,mean_scale}``,
  ``decoder.{i}``), so reference checkpoints load unchanged;
* construction consumes the CPU generator in the reference's order with the
  same initialisers (torch defaults for Linear, glorot for GATConv), so the
  same seed yields the same initial weights.

Every GATConv block runs ``gat_conv`` (fused attention projections, logits,
segment softmax, aggregation and bias) followed by ``graphnorm_relu_dropout`` (GraphNorm with batch=None,
ReLU and Dropout in one op).  The type-matched mean, CSR and float one-hot are
per-batch data and are computed once per mini-batch (``vgan.data``).
"""
from __future__ import annotations

import ctypes
import math
from typing import List, Optional

import torch
import torch.nn as nn

from . import data as vdata
from . import ops
from ._lib import gemm_precision
from .nn import MLP, Linear, linear_att, linear_ln_act, run_blocks
from .rng import RNG

_CONV_TYPES = ("GCNCONV", "GRAPHCONV", "GATCONV", "GATV2CONV")


def _glorot_(t: torch.Tensor) -> None:
    bound = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-bound, bound)


class _GATLin(nn.Module):
    """The bias-free, glorot-initialised projection of GATConv (``lin.weight``)."""

    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(cout, cin))
        _glorot_(self.weight)  # torch_geometric Linear.__init__ -> reset_parameters


class GATConv(nn.Module):
    """GATConv(in, out) with heads=1 (torch_geometric 2.6.1 defaults) on the HIP core."""

    def __init__(self, in_channels: int, out_channels: int, negative_slope: float = 0.2):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.negative_slope = negative_slope
        self.lin = _GATLin(in_channels, out_channels)
        self.att_src = nn.Parameter(torch.empty(1, 1, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, 1, out_channels))
        self.bias = nn.Parameter(torch.empty(out_channels))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        _glorot_(self.lin.weight)
        _glorot_(self.att_src)
        _glorot_(self.att_dst)
        with torch.no_grad():
            self.bias.zero_()

    def forward(self, x: torch.Tensor, csr: ops.CSR) -> torch.Tensor:
        # projection + attention projections in one launch, then the edge
        # softmax / gather-sum kernel
        h, a_s, a_d = linear_att(x, self.lin.weight, self.att_src, self.att_dst)
        return ops.gat_conv(csr, h, self.att_src, self.att_dst, self.bias, self.negative_slope, pre=(a_s, a_d))


class GraphNorm(nn.Module):
    def __init__(self, channels: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(channels))
        self.bias = nn.Parameter(torch.zeros(channels))
        self.mean_scale = nn.Parameter(torch.ones(channels))


class GATEncoder(nn.Module):
    """The ``tgnn.Sequential("x, edge_index", [...])`` stack of models.py:68-90 /
    187-210: ``depth`` halving blocks then ``depth`` doubling blocks, each
    [GATConv -> GraphNorm -> ReLU -> Dropout] (children ``module_{4b+0..3}``)."""

    # no-grad forwards apply each GraphNorm in the next projection GEMM
    # (_forward_nograd_fused); False: the module path (tests compare the two)
    fused_nograd = True

    def __init__(self, width: int, depth: int, dropout: float = 0.2):
        super().__init__()
        self.dropout = dropout
        chans = [width]
        for _ in range(depth):
            chans.append(chans[-1] // 2)
        for _ in range(depth):
            chans.append(chans[-1] * 2)
        self.widths = chans
        self.num_blocks = 2 * depth
        for b, (cin, cout) in enumerate(zip(chans[:-1], chans[1:])):
            self.add_module(f"module_{4 * b}", GATConv(cin, cout))
            self.add_module(f"module_{4 * b + 1}", GraphNorm(cout))
            self.add_module(f"module_{4 * b + 2}", nn.ReLU(True))
            self.add_module(f"module_{4 * b + 3}", nn.Dropout(dropout))

    @property
    def out_channels(self) -> int:
        return self.widths[-1]

    def forward(self, x: torch.Tensor, csr: ops.CSR, rng: RNG, segments: int = 1) -> torch.Tensor:
        """``segments`` > 1: x holds that many stacked copies of the batch (csr
        block-diagonal), each normalised on its own as a separate forward."""
        if self.fused_nograd and ops._GN_FWD_FUSE and not torch.is_grad_enabled() and x.is_cuda and x.dim() == 2 \
                and gemm_precision() == "f32":
            y = self._forward_nograd_fused(x, csr, rng, segments)
            if y is not None:
                return y
        for b in range(self.num_blocks):
            conv: GATConv = getattr(self, f"module_{4 * b}")
            norm: GraphNorm = getattr(self, f"module_{4 * b + 1}")
            h = conv(x, csr)
            keep = rng.keep_mask(h.shape, self.dropout, h.device) if self.training else None
            x = ops.graphnorm_relu_dropout(h, norm.weight, norm.bias, norm.mean_scale, keep, norm.eps, segments)
        _ring_checked(csr)
        return x


    def _forward_nograd_fused(self, x: torch.Tensor, csr: ops.CSR, rng: RNG, segments: int):
        """The no-grad forward (critic labels, validation, inference) with each
        block's GraphNorm + ReLU + Dropout applied by the NEXT block's
        projection GEMM as it loads its operand (vg_gat_lin_att_gn) -- nothing
        needs the normalised activations afterwards, so they are never
        written: one launch and one [rows, C] write + read fewer per block.
        The statistics still come from the aggregation's partials
        (vg_graphnorm_stats_gnp); the dropout multipliers are the same Philox
        draws (in-kernel, device RNG) or none (eval).  The projection sees the
        apply kernel's values up to FMA contraction (1e-6,
        tests/test_gnp_gpu.py).  None (the caller runs the module path) for
        host-drawn masks, C > 64 projections or short segments."""
        from ._lib import LIB, VgGnApply, check, dense, ptr, stream_handle, sync_counter

        rows = x.shape[0]
        S = int(segments)
        n = rows // S
        if rows % S or n < 64 or not x.is_contiguous():
            return None
        if self.training and getattr(rng, "mode", None) != "device":
            return None  # host / fixed masks are tensors: the module path (decided before any draw)
        if csr.seg_rows != n or csr.num_nodes != rows:
            return None
        for c in self.widths[1:]:  # every block's aggregation must form its GraphNorm partials
            g = int(LIB.vg_gat_gnp_rows(rows, c))
            if g <= 0 or n < g:
                return None
        dev = x.device
        st = stream_handle(dev)
        pend = None  # (O, desc, stats, c): the previous block's GraphNorm, applied in this projection
        for b in range(self.num_blocks):
            conv: GATConv = getattr(self, f"module_{4 * b}")
            norm: GraphNorm = getattr(self, f"module_{4 * b + 1}")
            c = conv.out_channels
            spec = rng.keep_mask((rows, c), self.dropout, dev) if self.training else None
            if spec is not None and isinstance(spec, torch.Tensor):
                raise RuntimeError("device RNG returned a mask tensor")
            H = torch.empty(rows, c, dtype=torch.float32, device=dev)
            a_s = torch.empty(rows, dtype=torch.float32, device=dev)
            a_d = torch.empty(rows, dtype=torch.float32, device=dev)
            if pend is not None:
                xin, desc, _, cin = pend
                check(LIB.vg_gat_lin_att_gn(ptr(xin), ptr(conv.lin.weight), rows, cin, c, ptr(conv.att_src),
                                            ptr(conv.att_dst), ptr(H), ptr(a_s), ptr(a_d), ctypes.byref(desc), st),
                      "vg_gat_lin_att_gn")
                pend = None
            else:
                cin = x.shape[1]
                check(dense("vg_gat_lin_att")(ptr(x), cin, ptr(conv.lin.weight), rows, cin, c, ptr(conv.att_src),
                                              ptr(conv.att_dst), ptr(H), ptr(a_s), ptr(a_d), st), "vg_gat_lin_att")
            O = torch.empty(rows, c, dtype=torch.float32, device=dev)
            alpha = torch.empty(csr.num_edges, dtype=torch.float32, device=dev)
            gnp, g = ops.gnp_buffer(csr, c, dev)  # None: a ring layer without partials (VGAN_RING_GNP=0)
            ops.aggregate_fwd_raw(csr, c, ptr(H), ptr(a_s), ptr(a_d), ptr(conv.bias), float(conv.negative_slope),
                                  ptr(O), ptr(alpha), st, gnp)
            stats = torch.empty(S * 2 * c, dtype=torch.float32, device=dev)
            ws = None if gnp is not None else \
                torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(S, n, c)), dtype=torch.float32, device=dev)
            nxt = getattr(self, f"module_{4 * (b + 1)}").out_channels if b + 1 < self.num_blocks else 0
            drop = (float(spec.p), int(spec.seed), ptr(spec.iter), int(spec.salt) & 0xFFFFFFFF) if spec is not None \
                else (0.0, 0, None, 0)
            if 0 < nxt <= 64 and c <= 128 and c % 4 == 0:
                if gnp is not None:
                    check(LIB.vg_graphnorm_stats_gnp(S, n, c, ptr(gnp), g, ptr(norm.mean_scale), float(norm.eps),
                                                     ptr(stats), st), "vg_graphnorm_stats_gnp")
                else:
                    check(LIB.vg_graphnorm_stats(ptr(O), S, n, c, ptr(norm.mean_scale), float(norm.eps), ptr(stats),
                                                 ptr(ws), st), "vg_graphnorm_stats")
                desc = VgGnApply(stats=stats.data_ptr(), weight=norm.weight.data_ptr(), bias=norm.bias.data_ptr(),
                                 mean_scale=norm.mean_scale.data_ptr(), keep=None, eps=float(norm.eps),
                                 p_drop=drop[0], seg_rows=n, salt=drop[3], seed=drop[1], iter=drop[2], y=None,
                                 keep_out=None)
                pend = (O, desc, stats, c)  # stats / O stay referenced until the GEMM is enqueued
                continue
            y = torch.empty(rows, c, dtype=torch.float32, device=dev)
            w_, b_, ms_ = ptr(norm.weight), ptr(norm.bias), ptr(norm.mean_scale)
            if gnp is not None:
                check(LIB.vg_graphnorm_fwd_gnp(ptr(O), S, n, c, w_, b_, ms_, None, *drop, float(norm.eps), ptr(y), None,
                                               ptr(stats), ptr(gnp), g, st), "vg_graphnorm_fwd_gnp")
            elif spec is not None:
                check(LIB.vg_graphnorm_fwd_drop(ptr(O), S, n, c, w_, b_, ms_, *drop, float(norm.eps), ptr(y), None,
                                                ptr(stats), ptr(ws), sync_counter(dev), st), "vg_graphnorm_fwd_drop")
            else:
                check(LIB.vg_graphnorm_fwd_seg(ptr(O), S, n, c, w_, b_, ms_, None, float(norm.eps), ptr(y), ptr(stats),
                                               ptr(ws), sync_counter(dev), st), "vg_graphnorm_fwd_seg")
            x = y
        _ring_checked(csr)
        return x


def _ring_checked(csr: ops.CSR) -> None:
    """After an encoder forward that aggregated on the LDS ring (large graphs,
    ops.CSR.ring_on): raise if one of its bounded hand-over waits expired --
    one host sync per such forward, none inside a stream capture."""
    if csr.__dict__.pop("_ring_used", False) and not torch.cuda.is_current_stream_capturing():
        csr.ring_check()


def _mlp(widths: List[int], norm: bool, act) -> MLP:
    mods: List[nn.Module] = []
    for a, b in zip(widths[:-1], widths[1:]):
        mods.append(Linear(a, b))
        if norm:
            mods.append(nn.LayerNorm(b))
        mods.append(act())
    return MLP(*mods)


def _check_conv(kind: str) -> None:
    if kind not in _CONV_TYPES:
        raise ValueError(f"Invalid conv_type: {kind}")
    if kind != "GATCONV":
        raise NotImplementedError(f"{kind}: only GATCONV (the configured default) has a HIP path")


class VoxelGNNGenerator(nn.Module):
    """models.py:14-155."""

    def __init__(self, configuration, local_graph_dim: int, voxel_graph_dim: int):
        super().__init__()
        cfg = configuration
        _check_conv(cfg.GENERATOR_CONV_TYPE)
        self.configuration = cfg
        self.local_graph_dim, self.voxel_graph_dim = local_graph_dim, voxel_graph_dim
        hl, hg, zd = cfg.LOCAL_ENCODER_HIDDEN_DIM, cfg.GENERATOR_HIDDEN_DIM, cfg.Z_DIM
        lrelu = lambda: nn.LeakyReLU(0.2)  # noqa: E731
        self.matched_features_encoder = _mlp([local_graph_dim] + [hl] * (cfg.LOCAL_GRAPH_ENCODER_REPEAT + 1), True,
                                             lrelu)
        self.mlp_encoder = _mlp([hl + voxel_graph_dim + zd] + [hg] * (cfg.GENERATOR_MLP_ENCODER_REPEAT + 1), True,
                                lrelu)
        self.encoder = GATEncoder(hg, cfg.GENERATOR_ENCODER_REPEAT, cfg.ENCODER_DROPOUT_RATE)
        dec = list(_mlp([hl + voxel_graph_dim + zd + self.encoder.out_channels + hg, hg, hg // 2, hg // 4, hg // 8],
                        True, lrelu).children())
        dec.append(Linear(hg // 8, cfg.NUM_CLASSES))
        self.decoder = MLP(*dec)
        self.rng = RNG(getattr(cfg, "runtime", {}).get("rng", "device"))
        self.tau = 1.0
        self.to(cfg.DEVICE)

    def _mlp_blocks(self, mlp: nn.Module):
        mods = list(mlp.children())
        return [tuple(mods[i:i + 3]) for i in range(0, len(mods) - 2, 3)
                if isinstance(mods[i], nn.Linear) and isinstance(mods[i + 1], nn.LayerNorm)
                and isinstance(mods[i + 2], nn.LeakyReLU)]

    def _first_block_ms(self, block, srcs, emvx, emvx_w0, rows, n):
        """First [Linear, LayerNorm, LeakyReLU] block over stacked copies:
        the copy-invariant columns [em | voxel.x] once on N rows (vg_gemm into
        the addend, bias included), the per-copy columns read in place from
        their own tensors (vg_gemm_ln_act_ms) -- no torch.cat, no repeat."""
        from ._lib import LIB, VgASrc, check, dense, ptr, stream_handle

        lin, ln, act = block
        w = lin.weight
        m, ktot = w.shape
        dev = w.device
        st = stream_handle(dev)
        add = torch.empty(n, m, dtype=torch.float32, device=dev)
        check(dense("vg_gemm")(ptr(emvx), emvx.shape[1], ctypes.c_void_p(w.data_ptr() + 4 * emvx_w0), ktot, 1, ptr(lin.bias),
                          0, None, 0, ptr(add), m, n, m, emvx.shape[1], st), "vg_gemm")
        arr = (VgASrc * len(srcs))(*[VgASrc(t.data_ptr(), t.stride(0), cols, w0, 0) for t, cols, w0 in srcs])
        y = torch.empty(rows, m, dtype=torch.float32, device=dev)
        check(dense("vg_gemm_ln_act_ms")(arr, len(srcs), ptr(w), ktot, rows, m, None, ptr(add), m, n, ptr(ln.weight),
                                    ptr(ln.bias), float(ln.eps), float(act.negative_slope), ptr(y), m, st),
              "vg_gemm_ln_act_ms")
        return y

    def _forward_stacked_nograd(self, prep, z, k: int):
        """The no-grad forward over k stacked copies (critic labels, inference
        sweep): models.py:119-145 with both concatenations replaced by
        multi-source GEMMs and the copy-invariant [em | voxel.x] products
        formed once per building batch.  None when a layer shape falls outside
        the fused kernels (then the generic path runs)."""
        mlp_b, dec_b = self._mlp_blocks(self.mlp_encoder), self._mlp_blocks(self.decoder)
        if not mlp_b or not dec_b or not all(64 < b[0].out_features <= 128 for b in (mlp_b[0], dec_b[0])):
            return None
        em = self.matched_features_encoder(prep.matched_x)
        vx = prep.voxel_x
        n = vx.shape[0]
        rows = k * n
        hl, vd = em.shape[1], vx.shape[1]
        zz = z.reshape(rows, -1).contiguous()
        zd = zz.shape[1]
        emvx = torch.cat([em, vx], dim=-1).contiguous()  # N rows only
        # MLP encoder input [em | voxel.x | z] (models.py:131)
        x = self._first_block_ms(mlp_b[0], [(zz, zd, hl + vd)], emvx, 0, rows, n)
        for lin, ln, act in mlp_b[1:]:
            x = linear_ln_act(x, lin.weight, lin.bias, ln.weight, ln.bias, ln.eps, act.negative_slope)
        csr = prep.csr.stacked(k)
        enc = self.encoder(x, csr, self.rng, segments=k)
        ec, hg = enc.shape[1], x.shape[1]
        # decoder input [enc | x | em | voxel.x | z] (models.py:145)
        d = self._first_block_ms(dec_b[0], [(enc, ec, 0), (x, hg, ec), (zz, zd, ec + hg + hl + vd)], emvx, ec + hg,
                                 rows, n)
        mods = list(self.decoder.children())[3:]
        return run_blocks(mods, d)

    def forward(self, local_graph, voxel_graph, z, noise: Optional[torch.Tensor] = None,
                stacked: Optional[bool] = None):
        """z [1, N, Z] (the reference's shape) -> ([N, 7] x 3).  z [k, N, Z]
        with k > 1 draws k independent samples in ONE stacked forward (the
        critic iterations' generator passes, or an inference sweep) and
        returns [k, N, 7] tensors; the program-feature encoder runs once.
        ``stacked=True`` takes that no-grad path (multi-source first layers,
        no concatenation) at k = 1 too, returning [1, N, 7] tensors."""
        prep = vdata.prepared(local_graph, voxel_graph, self.configuration.NUM_CLASSES)
        k = z.shape[0] if z.dim() == 3 else 1
        use_stacked = k > 1 if stacked is None else bool(stacked)
        if use_stacked and not torch.is_grad_enabled() and prep.voxel_x.is_cuda:
            logits = self._forward_stacked_nograd(prep, z, k)
            if logits is not None:
                n = prep.voxel_x.shape[0]
                if noise is None:
                    noise = self.rng.exponential(logits.shape, logits.device)
                label_hard, label_soft = ops.gumbel_head(logits, noise.reshape(logits.shape), self.tau)
                return logits.view(k, n, -1), label_hard.view(k, n, -1), label_soft.view(k, n, -1)
        em = self.matched_features_encoder(prep.matched_x)
        vx = prep.voxel_x
        n = vx.shape[0]
        if k == 1:
            zz = z.reshape(n, -1)
            csr = prep.csr
        else:
            zz = z.reshape(k * n, -1)
            em = em.repeat(k, 1)
            vx = vx.repeat(k, 1)
            csr = prep.csr.stacked(k)
        x = self.mlp_encoder(torch.cat([em, vx, zz], dim=-1))
        enc = self.encoder(x, csr, self.rng, segments=k)
        logits = self.decoder(torch.cat([enc, x, em, vx, zz], dim=-1))
        if noise is None:
            noise = self.rng.exponential(logits.shape, logits.device)
        label_hard, label_soft = ops.gumbel_head(logits, noise.reshape(logits.shape), self.tau)
        if k > 1:
            return logits.view(k, n, -1), label_hard.view(k, n, -1), label_soft.view(k, n, -1)
        return logits, label_hard, label_soft


class VoxelGNNDiscriminator(nn.Module):
    """models.py:158-245 (per-node critic scores [N, 1])."""

    def __init__(self, configuration, local_graph_dim: int, voxel_graph_dim: int):
        super().__init__()
        cfg = configuration
        _check_conv(cfg.DISCRIMINATOR_CONV_TYPE)
        self.configuration = cfg
        self.local_graph_dim, self.voxel_graph_dim = local_graph_dim, voxel_graph_dim
        hd = cfg.DISCRIMINATOR_HIDDEN_DIM
        relu = lambda: nn.ReLU(True)  # noqa: E731
        self.mlp_encoder = _mlp([local_graph_dim + voxel_graph_dim + cfg.NUM_CLASSES, hd, hd], False, relu)
        self.encoder = GATEncoder(hd, cfg.DISCRIMINATOR_ENCODER_REPEAT, cfg.ENCODER_DROPOUT_RATE)
        dec = list(_mlp([hd, hd // 2, hd // 4, hd // 8], False, relu).children())
        dec.append(Linear(hd // 8, 1))
        if not cfg.USE_WGANGP:
            dec.append(nn.Sigmoid())
        self.decoder = MLP(*dec)
        self.rng = RNG(getattr(cfg, "runtime", {}).get("rng", "device"))
        self.to(cfg.DEVICE)

    def forward(self, local_graph, voxel_graph, label_hard):
        prep = vdata.prepared(local_graph, voxel_graph, self.configuration.NUM_CLASSES)
        label = label_hard.squeeze(0)
        if label.dtype != torch.float32:
            label = label.to(torch.float32)
        feats = torch.cat([prep.matched_voxel_x, label], dim=-1)
        return self.decoder(self.encoder(self.mlp_encoder(feats), prep.csr, self.rng))
