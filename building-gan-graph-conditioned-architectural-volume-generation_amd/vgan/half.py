"""f16 generator forward for inference (BASELINE.json configs[4]: "Generator-only
inference sweep ... fp16").

``HalfGenerator(G)`` snapshots a ``VoxelGNNGenerator``'s parameters into the f16
layout of ``include/vgan.h``'s f16 section and runs the eval-mode forward of
``models.py:119-155`` on the f16 kernels:

* every [Linear, LayerNorm, LeakyReLU] block is one ``vg_hgemm_ln_act`` (f16
  MFMA, LayerNorm in the epilogue), the decoder head one ``vg_hgemm`` with f32
  logits;
* every GATConv is ``vg_hgat_lin_att`` (projection + attention projections) and
  ``vg_hgat_fwd`` (edge softmax + gather-sum on f16 rows, half the bytes of the
  f32 scatter kernel), every GraphNorm + ReLU ``vg_graphnorm_fwd_h``;
* the two concatenations of the reference (``models.py:131`` and ``:145``) are
  ONE row buffer ``[enc | x | em | voxel.x | z | 0-pad]``: the encoders write
  their outputs straight into its column slices and the MLP encoder reads its
  input ``[em | voxel.x | z]`` from the same rows, so no concatenation runs;
* the type head stays f32 (``ops.gumbel_head``).

Rows are padded to multiples of 8 halves (16-byte fragments for the MFMA);
pad columns are zero.  Accumulation is f32 everywhere.  Results differ from the
f32 forward by f16 rounding only (``tests/test_half_gpu.py`` states the bounds).
Call ``refresh()`` after the generator's weights change.
"""
from __future__ import annotations

import os
import weakref
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import data as vdata
from . import ops
from ._lib import LIB, check, ptr, stream_handle

# sweep_labels as ONE hipGraph launch per batch (vg_hgen_sweep_graphed: the
# native call captured, an executable graph updated in place); 0: the native
# call launches its kernels directly (vg_hgen_sweep)
_GRAPH = os.environ.get("VGAN_HGEN_GRAPH", "1") == "1"



def _r8(c: int) -> int:
    return (c + 7) // 8 * 8


def _w16(weight: torch.Tensor) -> torch.Tensor:
    """[M, K] f32 -> [M, K rounded up to 8] f16, zero pad columns."""
    m, k = weight.shape
    w = torch.zeros(m, _r8(k), dtype=torch.float16, device=weight.device)
    w[:, :k] = weight.detach()
    return w


class HalfGenerator:
    def __init__(self, generator):
        self.G = generator
        self.trace = None  # a list: the forward appends (name, f32 copy) of every stage (debugging)
        self.refresh()

    def _t(self, name, t, c):
        if self.trace is not None:
            self.trace.append((name, t[:, :c].float().clone()))

    @torch.no_grad()
    def refresh(self) -> None:
        G = self.G
        self._md = None  # the native model descriptor points at the images below
        dev = next(G.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("vgan HIP ops require tensors on a ROCm device (no CPU fallback)")
        self.device = dev
        self.matched = self._mlp_blocks(G.matched_features_encoder)
        self.mlp = self._mlp_blocks(G.mlp_encoder)
        dec = list(G.decoder.children())
        self.decoder = self._mlp_blocks(nn.Sequential(*dec[:-1]))
        head: nn.Linear = dec[-1]
        self.head = (_w16(head.weight), head.bias.detach().float().contiguous(), head.out_features,
                     head.in_features)
        self.gat: List[tuple] = []
        enc = G.encoder
        for b in range(enc.num_blocks):
            conv = getattr(enc, f"module_{4 * b}")
            norm = getattr(enc, f"module_{4 * b + 1}")
            self.gat.append((_w16(conv.lin.weight), conv.att_src.detach().reshape(-1).float().contiguous(),
                             conv.att_dst.detach().reshape(-1).float().contiguous(),
                             conv.bias.detach().float().contiguous(), conv.in_channels, conv.out_channels,
                             float(conv.negative_slope), norm.weight.detach().float().contiguous(),
                             norm.bias.detach().float().contiguous(),
                             norm.mean_scale.detach().float().contiguous(), float(norm.eps)))

    @staticmethod
    def _mlp_blocks(mlp: nn.Module) -> List[tuple]:
        mods = list(mlp.children())
        out = []
        for i in range(0, len(mods), 3):
            lin, ln, act = mods[i:i + 3]
            if not (isinstance(lin, nn.Linear) and isinstance(ln, nn.LayerNorm) and isinstance(act, nn.LeakyReLU)):
                raise TypeError("expected [Linear, LayerNorm, LeakyReLU] blocks")
            out.append((_w16(lin.weight), lin.bias.detach().float().contiguous(),
                        ln.weight.detach().float().contiguous(), ln.bias.detach().float().contiguous(),
                        float(ln.eps), float(act.negative_slope), lin.out_features, lin.in_features))
        return out

    # ----------------------------------------------------------------- layers
    def _run_mlp(self, blocks, a: torch.Tensor, lda: int, k_in: int, rows: int, last_out=None, last_ld=0):
        """The MLP's blocks over ``rows`` rows of ``a`` (stride lda, k_in
        columns); the last block writes into ``last_out`` (stride last_ld) when
        given.  Returns (output, its stride)."""
        s = stream_handle(self.device)
        k = k_in
        for j, (w, b, g, be, eps, slope, m, kin) in enumerate(blocks):
            if _r8(kin) != _r8(k):
                raise ValueError("MLP input width mismatch")
            if j == len(blocks) - 1 and last_out is not None:
                out, ldo = last_out, last_ld
            else:
                out, ldo = torch.empty(rows, _r8(m), dtype=torch.float16, device=self.device), _r8(m)
            check(LIB.vg_hgemm_ln_act(ptr(a), lda, ptr(w), w.shape[1], rows, m, _r8(kin), ptr(b), ptr(g),
                                      ptr(be), eps, slope, ptr(out), ldo, s), "vg_hgemm_ln_act")
            a, lda, k = out, ldo, m
        return a, lda

    @torch.no_grad()
    def logits(self, local_graph, voxel_graph, z: torch.Tensor) -> torch.Tensor:
        """[k * N, 7] f32 logits of the eval forward for z [k, N, Z] (or [1, N, Z])."""
        cfg = self.G.configuration
        prep = vdata.prepared(local_graph, voxel_graph, cfg.NUM_CLASSES)
        dev = self.device
        s = stream_handle(dev)
        n = prep.voxel_x.shape[0]
        kk = z.shape[0] if z.dim() == 3 else 1
        rows = kk * n
        hl = self.matched[-1][6]
        hg = self.mlp[-1][6]
        enc_c = self.gat[-1][5]
        vd = prep.voxel_x.shape[1]
        zd = z.shape[-1]
        # row buffer [enc | x | em | voxel.x | z | pad]  (models.py:145 order)
        o_x, o_em = enc_c, enc_c + hg
        o_vx = o_em + hl
        o_z = o_vx + vd
        width = o_z + zd
        ld = _r8(width)
        buf = torch.empty(rows, ld, dtype=torch.float16, device=dev)
        view = buf.view(kk, n, ld)
        view[:, :, o_vx:o_z] = prep.voxel_x.to(torch.float16)
        view[:, :, o_z:width] = z.reshape(kk, n, zd).to(torch.float16)
        if ld > width:
            buf[:, width:].zero_()
        # program-feature encoder once on N rows, broadcast into every copy
        mx = prep.matched_x
        a0 = torch.zeros(n, _r8(mx.shape[1]), dtype=torch.float16, device=dev)
        a0[:, :mx.shape[1]] = mx
        em, _ = self._run_mlp(self.matched, a0, a0.shape[1], mx.shape[1], n)
        self._t("em", em, hl)
        view[:, :, o_em:o_em + hl] = em[:, :hl]
        # MLP encoder: reads [em | voxel.x | z] in place, writes x into its slice
        self._run_mlp(self.mlp, buf[:, o_em:], ld, width - o_em, rows, last_out=buf[:, o_x:], last_ld=ld)
        self._t("x", buf[:, o_x:], hg)
        # GAT encoder over the stacked block-diagonal graph
        csr = prep.csr if kk == 1 else prep.csr.stacked(kk)
        x, ldx = buf[:, o_x:], ld
        nb = len(self.gat)
        # a block's GraphNorm + ReLU is applied by the next block's projection
        # as it loads its operand (vg_hgat_lin_att_gn) when the statistics come
        # from the aggregation's partials; the last block's is stored (it
        # feeds the decoder's row buffer).  hgen_engine.hip makes the same
        # choices.  pend: (agg, gw, gb, gms, stats, channels) of that GraphNorm
        pend = None
        for b, (w, att_s, att_d, bias, cin, cout, slope, gw, gb, gms, eps) in enumerate(self.gat):
            ldh = _r8(cout)
            h = torch.empty(rows, ldh, dtype=torch.float16, device=dev)
            a_s = torch.empty(rows, dtype=torch.float32, device=dev)
            a_d = torch.empty(rows, dtype=torch.float32, device=dev)
            if pend is not None:
                p_agg, p_w, p_b, p_ms, p_st, p_c = pend
                check(LIB.vg_hgat_lin_att_gn(ptr(p_agg), p_agg.shape[1], ptr(w), w.shape[1], rows, _r8(cin), cout,
                                             ptr(att_s), ptr(att_d), ptr(h), ldh, ptr(a_s), ptr(a_d), ptr(p_w),
                                             ptr(p_b), ptr(p_ms), ptr(p_st), kk, n, p_c, s), "vg_hgat_lin_att_gn")
                pend = None
            else:
                check(LIB.vg_hgat_lin_att(ptr(x), ldx, ptr(w), w.shape[1], rows, _r8(cin), cout, ptr(att_s),
                                          ptr(att_d), ptr(h), ldh, ptr(a_s), ptr(a_d), s), "vg_hgat_lin_att")
            agg = torch.empty_like(h)
            # the GraphNorm's column partials from the aggregation's epilogue
            # when one copy spans a partial block (always, at sweep sizes)
            g = int(LIB.vg_hgat_gnp_rows(rows, ldh))
            gnp = torch.empty(int(LIB.vg_hgat_gnp_floats(rows, ldh)), dtype=torch.float32, device=dev) \
                if 0 < g <= n else None
            if gnp is not None:
                check(LIB.vg_hgat_fwd_gnp(ptr(csr.row_ptr), ptr(csr.col), rows, cout, ldh, ptr(h), ptr(a_s), ptr(a_d),
                                          ptr(bias), slope, ptr(agg), ldh, n, ptr(gnp), s), "vg_hgat_fwd_gnp")
            else:
                check(LIB.vg_hgat_fwd(ptr(csr.row_ptr), ptr(csr.col), rows, cout, ldh, ptr(h), ptr(a_s), ptr(a_d),
                                      ptr(bias), slope, ptr(agg), ldh, s), "vg_hgat_fwd")
            stats = torch.empty(kk * 2 * cout, dtype=torch.float32, device=dev)
            if gnp is not None and b < nb - 1 and kk <= int(LIB.vg_hgat_gna_max_segments()) \
                    and self.trace is None:
                check(LIB.vg_graphnorm_stats_gnp(kk, n, cout, ptr(gnp), g, ptr(gms), eps, ptr(stats), s),
                      "vg_graphnorm_stats_gnp")
                pend = (agg, gw, gb, gms, stats, cout)
                continue
            if b == nb - 1:
                y, ldy = buf, ld  # the last block writes enc into columns [0, enc_c)
            else:
                y, ldy = torch.empty_like(h), ldh
            if gnp is not None:
                check(LIB.vg_graphnorm_fwd_h_gnp(ptr(agg), ldh, kk, n, cout, ptr(gw), ptr(gb), ptr(gms), eps, ptr(y),
                                                 ldy, ptr(stats), ptr(gnp), g, s), "vg_graphnorm_fwd_h_gnp")
            else:
                ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(kk, n, cout)), dtype=torch.float32, device=dev)
                check(LIB.vg_graphnorm_fwd_h(ptr(agg), ldh, kk, n, cout, ptr(gw), ptr(gb), ptr(gms), eps, ptr(y), ldy,
                                             ptr(stats), ptr(ws), s), "vg_graphnorm_fwd_h")
            x, ldx = y, ldy
            self._t(f"gat{b}", y, cout)
        # decoder over the whole row buffer, f32 logits
        d, ldd = self._run_mlp(self.decoder, buf, ld, width, rows)
        w, bias, m, kin = self.head
        logits = torch.empty(rows, m, dtype=torch.float32, device=dev)
        check(LIB.vg_hgemm(ptr(d), ldd, ptr(w), w.shape[1], rows, m, _r8(kin), ptr(bias), 0, 0.0, ptr(logits), m, 1,
                           s), "vg_hgemm")
        return logits

    # ------------------------------------------------- one native call per batch
    def _native_model(self):
        """The vg_hgen_model of the current weight images (rebuilt by refresh)."""
        from ._lib import VG_HGEN_MAX_BLOCKS, VG_HGEN_MAX_LAYERS, VgHgenModel

        md = self.__dict__.get("_md")
        if md is not None:
            return md
        if max(len(self.matched), len(self.mlp), len(self.decoder)) > VG_HGEN_MAX_LAYERS or \
                len(self.gat) > VG_HGEN_MAX_BLOCKS:
            raise ValueError("generator too deep for vg_hgen_sweep")
        md = VgHgenModel()
        md.n_matched, md.n_mlp, md.n_blocks, md.n_dec = len(self.matched), len(self.mlp), len(self.gat), \
            len(self.decoder)

        def lin(dst, blk):
            w, b, g, be, eps, slope, m, kin = blk
            dst.weight, dst.ldw, dst.bias, dst.gamma, dst.beta = w.data_ptr(), w.shape[1], b.data_ptr(), \
                g.data_ptr(), be.data_ptr()
            dst.eps, dst.slope, dst.in_, dst.out = eps, slope, kin, m

        for dst, src in ((md.matched, self.matched), (md.mlp, self.mlp), (md.dec, self.decoder)):
            for i, blk in enumerate(src):
                lin(dst[i], blk)
        w, bias, m, kin = self.head
        md.head.weight, md.head.ldw, md.head.bias, md.head.in_, md.head.out = w.data_ptr(), w.shape[1], \
            bias.data_ptr(), kin, m
        for i, (w, att_s, att_d, bias, cin, cout, slope, gw, gb, gms, eps) in enumerate(self.gat):
            d = md.block[i]
            d.lin_weight, d.ldw, d.att_src, d.att_dst, d.bias, d.slope = w.data_ptr(), w.shape[1], att_s.data_ptr(), \
                att_d.data_ptr(), bias.data_ptr(), slope
            d.gn_weight, d.gn_bias, d.gn_mean_scale, d.gn_eps, d.in_, d.out = gw.data_ptr(), gb.data_ptr(), \
                gms.data_ptr(), eps, cin, cout
        self._md = md
        return md

    @torch.no_grad()
    def sweep_labels(self, local_graph, voxel_graph, copies: int, taus: torch.Tensor,
                     logits: Optional[torch.Tensor] = None, graph: Optional[bool] = None) -> torch.Tensor:
        """InferenceSweep._forward on this f16 generator as ONE native call
        (vg_hgen_sweep): RNG.reset(), z for ``copies`` stacked copies, the
        forward, Exp(1) noise, the Gumbel head at ``taus`` [copies] and the
        argmax -- the same kernels in the same order as ``__call__`` preceded
        by the reset and z draw, so the [copies, N] int8 labels are
        bit-identical to that path's.  ``logits`` [copies * N, classes] f32
        receives the logits when given.  ``graph`` (default VGAN_HGEN_GRAPH):
        the call captured into a hipGraph and launched as one
        (vg_hgen_sweep_graphed), unless the stream is already capturing."""
        import ctypes

        from ._lib import LIB, VgHgenBatch

        G = self.G
        cfg = G.configuration
        prep = vdata.prepared(local_graph, voxel_graph, cfg.NUM_CLASSES)
        dev = self.device
        rng = G.rng
        if rng.mode != "device":
            raise ValueError("vg_hgen_sweep draws z and the noise on the device (RNG mode 'device')")
        had = dict(rng._iters)
        ctrs = rng.reset(defer=True)
        for t in ctrs:  # counters of other devices advance as RNG.reset would
            if t.device != dev:
                t.add_(1)
        it = rng._iter(dev)
        advance = 1 if any(t.device == dev for t in had.values()) else 0
        salt0 = rng._salt
        rng._salt = salt0 + 2  # z (RNG.normal) and the Gumbel noise (RNG.exponential)
        vx, mx = prep.voxel_x.contiguous(), prep.matched_x.contiguous()
        csr = prep.csr
        n = int(vx.shape[0])
        for name, t in (("taus", taus), ("voxel_x", vx), ("matched_x", mx), ("csr.row_ptr", csr.row_ptr),
                        ("csr.col", csr.col)):
            if t.device != dev:  # raw pointers go to device kernels: a host or other-device tensor is refused
                raise ValueError(f"sweep_labels: {name} is on {t.device}, the generator on {dev}")
        tt = taus.reshape(-1).to(torch.float32).contiguous()
        if tt.numel() != copies:
            raise ValueError("one temperature per stacked copy")
        bt = VgHgenBatch()
        bt.n, bt.copies, bt.voxel_dim, bt.matched_dim, bt.z_dim, bt.num_edges = n, int(copies), vx.shape[1], \
            mx.shape[1], int(cfg.Z_DIM), csr.num_edges
        bt.voxel_x, bt.matched_x, bt.row_ptr, bt.col, bt.taus = vx.data_ptr(), mx.data_ptr(), \
            csr.row_ptr.data_ptr(), csr.col.data_ptr(), tt.data_ptr()
        bt.seed, bt.iter, bt.advance_iter = int(rng.seed) & ((1 << 64) - 1), it.data_ptr(), advance
        bt.z_salt, bt.noise_salt = 0x40000000 | (salt0 + 1), 0x40000000 | (salt0 + 2)
        md = self._native_model()
        need = int(LIB.vg_hgen_arena_bytes(ctypes.byref(md), ctypes.byref(bt)))
        if need < 0:
            raise ValueError(f"vg_hgen_arena_bytes: {need}")
        arena = self.__dict__.get("_arena")
        if arena is None or arena.numel() < need:
            # earlier arenas stay alive: a captured sweep graph may still replay on them
            if arena is not None:
                self.__dict__.setdefault("_old_arenas", []).append(arena)
            arena = self._arena = torch.empty(need + need // 4, dtype=torch.uint8, device=dev)
        labels = torch.empty(copies, n, dtype=torch.int8, device=dev)
        if logits is not None and (logits.dtype != torch.float32 or not logits.is_contiguous() or
                                   logits.numel() != copies * n * self.head[2]):
            raise ValueError("logits must be a contiguous f32 [copies * N, classes] tensor")
        lg = None if logits is None else logits.data_ptr()
        # the generator's device is current for the native calls: the graph
        # handle's capture stream belongs to the device current at its creation
        with torch.cuda.device(dev):
            if (_GRAPH if graph is None else graph) and not torch.cuda.is_current_stream_capturing():
                check(LIB.vg_hgen_sweep_graphed(self._graph_handle(), ctypes.byref(md), ctypes.byref(bt),
                                                arena.data_ptr(), arena.numel(), labels.data_ptr(), lg,
                                                stream_handle(dev)), "vg_hgen_sweep_graphed")
            else:
                check(LIB.vg_hgen_sweep(ctypes.byref(md), ctypes.byref(bt), arena.data_ptr(), arena.numel(),
                                        labels.data_ptr(), lg, stream_handle(dev)), "vg_hgen_sweep")
        return labels

    def _graph_handle(self) -> int:
        """The two executable graphs of vg_hgen_sweep_graphed, destroyed with
        this object (after their last launches complete)."""
        h = self.__dict__.get("_hgraph")
        if h is None:
            with torch.cuda.device(self.device):  # the capture stream is made on the current device
                h = LIB.vg_hgen_graph_create()
            if not h:
                raise RuntimeError("vg_hgen_graph_create failed")
            self._hgraph = h
            weakref.finalize(self, LIB.vg_hgen_graph_destroy, h)
        return h

    def graph_stats(self) -> Tuple[int, int]:
        """(instantiations, in-place updates) of the graphed sweep so far."""
        import ctypes

        h = self.__dict__.get("_hgraph")
        if h is None:
            return 0, 0
        a, b = ctypes.c_int32(0), ctypes.c_int32(0)
        check(LIB.vg_hgen_graph_stats(h, ctypes.byref(a), ctypes.byref(b)), "vg_hgen_graph_stats")
        return a.value, b.value

    @torch.no_grad()
    def __call__(self, local_graph, voxel_graph, z: torch.Tensor, noise: Optional[torch.Tensor] = None,
                 tau=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(logits, label_hard, label_soft) like ``VoxelGNNGenerator.forward`` in
        eval mode; [k, N, 7] for a stacked z [k, N, Z]."""
        logits = self.logits(local_graph, voxel_graph, z)
        if noise is None:
            noise = self.G.rng.exponential(logits.shape, logits.device)
        tau = self.G.tau if tau is None else tau
        hard, soft = ops.gumbel_head(logits, noise.reshape(logits.shape), tau)
        if z.dim() == 3 and z.shape[0] > 1:
            k = z.shape[0]
            return logits.view(k, -1, logits.shape[1]), hard.view(k, -1, hard.shape[1]), soft.view(k, -1, soft.shape[1])
        return logits, hard, soft
