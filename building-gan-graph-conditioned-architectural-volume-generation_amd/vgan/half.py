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

from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import data as vdata
from . import ops
from ._lib import LIB, check, ptr, stream_handle


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
        for b, (w, att_s, att_d, bias, cin, cout, slope, gw, gb, gms, eps) in enumerate(self.gat):
            ldh = _r8(cout)
            h = torch.empty(rows, ldh, dtype=torch.float16, device=dev)
            a_s = torch.empty(rows, dtype=torch.float32, device=dev)
            a_d = torch.empty(rows, dtype=torch.float32, device=dev)
            check(LIB.vg_hgat_lin_att(ptr(x), ldx, ptr(w), w.shape[1], rows, _r8(cin), cout, ptr(att_s),
                                      ptr(att_d), ptr(h), ldh, ptr(a_s), ptr(a_d), s), "vg_hgat_lin_att")
            agg = torch.empty_like(h)
            check(LIB.vg_hgat_fwd(ptr(csr.row_ptr), ptr(csr.col), rows, cout, ldh, ptr(h), ptr(a_s), ptr(a_d),
                                  ptr(bias), slope, ptr(agg), ldh, s), "vg_hgat_fwd")
            if b == nb - 1:
                y, ldy = buf, ld  # the last block writes enc into columns [0, enc_c)
            else:
                y, ldy = torch.empty_like(h), ldh
            stats = torch.empty(kk * 2 * cout, dtype=torch.float32, device=dev)
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
