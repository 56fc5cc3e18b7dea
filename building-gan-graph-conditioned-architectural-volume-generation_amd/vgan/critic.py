"""Explicit WGAN-GP critic: loss and discriminator gradient without autograd.

Replaces ``_compute_discriminator_loss(...)`` followed by ``d_loss.backward()``
(``trainer.py:291-332``, ``:476-479``): D(real), D(fake), the gradient penalty
on D(eps*real + (1-eps)*soft) with ``create_graph=True``, and the double
backward through it.  Autograd runs that as ~2,000 small kernels per critic
iteration; here it is ~250 launches of fused HIP kernels in four passes over
the discriminator's op chain x_k = f_k(x_{k-1}; theta_k):

  A  one stacked forward of the real / fake / mix copies ([3N, C] tensors, a
     block-diagonal CSR, per-copy GraphNorm statistics);
  B  input VJP of the mix copy with seed 1 -> g = dD/dlabel, the penalty and
     its seed u0 = dGP/dg (vg_gp_head);
  C  tangent sweep u_k = J_k u_{k-1} from u0 with the second-order terms of
     Q_k = <d_k, J_k u_{k-1}> (d_k from pass B): dQ_k/dtheta_k into the
     gradient, dQ_k/dx_{k-1} kept as an injection (vg_gat_jvp2,
     vg_graphnorm_jvp2, and for the linear layers W_bar += d^T u);
  D  one stacked VJP of all copies (seeds -1/N real, +1/N fake, 0 mix) with
     the injections added to the mix copy's adjoints (vg_gat_bwd_ex,
     vg_graphnorm_bwd_seg), parameter gradients accumulated.

The pass structure is checked against plain double backward in float64 on
the CPU (tests/test_critic_ref_cpu.py); every kernel against autograd units
and the whole engine against the reference's CPU critic on the GPU.

Gradients are ACCUMULATED into the discriminator's ``.grad`` (views into its
flat gradient buffer), like ``backward()``; the caller zeroes them first.
Randomness is drawn in the reference's order (dropout masks of D(real), of
D(fake), eps, masks of D(mix)) in host / fixed RNG modes; device mode draws
each layer's stacked mask in one call.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn

from . import data as vdata
from ._lib import LIB, check, ptr, stream_handle, sync_counter

ACT_NONE, ACT_RELU, ACT_MASK = 0, 1, 3


def _f(*shape, dev):
    return torch.empty(*shape, dtype=torch.float32, device=dev)


def _off(t: torch.Tensor, floats: int):
    """Device pointer `floats` elements into t."""
    import ctypes

    return ctypes.c_void_p(t.data_ptr() + 4 * floats)


class CriticEngine:
    def __init__(self, discriminator: nn.Module, configuration):
        D = discriminator
        if not getattr(configuration, "USE_WGANGP", True):
            raise ValueError("the critic engine implements the WGAN-GP loss (USE_WGANGP=True)")
        self.D = D
        self.lam = float(configuration.LAMBDA_GP)
        self.n_classes = int(configuration.NUM_CLASSES)
        self.mlp: List[nn.Linear] = [m for m in D.mlp_encoder if isinstance(m, nn.Linear)]
        self.dec: List[nn.Linear] = [m for m in D.decoder if isinstance(m, nn.Linear)]
        enc = D.encoder
        self.blocks = [(getattr(enc, f"module_{4 * b}"), getattr(enc, f"module_{4 * b + 1}"))
                       for b in range(enc.num_blocks)]
        self.dropout = float(enc.dropout)
        self._consts = {}

    # ---------------------------------------------------------- helpers
    def _const(self, key, make):
        t = self._consts.get(key)
        if t is None:
            t = self._consts[key] = make()
        return t

    def _keeps(self, rng, n: int, dev, training: bool):
        """Dropout multipliers [3N, C_b] per block and eps [N, 1], drawn in the
        reference's order (D(real) masks, D(fake) masks, eps, D(mix) masks)."""
        widths = [conv.out_channels for conv, _ in self.blocks]
        if not training:
            return [None] * len(widths), rng.uniform((n, 1), dev)
        if rng.mode == "device":  # DropSpecs: drawn inside the GraphNorm kernel
            keeps = [rng.keep_mask((3 * n, c), self.dropout, dev) for c in widths]
            return keeps, rng.uniform((n, 1), dev)
        real = [rng.keep_mask((n, c), self.dropout, dev) for c in widths]
        fake = [rng.keep_mask((n, c), self.dropout, dev) for c in widths]
        eps = rng.uniform((n, 1), dev)
        mix = [rng.keep_mask((n, c), self.dropout, dev) for c in widths]
        return [torch.cat([a, b, c]) for a, b, c in zip(real, fake, mix)], eps

    @staticmethod
    def _gemm(st, A, lda, B, ldb, bt, C, ldc, n, m, k, bias=None, act=ACT_NONE, aux=None, ldaux=0):
        check(LIB.vg_gemm(A, lda, B, ldb, bt, bias, act, aux, ldaux, C, ldc, n, m, k, st), "vg_gemm")

    @staticmethod
    def _gemm_tn(st, dev, A, lda, B, ldb, n, m, k, C, ldc, db=None):
        ws = _f(max(1, int(LIB.vg_gemm_tn_ws_floats(n, m, k))), dev=dev)
        check(LIB.vg_gemm_tn(A, lda, B, ldb, n, m, k, C, ldc, db, 1, ptr(ws), st), "vg_gemm_tn")

    # ------------------------------------------------------------ engine
    def loss_and_grad(self, local_graph, voxel_graph, label_hard, label_soft, rng) -> torch.Tensor:
        """d_loss (device scalar) of trainer.py:318-332; D's parameter gradients
        are added to their .grad."""
        D = self.D
        prep = vdata.prepared(local_graph, voxel_graph, self.n_classes)
        mvx, real = prep.matched_voxel_x, prep.onehot_f
        n, F = mvx.shape
        K = self.n_classes
        hard = label_hard.reshape(n, K)
        soft = label_soft.reshape(n, K)
        if hard.dtype != torch.float32:
            hard = hard.float()
        hard, soft = hard.contiguous(), soft.contiguous()
        dev = mvx.device
        st = stream_handle(dev)
        sy = sync_counter(dev)
        R, W0 = 3 * n, F + K
        csr = prep.csr
        csr3 = csr.stacked(3)
        E = csr.num_edges
        for p in D.parameters():
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        keeps, eps = self._keeps(rng, n, dev, D.training)
        eps = eps.reshape(n).contiguous()

        # ---------------------------------------------------------- pass A
        X0 = _f(R, W0, dev=dev)
        check(LIB.vg_critic_input(ptr(mvx), n, F, ptr(real), ptr(hard), ptr(soft), ptr(eps), K, ptr(X0), st),
              "vg_critic_input")
        mlp_out = []
        x, xw = X0, W0
        for lin in self.mlp:
            o = lin.out_features
            y = _f(R, o, dev=dev)
            self._gemm(st, ptr(x), xw, ptr(lin.weight), xw, 1, ptr(y), o, R, o, xw, ptr(lin.bias), ACT_RELU)
            mlp_out.append(y)
            x, xw = y, o
        blk = []
        for (conv, norm), keep in zip(self.blocks, keeps):
            c = conv.out_channels
            H = _f(R, c, dev=dev)
            self._gemm(st, ptr(x), xw, ptr(conv.lin.weight), xw, 1, ptr(H), c, R, c, xw)
            O = _f(R, c, dev=dev)
            alpha, a_s, a_d = _f(3 * E, dev=dev), _f(R, dev=dev), _f(R, dev=dev)
            check(LIB.vg_gat_fwd(ptr(csr3.row_ptr), ptr(csr3.col), R, c, ptr(H), ptr(conv.att_src),
                                 ptr(conv.att_dst), ptr(conv.bias), float(conv.negative_slope), ptr(O), ptr(alpha),
                                 ptr(a_s), ptr(a_d), st), "vg_gat_fwd")
            Y, stats = _f(R, c, dev=dev), _f(3 * 2 * c, dev=dev)
            ws = _f(int(LIB.vg_graphnorm_seg_ws_floats(3, n, c)), dev=dev)
            if keep is not None and not isinstance(keep, torch.Tensor):  # DropSpec
                spec, keep = keep, _f(R, c, dev=dev)
                check(LIB.vg_graphnorm_fwd_drop(ptr(O), 3, n, c, ptr(norm.weight), ptr(norm.bias),
                                                ptr(norm.mean_scale), float(spec.p), int(spec.seed), ptr(spec.iter),
                                                int(spec.salt) & 0xFFFFFFFF, float(norm.eps), ptr(Y), ptr(keep),
                                                ptr(stats), ptr(ws), sy, st), "vg_graphnorm_fwd_drop")
            else:
                check(LIB.vg_graphnorm_fwd_seg(ptr(O), 3, n, c, ptr(norm.weight), ptr(norm.bias),
                                               ptr(norm.mean_scale), ptr(keep), float(norm.eps), ptr(Y), ptr(stats),
                                               ptr(ws), sy, st), "vg_graphnorm_fwd_seg")
            blk.append(dict(X=x, xw=xw, H=H, O=O, alpha=alpha, a_s=a_s, a_d=a_d, Y=Y, stats=stats, keep=keep, c=c))
            x, xw = Y, c
        dec_out = []
        for i, lin in enumerate(self.dec):
            o = lin.out_features
            z = _f(R, o, dev=dev)
            act = ACT_NONE if i == len(self.dec) - 1 else ACT_RELU
            self._gemm(st, ptr(x), xw, ptr(lin.weight), xw, 1, ptr(z), o, R, o, xw, ptr(lin.bias), act)
            dec_out.append(z)
            x, xw = z, o
        scores = dec_out[-1]
        if scores.shape[1] != 1:
            raise ValueError("the critic must output one score per node")

        mrow = 2 * n  # first row of the mix copy

        def mix(t: torch.Tensor, width: int):
            return _off(t, mrow * width)

        # ---------------------------------------------------------- pass B
        ones = self._const(("ones", n), lambda: torch.ones(n, 1, dtype=torch.float32, device=dev))
        nd = len(self.dec)
        p_dec: List[Optional[torch.Tensor]] = [None] * nd
        adj, aw = ones, 1
        for i in range(nd - 1, 0, -1):
            Wt = self.dec[i].weight
            m = Wt.shape[1]
            a = _f(n, m, dev=dev)
            self._gemm(st, ptr(adj), aw, ptr(Wt), m, 0, ptr(a), m, n, m, aw, None, ACT_MASK, mix(dec_out[i - 1], m), m)
            p_dec[i - 1] = a
            adj, aw = a, m
        W = self.dec[0].weight
        dY = _f(n, W.shape[1], dev=dev)
        self._gemm(st, ptr(adj), aw, ptr(W), W.shape[1], 0, ptr(dY), W.shape[1], n, W.shape[1], aw)
        nb = len(self.blocks)
        dY_b, dO_b, dH_b = [None] * nb, [None] * nb, [None] * nb
        p_mlp: List[Optional[torch.Tensor]] = [None] * len(self.mlp)
        for b in range(nb - 1, -1, -1):
            (conv, norm), B = self.blocks[b], blk[b]
            c = B["c"]
            dY_b[b] = dY
            dO = _f(n, c, dev=dev)
            ws = _f(int(LIB.vg_graphnorm_seg_ws_floats(1, n, c)), dev=dev)
            check(LIB.vg_graphnorm_bwd_seg(mix(B["O"], c), 1, n, c, ptr(norm.weight), ptr(norm.bias),
                                           ptr(norm.mean_scale), mix(B["keep"], c) if B["keep"] is not None else None,
                                           float(norm.eps), _off(B["stats"], 2 * 2 * c), ptr(dY), ptr(dO), None, None,
                                           None, 0, None, 0, ptr(ws), sy, st), "vg_graphnorm_bwd_seg")
            dH = _f(n, c, dev=dev)
            ws = _f(int(LIB.vg_gat_bwd_ws_floats(n, E, c)), dev=dev)
            check(LIB.vg_gat_bwd_ex(ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot),
                                    ptr(csr.csc_dst), n, E, c, mix(B["H"], c), ptr(conv.att_src), ptr(conv.att_dst),
                                    _off(B["a_s"], mrow), _off(B["a_d"], mrow), _off(B["alpha"], 2 * E), ptr(dO),
                                    float(conv.negative_slope), ptr(dH), None, None, None, 0, None, 0, ptr(ws), st),
                  "vg_gat_bwd_ex")
            dO_b[b], dH_b[b] = dO, dH
            cin = B["xw"]
            dX = _f(n, cin, dev=dev)
            if b > 0:
                self._gemm(st, ptr(dH), c, ptr(conv.lin.weight), cin, 0, ptr(dX), cin, n, cin, c)
                dY = dX
            else:
                self._gemm(st, ptr(dH), c, ptr(conv.lin.weight), cin, 0, ptr(dX), cin, n, cin, c, None, ACT_MASK,
                           mix(mlp_out[-1], cin), cin)
                p_mlp[-1] = dX
        for i in range(len(self.mlp) - 1, 0, -1):
            Wt = self.mlp[i].weight
            m = Wt.shape[1]
            a = _f(n, m, dev=dev)
            self._gemm(st, ptr(p_mlp[i]), Wt.shape[0], ptr(Wt), m, 0, ptr(a), m, n, m, Wt.shape[0], None, ACT_MASK,
                       mix(mlp_out[i - 1], m), m)
            p_mlp[i - 1] = a
        W = self.mlp[0].weight
        hd = W.shape[0]
        g = _f(n, K, dev=dev)
        self._gemm(st, ptr(p_mlp[0]), hd, _off(W, F), W0, 0, ptr(g), K, n, K, hd)
        u0, out = _f(n, K, dev=dev), _f(2, dev=dev)
        check(LIB.vg_gp_head(ptr(g), n, K, ptr(scores), self.lam, ptr(u0), ptr(out), st), "vg_gp_head")

        # ---------------------------------------------------------- pass C
        uY = _f(n, hd, dev=dev)
        self._gemm(st, ptr(u0), K, _off(W, F), W0, 1, ptr(uY), hd, n, hd, K, None, ACT_MASK, mix(mlp_out[0], hd), hd)
        self._gemm_tn(st, dev, ptr(p_mlp[0]), hd, ptr(u0), K, n, hd, K, _off(W.grad, F), W0)
        uw = hd
        for i in range(1, len(self.mlp)):
            lin = self.mlp[i]
            o = lin.out_features
            un = _f(n, o, dev=dev)
            self._gemm(st, ptr(uY), uw, ptr(lin.weight), uw, 1, ptr(un), o, n, o, uw, None, ACT_MASK,
                       mix(mlp_out[i], o), o)
            self._gemm_tn(st, dev, ptr(p_mlp[i]), o, ptr(uY), uw, n, o, uw, ptr(lin.weight.grad), uw)
            uY, uw = un, o
        hinj_b, oinj_b = [None] * nb, [None] * nb
        for b in range(nb):
            (conv, norm), B = self.blocks[b], blk[b]
            c, cin = B["c"], B["xw"]
            uH = _f(n, c, dev=dev)
            self._gemm(st, ptr(uY), cin, ptr(conv.lin.weight), cin, 1, ptr(uH), c, n, c, cin)
            self._gemm_tn(st, dev, ptr(dH_b[b]), c, ptr(uY), cin, n, c, cin, ptr(conv.lin.weight.grad), cin)
            uO, hinj = _f(n, c, dev=dev), _f(n, c, dev=dev)
            ws = _f(int(LIB.vg_gat_jvp2_ws_floats(n, E, c)), dev=dev)
            check(LIB.vg_gat_jvp2(ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot),
                                  ptr(csr.csc_dst), n, E, c, mix(B["H"], c), ptr(uH), ptr(dO_b[b]), ptr(conv.att_src),
                                  ptr(conv.att_dst), _off(B["a_s"], mrow), _off(B["a_d"], mrow),
                                  _off(B["alpha"], 2 * E), float(conv.negative_slope), ptr(uO), ptr(hinj),
                                  ptr(conv.att_src.grad), ptr(conv.att_dst.grad), ptr(ws), st), "vg_gat_jvp2")
            uYn, oinj = _f(n, c, dev=dev), _f(n, c, dev=dev)
            ws = _f(int(LIB.vg_graphnorm_seg_ws_floats(1, n, c)), dev=dev)
            check(LIB.vg_graphnorm_jvp2(mix(B["O"], c), n, c, ptr(norm.weight), ptr(norm.bias), ptr(norm.mean_scale),
                                        mix(B["keep"], c) if B["keep"] is not None else None, float(norm.eps),
                                        _off(B["stats"], 2 * 2 * c), ptr(uO), ptr(dY_b[b]), ptr(uYn), ptr(oinj),
                                        ptr(norm.weight.grad), ptr(norm.mean_scale.grad), ptr(ws), sy, st),
                  "vg_graphnorm_jvp2")
            hinj_b[b], oinj_b[b] = hinj, oinj
            uY, uw = uYn, c
        for i, lin in enumerate(self.dec):
            o = lin.out_features
            if i < nd - 1:
                un = _f(n, o, dev=dev)
                self._gemm(st, ptr(uY), uw, ptr(lin.weight), uw, 1, ptr(un), o, n, o, uw, None, ACT_MASK,
                           mix(dec_out[i], o), o)
                self._gemm_tn(st, dev, ptr(p_dec[i]), o, ptr(uY), uw, n, o, uw, ptr(lin.weight.grad), uw)
                uY, uw = un, o
            else:
                self._gemm_tn(st, dev, ptr(ones), 1, ptr(uY), uw, n, 1, uw, ptr(lin.weight.grad), uw)

        # ---------------------------------------------------------- pass D
        def make_seeds():
            s = torch.zeros(R, 1, dtype=torch.float32, device=dev)
            s[:n] = -1.0 / n
            s[n:2 * n] = 1.0 / n
            return s

        seeds = self._const(("seeds", n), make_seeds)
        dec_in = [blk[-1]["Y"] if blk else mlp_out[-1]] + dec_out[:-1]
        dec_in_w = [self.dec[0].in_features] + [l.out_features for l in self.dec[:-1]]
        adj, aw = seeds, 1
        for i in range(nd - 1, -1, -1):
            lin = self.dec[i]
            self._gemm_tn(st, dev, ptr(adj), aw, ptr(dec_in[i]), dec_in_w[i], R, aw, dec_in_w[i], ptr(lin.weight.grad),
                          dec_in_w[i], ptr(lin.bias.grad))
            m = dec_in_w[i]
            a = _f(R, m, dev=dev)
            if i > 0:
                self._gemm(st, ptr(adj), aw, ptr(lin.weight), m, 0, ptr(a), m, R, m, aw, None, ACT_MASK,
                           ptr(dec_out[i - 1]), m)
            else:
                self._gemm(st, ptr(adj), aw, ptr(lin.weight), m, 0, ptr(a), m, R, m, aw)
            adj, aw = a, m
        dY = adj
        for b in range(nb - 1, -1, -1):
            (conv, norm), B = self.blocks[b], blk[b]
            c, cin = B["c"], B["xw"]
            dO = _f(R, c, dev=dev)
            ws = _f(int(LIB.vg_graphnorm_seg_ws_floats(3, n, c)), dev=dev)
            check(LIB.vg_graphnorm_bwd_seg(ptr(B["O"]), 3, n, c, ptr(norm.weight), ptr(norm.bias),
                                           ptr(norm.mean_scale), ptr(B["keep"]), float(norm.eps), ptr(B["stats"]),
                                           ptr(dY), ptr(dO), ptr(norm.weight.grad), ptr(norm.bias.grad),
                                           ptr(norm.mean_scale.grad), 1, ptr(oinj_b[b]), mrow * c, ptr(ws), sy, st),
                  "vg_graphnorm_bwd_seg")
            dH = _f(R, c, dev=dev)
            ws = _f(int(LIB.vg_gat_bwd_ws_floats(R, 3 * E, c)), dev=dev)
            check(LIB.vg_gat_bwd_ex(ptr(csr3.row_ptr), ptr(csr3.col), ptr(csr3.csc_ptr), ptr(csr3.csc_slot),
                                    ptr(csr3.csc_dst), R, 3 * E, c, ptr(B["H"]), ptr(conv.att_src), ptr(conv.att_dst),
                                    ptr(B["a_s"]), ptr(B["a_d"]), ptr(B["alpha"]), ptr(dO), float(conv.negative_slope),
                                    ptr(dH), ptr(conv.att_src.grad), ptr(conv.att_dst.grad), ptr(conv.bias.grad), 1,
                                    ptr(hinj_b[b]), mrow, ptr(ws), st), "vg_gat_bwd_ex")
            self._gemm_tn(st, dev, ptr(dH), c, ptr(B["X"]), cin, R, c, cin, ptr(conv.lin.weight.grad), cin)
            dX = _f(R, cin, dev=dev)
            if b > 0:
                self._gemm(st, ptr(dH), c, ptr(conv.lin.weight), cin, 0, ptr(dX), cin, R, cin, c)
            else:
                self._gemm(st, ptr(dH), c, ptr(conv.lin.weight), cin, 0, ptr(dX), cin, R, cin, c, None, ACT_MASK,
                           ptr(mlp_out[-1]), cin)
            dY = dX
        pm = dY
        for i in range(len(self.mlp) - 1, -1, -1):
            lin = self.mlp[i]
            o, m = lin.out_features, lin.in_features
            xin = X0 if i == 0 else mlp_out[i - 1]
            self._gemm_tn(st, dev, ptr(pm), o, ptr(xin), m, R, o, m, ptr(lin.weight.grad), m, ptr(lin.bias.grad))
            if i > 0:
                a = _f(R, m, dev=dev)
                self._gemm(st, ptr(pm), o, ptr(lin.weight), m, 0, ptr(a), m, R, m, o, None, ACT_MASK,
                           ptr(mlp_out[i - 1]), m)
                pm = a
        self.last_gp = out[1]
        return out[0]
