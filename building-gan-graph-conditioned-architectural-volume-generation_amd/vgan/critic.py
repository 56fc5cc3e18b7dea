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

import ctypes
import os

import torch
import torch.nn as nn

from . import data as vdata
from . import ops
from ._lib import (_GN_ROWS, LIB, FoldCollector, VgGnApply, VgGnBwdIn, VgGnJvp, check, dense, gemm_precision,
                   linear_chain, ptr, stream_handle, sync_counter)
from . import _lib

ACT_NONE, ACT_RELU, ACT_MASK, ACT_ADD = 0, 1, 3, 4  # vg_gemm act codes (include/vgan.h)
_CHAIN_TANGENT = os.environ.get("VGAN_CHAIN_TANGENT", "1") == "1"
# VGAN_GN_FUSE=0: the GraphNorm backward's column partials in their own pass
# instead of the epilogue of the GEMM producing its g_y (A/B knob)
_GN_FUSE = os.environ.get("VGAN_GN_FUSE", "1") == "1"
# VGAN_NATIVE_CRITIC=0: every critic iteration through the Python engine below
# instead of vg_critic_loss_and_grad (the same launches issued from C++,
# bit-identical; include/vgan.h) -- A/B and parity knob
_NATIVE = os.environ.get("VGAN_NATIVE_CRITIC", "1") == "1"


def _f(*shape, dev):
    return torch.empty(*shape, dtype=torch.float32, device=dev)


def _off(t: torch.Tensor, floats: int):
    """Device pointer `floats` elements into t."""
    return t.data_ptr() + 4 * floats


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

    def prepare_batch(self, prep) -> None:
        """Build this batch's constants (the adjoint seeds of every critic
        iteration) and the stacked graph now, outside any capture -- and size
        the native engine's arena for it (a capture cannot grow it)."""
        n = prep.matched_voxel_x.shape[0]
        self._seeds(prep)
        prep.csr.stacked(3).ell()
        if self._native_config_ok(n):
            model = self._native_model()
            if model is not None:
                batch = self._native_batch(prep, None, None, None, None)
                if batch is not None:
                    self._arena_for(model, batch, prep.matched_voxel_x.device)

    @staticmethod
    def _seeds(prep) -> torch.Tensor:
        """The batch's adjoint seeds [4N, 1]: -1/N real | +1/N fake | 0 mix |
        1 pass-B seed (built once per batch)."""
        s_ = prep.consts.get("critic_seeds4")
        if s_ is None:
            n = prep.matched_voxel_x.shape[0]
            s_ = torch.zeros(4 * n, 1, dtype=torch.float32, device=prep.matched_voxel_x.device)
            s_[:n] = -1.0 / n
            s_[n:2 * n] = 1.0 / n
            s_[3 * n:] = 1.0
            prep.consts["critic_seeds4"] = s_
        return s_

    # --------------------------------------------------- native engine
    # vg_critic_loss_and_grad issues loss_and_grad's launches from C++ (same
    # kernels, order and arguments: bit-identical) with every temporary in
    # one arena: ~1-2 us of host time per launch instead of ~10.  Used when
    # the configuration is loss_and_grad's default one (the knobs below at
    # their defaults, device-drawn dropout and eps, n >= 64); anything else
    # runs the Python engine.
    def _native_config_ok(self, n: int) -> bool:
        return (_NATIVE and _GN_FUSE and n >= 64 and _CHAIN_TANGENT and _lib._GN_ROWS and not _lib._GN_APPLY_GEMM
                and not _lib._GN_JVP_FUSE and not _lib._JVP_GROUP and _lib._TN_GROUP and _lib._CHAIN
                and not _lib._LAST_BLOCK and ops._GN_FWD_FUSE and self.D.training
                and max(len(self.mlp), len(self.blocks), len(self.dec)) <= _lib.VG_CRITIC_MAX_LAYERS)

    def _native_model(self):
        """The vg_critic_model of D's parameters and gradient views (rebuilt
        when any of their addresses changes), or None."""
        params = self.__dict__.get("_params")
        if params is None:
            params = self._params = list(self.D.parameters())
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        key = (gemm_precision(),) + tuple(p.data_ptr() for p in params) + tuple(p.grad.data_ptr() for p in params)
        cached = self.__dict__.get("_native_key")
        if cached is not None and cached == key:
            return self._native_md
        m = _lib.VgCriticModel()
        m.n_mlp, m.n_blocks, m.n_dec = len(self.mlp), len(self.blocks), len(self.dec)
        m.bf16 = 1 if gemm_precision() == "bf16" else 0
        m.lambda_gp, m.p_drop = self.lam, self.dropout

        def lin(dst, l):
            dst.weight, dst.bias = l.weight.data_ptr(), l.bias.data_ptr()
            dst.g_weight, dst.g_bias = l.weight.grad.data_ptr(), l.bias.grad.data_ptr()
            dst.in_, dst.out = l.in_features, l.out_features

        for i, l in enumerate(self.mlp):
            lin(m.mlp[i], l)
        for i, l in enumerate(self.dec):
            lin(m.dec[i], l)
        for i, (conv, norm) in enumerate(self.blocks):
            b = m.block[i]
            if getattr(conv.lin, "bias", None) is not None:  # (GATConv's lin has none)
                return None
            b.lin_weight, b.att_src, b.att_dst, b.bias = (conv.lin.weight.data_ptr(), conv.att_src.data_ptr(),
                                                          conv.att_dst.data_ptr(), conv.bias.data_ptr())
            b.g_lin_weight, b.g_att_src, b.g_att_dst, b.g_bias = (conv.lin.weight.grad.data_ptr(),
                                                                  conv.att_src.grad.data_ptr(),
                                                                  conv.att_dst.grad.data_ptr(), conv.bias.grad.data_ptr())
            b.gn_weight, b.gn_bias, b.gn_mean_scale = (norm.weight.data_ptr(), norm.bias.data_ptr(),
                                                       norm.mean_scale.data_ptr())
            b.g_gn_weight, b.g_gn_bias, b.g_gn_mean_scale = (norm.weight.grad.data_ptr(), norm.bias.grad.data_ptr(),
                                                             norm.mean_scale.grad.data_ptr())
            b.gn_eps, b.slope = float(norm.eps), float(conv.negative_slope)
            b.in_, b.out = conv.in_channels, conv.out_channels
        self._native_key, self._native_md = key, m
        return m

    @staticmethod
    def _csr_ref(dst, csr, ell=None, w=0) -> None:
        dst.row_ptr, dst.col = csr.row_ptr.data_ptr(), csr.col.data_ptr()
        dst.csc_ptr, dst.csc_slot, dst.csc_dst = (csr.csc_ptr.data_ptr(), csr.csc_slot.data_ptr(),
                                                  csr.csc_dst.data_ptr())
        dst.ell = ell.data_ptr() if ell is not None else None
        dst.num_nodes, dst.num_edges, dst.ell_width = csr.num_nodes, csr.num_edges, w if ell is not None else 0

    def _native_batch(self, prep, hard, soft, eps, keeps):
        """vg_critic_batch of this batch (labels and draw specs None: sizes only)."""
        mvx = prep.matched_voxel_x
        seeds = self._seeds(prep)
        if mvx.dtype != torch.float32 or not mvx.is_contiguous():
            return None
        b = _lib.VgCriticBatch()
        b.n, b.feat = mvx.shape
        b.classes = self.n_classes
        b.mvx, b.real, b.seeds4 = mvx.data_ptr(), prep.onehot_f.data_ptr(), seeds.data_ptr()
        csr = prep.csr
        csr3 = csr.stacked(3)
        self._csr_ref(b.g1, csr)
        ell3, w3 = csr3.ell()
        self._csr_ref(b.g3, csr3, ell3, w3)
        if hard is not None:
            seed, it, salt = eps
            b.hard, b.soft = hard.data_ptr(), soft.data_ptr()
            b.seed, b.iter, b.eps_salt = seed, it.data_ptr(), salt & 0xFFFFFFFF
            for i, k in enumerate(keeps):
                b.keep_salt[i] = int(k.salt) & 0xFFFFFFFF
            dev = mvx.device
            b.gp_counter = self._const(("gp_counter", dev),
                                       lambda: torch.zeros(1, dtype=torch.int32, device=dev)).data_ptr()
        return b

    def _arena_for(self, model, batch, dev):
        """(arena tensor, floats) holding the native engine's temporaries for
        this batch, grown outside a capture (grown 25 % ahead); a replaced
        arena is kept alive, since recorded graphs may still reference it.
        None when it is too small and a capture is running."""
        need = int(LIB.vg_critic_arena_floats(ctypes.byref(model), ctypes.byref(batch)))
        if need < 0:
            return None
        cur = self.__dict__.get("_arena")
        if cur is not None and cur[1] >= need and cur[0].device == dev:
            return cur
        if torch.cuda.is_current_stream_capturing():
            return None
        floats = (need * 5 // 4 + 63) // 64 * 64
        t = torch.empty(floats + 64, dtype=torch.float32, device=dev)
        off = (-t.data_ptr() % 256) // 4  # 256-byte aligned base
        if cur is not None:
            self.__dict__.setdefault("_old_arenas", []).append(cur)
        self._arena = (t, floats, t.data_ptr() + 4 * off)
        return self._arena

    def _native(self, prep, hard, soft, keeps, eps, dev, st, out=None):
        """loss_and_grad through vg_critic_loss_and_grad, or None (the
        configuration or this batch is not the native engine's).  ``out``: two
        contiguous device floats to write (d_loss, penalty) into."""
        n = prep.matched_voxel_x.shape[0]
        if not self._native_config_ok(n) or isinstance(eps, torch.Tensor) or eps is None:
            return None
        if len(keeps) != len(self.blocks) or any(k is None or isinstance(k, torch.Tensor) for k in keeps):
            return None
        seed, it, _ = eps
        if any(k.seed != seed or k.iter is not it for k in keeps):
            return None
        model = self._native_model()
        if model is None:
            return None
        batch = self._native_batch(prep, hard, soft, eps, keeps)
        if batch is None:
            return None
        arena = self._arena_for(model, batch, dev)
        if arena is None:
            return None
        if out is None or out.numel() != 2 or not out.is_contiguous() or out.dtype != torch.float32 \
                or out.device != dev:
            out = _f(2, dev=dev)
        check(LIB.vg_critic_loss_and_grad(ctypes.byref(model), ctypes.byref(batch), arena[2], arena[1], ptr(out), st),
              "vg_critic_loss_and_grad")
        self.native_calls = self.__dict__.get("native_calls", 0) + 1
        self.last_gp = out[1]
        return out[0]

    def _keeps(self, rng, n: int, dev, training: bool):
        """Dropout multipliers [3N, C_b] per block and eps [N, 1], drawn in the
        reference's order (D(real) masks, D(fake) masks, eps, D(mix) masks)."""
        widths = [conv.out_channels for conv, _ in self.blocks]
        # device mode: eps as (seed, counter, salt), drawn by vg_critic_input_drawn
        # itself -- the same numbers rng.uniform would write, without its launch
        spec = getattr(rng, "uniform_spec", None)  # (stand-in RNGs of the tests have none)
        draw_eps = (lambda: (spec((n, 1), dev) if spec is not None else None) or rng.uniform((n, 1), dev))
        if not training:
            return [None] * len(widths), draw_eps()
        if rng.mode == "device":  # DropSpecs: drawn inside the GraphNorm kernel
            keeps = [rng.keep_mask((3 * n, c), self.dropout, dev) for c in widths]
            return keeps, draw_eps()
        real = [rng.keep_mask((n, c), self.dropout, dev) for c in widths]
        fake = [rng.keep_mask((n, c), self.dropout, dev) for c in widths]
        eps = rng.uniform((n, 1), dev)
        mix = [rng.keep_mask((n, c), self.dropout, dev) for c in widths]
        return [torch.cat([a, b, c]) for a, b, c in zip(real, fake, mix)], eps

    @staticmethod
    def _gemm(st, A, lda, B, ldb, bt, C, ldc, n, m, k, bias=None, act=ACT_NONE, aux=None, ldaux=0):
        check(dense("vg_gemm")(A, lda, B, ldb, bt, bias, act, aux, ldaux, C, ldc, n, m, k, st), "vg_gemm")

    @staticmethod
    def _gemm_tn(folds, st, dev, A, lda, B, ldb, n, m, k, C, ldc, db=None, db_rows=None):
        """Split-K weight gradient; its fold joins the iteration's batched folds."""
        ws = _f(max(1, int(LIB.vg_gemm_tn_ws_floats(n, m, k))), dev=dev)
        # A / B are buffers of loss_and_grad, alive until its folds.flush()
        folds.tn((A, lda, B, ldb, n, m, k, C, ldc, db, n if db_rows is None else db_rows, 1, ptr(ws)), st,
                 keep=(ws,))

    # ------------------------------------------------------------ engine
    def loss_and_grad(self, local_graph, voxel_graph, label_hard, label_soft, rng, out=None) -> torch.Tensor:
        """d_loss (device scalar) of trainer.py:318-332; D's parameter gradients
        are added to their .grad.

        Buffers hold 4N rows: rows [0, 3N) the real / fake / mix copies of pass
        A (activations) and pass D (adjoints); rows [3N, 4N) of an activation
        buffer take pass C's tangent of that activation, rows [3N, 4N) of an
        adjoint buffer pass B's adjoint.  Every linear layer's weight gradient
        -- first order (pass D) plus second order (d_B^T u_C) -- is then ONE
        split-K product over the 4N rows; only the first 3N rows feed the bias
        gradient."""
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
        R, W0, X4 = 3 * n, F + K, 4 * n
        csr = prep.csr
        csr3 = csr.stacked(3)
        E = csr.num_edges
        params = self.__dict__.get("_params")
        if params is None:  # (a module walk per iteration cost ~20 us of host time)
            params = self._params = list(D.parameters())
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        keeps, eps = self._keeps(rng, n, dev, D.training)
        if isinstance(eps, torch.Tensor):
            eps = eps.reshape(n).contiguous()
        else:  # the launches below, issued from C++ (vg_critic_loss_and_grad)
            loss = self._native(prep, hard, soft, keeps, eps, dev, st, out)
            if loss is not None:
                return loss
        nb, nd, nm = len(self.blocks), len(self.dec), len(self.mlp)
        # parameter-gradient folds of passes C and D, run as one batch at the end
        folds = FoldCollector()
        mrow, trow = 2 * n, 3 * n  # first row of the mix copy / of the tangent (or pass-B) rows

        def rows(t: torch.Tensor, r0: int, width: int):
            return _off(t, r0 * width)

        # a tile straddles at most two stacked copies: n >= 64 rows per copy
        fuse_gn = _GN_FUSE and n >= 64

        def gn_inputs(b: int, mix: bool):
            """block b's GraphNorm input, keep and statistics: the mix copy's
            rows (pass B) or all three copies (pass D)"""
            B, c = blk[b], blk[b]["c"]
            x = rows(B["O"], mrow, c) if mix else ptr(B["O"])
            keep = None if B["keep"] is None else (rows(B["keep"], mrow, c) if mix else ptr(B["keep"]))
            stats = _off(B["stats"], 2 * 2 * c) if mix else ptr(B["stats"])
            return x, keep, stats

        def gemm_dy(A, lda, Wt, ldw, out, nrows: int, m: int, k: int, b: int, mix: bool):
            """out [nrows, m] = A Wt, the output gradient of block b's GraphNorm;
            with fuse_gn that backward's column partials come from this GEMM's
            epilogue (returned, for gn_bwd), else None."""
            if not fuse_gn:
                self._gemm(st, A, lda, Wt, ldw, 0, out, m, nrows, m, k)
                return None
            norm = self.blocks[b][1]
            tp = _f(int(LIB.vg_gemm_gn_tpart_floats(nrows, m)), dev=dev)
            x, keep, stats = gn_inputs(b, mix)
            check(dense("vg_gemm_gn_bwd")(A, lda, Wt, ldw, nrows, m, k, out, m, x, keep, n, ptr(norm.weight),
                                          ptr(norm.bias), ptr(norm.mean_scale), float(norm.eps), stats, ptr(tp), st),
                  "vg_gemm_gn_bwd")
            return tp

        def gn_bwd(b: int, mix: bool, tp, g_y, g_x, pgrads: bool, inj=None, inj_off: int = 0):
            """block b's GraphNorm(+ReLU+Dropout) backward: g_x from g_y.
            g_x None: the column sums only -- returns the descriptor with which
            vg_gat_bwd_gn forms g_x in its destination-row pass (and the
            workspace holding the sums)."""
            norm, c = self.blocks[b][1], blk[b]["c"]
            S = 1 if mix else 3
            x, keep, stats = gn_inputs(b, mix)
            ws = _f(int(LIB.vg_graphnorm_seg_ws_floats(S, n, c)), dev=dev)
            pg = (ptr(norm.weight.grad), ptr(norm.bias.grad), ptr(norm.mean_scale.grad)) if pgrads else (None,) * 3
            gx = None if g_x is None else ptr(g_x)
            if tp is not None:
                check(LIB.vg_graphnorm_bwd_seg_tiles(x, S, n, c, ptr(norm.weight), ptr(norm.bias), ptr(norm.mean_scale),
                                                     keep, float(norm.eps), stats, ptr(g_y), ptr(tp), gx, *pg,
                                                     1 if pgrads else 0, inj, inj_off, ptr(ws), st),
                      "vg_graphnorm_bwd_seg_tiles")
            else:
                check(LIB.vg_graphnorm_bwd_seg(x, S, n, c, ptr(norm.weight), ptr(norm.bias), ptr(norm.mean_scale),
                                               keep, float(norm.eps), stats, ptr(g_y), gx, *pg,
                                               1 if pgrads else 0, inj, inj_off, ptr(ws), sy, st),
                      "vg_graphnorm_bwd_seg")
            if g_x is not None:
                return None
            gn = VgGnBwdIn(x=x, keep=keep, g_y=ptr(g_y), inj=inj, weight=ptr(norm.weight), bias=ptr(norm.bias),
                           mean_scale=ptr(norm.mean_scale), stats=stats,
                           sums=_off(ws, int(LIB.vg_graphnorm_bwd_sums_offset(S, c))), eps=float(norm.eps),
                           segments=S, seg_rows=n, inj_offset=inj_off if inj else 0)
            return gn, ws

        # ---------------------------------------------------------- pass A
        X0 = _f(X4, W0, dev=dev)
        if isinstance(eps, torch.Tensor):
            check(LIB.vg_critic_input(ptr(mvx), n, F, ptr(real), ptr(hard), ptr(soft), ptr(eps), K, 4, ptr(X0), st),
                  "vg_critic_input")
        else:
            seed, it, salt = eps
            check(LIB.vg_critic_input_drawn(ptr(mvx), n, F, ptr(real), ptr(hard), ptr(soft), seed, ptr(it), salt, K,
                                            4, ptr(X0), st), "vg_critic_input_drawn")
        mlp_out = []
        x, xw = X0, W0
        for lin in self.mlp:
            o = lin.out_features
            y = _f(X4, o, dev=dev)
            self._gemm(st, ptr(x), xw, ptr(lin.weight), xw, 1, ptr(y), o, R, o, xw, ptr(lin.bias), ACT_RELU)
            mlp_out.append(y)
            x, xw = y, o
        blk = []
        pend = None  # the previous block's GraphNorm, applied in this block's projection GEMM
        nb = len(self.blocks)
        for bi, ((conv, norm), keep) in enumerate(zip(self.blocks, keeps)):
            c = conv.out_channels
            H, a_s, a_d = _f(R, c, dev=dev), _f(R, dev=dev), _f(R, dev=dev)
            if pend is not None:  # x = the previous GraphNorm's INPUT; its y / keep written by this GEMM
                check(LIB.vg_gat_lin_att_gn(ptr(pend["O"]), ptr(conv.lin.weight), R, xw, c, ptr(conv.att_src),
                                            ptr(conv.att_dst), ptr(H), ptr(a_s), ptr(a_d), ctypes.byref(pend["desc"]),
                                            st), "vg_gat_lin_att_gn")
                pend = None
            else:
                check(dense("vg_gat_lin_att")(ptr(x), xw, ptr(conv.lin.weight), R, xw, c, ptr(conv.att_src),
                                              ptr(conv.att_dst), ptr(H), ptr(a_s), ptr(a_d), st), "vg_gat_lin_att")
            O, alpha = _f(R, c, dev=dev), _f(3 * E, dev=dev)
            gnp, g = ops.gnp_buffer(csr3, c, dev)  # the GraphNorm's column partials from the aggregation
            ops.aggregate_fwd_raw(csr3, c, ptr(H), ptr(a_s), ptr(a_d), ptr(conv.bias), float(conv.negative_slope),
                                  ptr(O), ptr(alpha), st, gnp)
            Y, stats = _f(X4, c, dev=dev), _f(3 * 2 * c, dev=dev)
            if gnp is not None:
                spec = keep if keep is not None and not isinstance(keep, torch.Tensor) else None
                if spec is not None:
                    keep = _f(R, c, dev=dev)
                    args = (None, float(spec.p), int(spec.seed), ptr(spec.iter), int(spec.salt) & 0xFFFFFFFF)
                else:
                    args = (ptr(keep), 0.0, 0, None, 0)
                blk.append(dict(X=x, xw=xw, H=H, O=O, alpha=alpha, a_s=a_s, a_d=a_d, Y=Y, stats=stats, keep=keep,
                                c=c))
                nxt = self.blocks[bi + 1][0].out_channels if bi + 1 < nb else 0
                if _lib._GN_APPLY_GEMM and 0 < nxt <= 64 and c <= 128 and n >= 64 and gemm_precision() == "f32":
                    check(LIB.vg_graphnorm_stats_gnp(3, n, c, ptr(gnp), g, ptr(norm.mean_scale), float(norm.eps),
                                                     ptr(stats), st), "vg_graphnorm_stats_gnp")
                    desc = VgGnApply(stats=stats.data_ptr(), weight=norm.weight.data_ptr(),
                                     bias=norm.bias.data_ptr(), mean_scale=norm.mean_scale.data_ptr(),
                                     keep=None if spec is not None or keep is None else keep.data_ptr(),
                                     eps=float(norm.eps), p_drop=float(spec.p) if spec is not None else 0.0, seg_rows=n,
                                     salt=(int(spec.salt) & 0xFFFFFFFF) if spec is not None else 0,
                                     seed=int(spec.seed) if spec is not None else 0,
                                     iter=spec.iter.data_ptr() if spec is not None else None, y=Y.data_ptr(),
                                     keep_out=keep.data_ptr() if spec is not None else None)
                    pend = dict(O=O, desc=desc)
                else:
                    check(LIB.vg_graphnorm_fwd_gnp(ptr(O), 3, n, c, ptr(norm.weight), ptr(norm.bias),
                                                   ptr(norm.mean_scale), *args, float(norm.eps), ptr(Y),
                                                   ptr(keep) if spec is not None else None, ptr(stats), ptr(gnp), g,
                                                   st), "vg_graphnorm_fwd_gnp")
                x, xw = Y, c
                continue
            ws = _f(int(LIB.vg_graphnorm_seg_ws_floats(3, n, c)), dev=dev)
            if keep is not None and not isinstance(keep, torch.Tensor):  # DropSpec: drawn in-kernel
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
        dec_out = [_f(R if i == nd - 1 else X4, lin.out_features, dev=dev) for i, lin in enumerate(self.dec)]
        dec_w = [xw] + [lin.out_features for lin in self.dec]
        if not linear_chain(ptr(x), xw, R, dec_w,
                            [dict(weight=lin.weight.data_ptr(), bias=lin.bias.data_ptr(), out=z.data_ptr(),
                                  ld_out=lin.out_features, act=ACT_NONE if i == nd - 1 else ACT_RELU)
                             for i, (lin, z) in enumerate(zip(self.dec, dec_out))], st):
            for i, lin in enumerate(self.dec):
                o = lin.out_features
                self._gemm(st, ptr(x), xw, ptr(lin.weight), xw, 1, ptr(dec_out[i]), o, R, o, xw, ptr(lin.bias),
                           ACT_NONE if i == nd - 1 else ACT_RELU)
                x, xw = dec_out[i], o
        scores = dec_out[-1]
        if scores.shape[1] != 1:
            raise ValueError("the critic must output one score per node")

        # adjoint buffers of pass D (rows [0,3N)) whose rows [3N,4N) pass B fills
        seeds = self._seeds(prep)
        adj_dec = [_f(X4, l.out_features, dev=dev) for l in self.dec[:-1]] + [seeds]
        adj_H = [_f(X4, B["c"], dev=dev) for B in blk]
        adj_mlp = [_f(X4, l.out_features, dev=dev) for l in self.mlp]

        def adj_chain(r0: int, nrows: int, r_aux: int) -> bool:
            """the decoder's adjoint chain adj_dec[nd-1] -> ... -> adj_dec[0]
            (rows r0.. of the adjoint buffers, masks from rows r_aux.. of the
            forward outputs) as one vg_linear_chain launch"""
            ws = [self.dec[i].weight.shape[0] for i in range(nd - 1, 0, -1)] + [self.dec[0].weight.shape[0]]
            return linear_chain(rows(adj_dec[nd - 1], r0, ws[0]), ws[0], nrows, ws,
                                [dict(weight=self.dec[i].weight.data_ptr(), w_trans=1, act=ACT_MASK,
                                      aux=rows(dec_out[i - 1], r_aux, self.dec[i].weight.shape[1]),
                                      ld_aux=self.dec[i].weight.shape[1],
                                      out=rows(adj_dec[i - 1], r0, self.dec[i].weight.shape[1]),
                                      ld_out=self.dec[i].weight.shape[1]) for i in range(nd - 1, 0, -1)], st)

        # ---------------------------------------------------------- pass B
        if not adj_chain(trow, n, mrow):
            for i in range(nd - 1, 0, -1):
                Wt = self.dec[i].weight
                aw, m = Wt.shape
                self._gemm(st, rows(adj_dec[i], trow, aw), aw, ptr(Wt), m, 0, rows(adj_dec[i - 1], trow, m), m, n, m,
                           aw, None, ACT_MASK, rows(dec_out[i - 1], mrow, m), m)
        W = self.dec[0].weight
        dY = _f(n, W.shape[1], dev=dev)
        tp = gemm_dy(rows(adj_dec[0], trow, W.shape[0]), W.shape[0], ptr(W), W.shape[1], ptr(dY), n, W.shape[1],
                     W.shape[0], nb - 1, True)
        dY_b, dO_b = [None] * nb, [None] * nb
        for b in range(nb - 1, -1, -1):
            (conv, norm), B = self.blocks[b], blk[b]
            c = B["c"]
            dY_b[b] = dY
            dO = _f(n, c, dev=dev)
            dH = rows(adj_H[b], trow, c)
            ws = _f(int(LIB.vg_gat_bwd_ws_floats(n, E, c)), dev=dev)
            if _GN_ROWS:  # g_x (= dO) formed in the GAT backward's destination-row pass
                gn, gws = gn_bwd(b, True, tp, dY, None, False)
                check(LIB.vg_gat_bwd_gn(ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot),
                                        ptr(csr.csc_dst), n, E, c, rows(B["H"], mrow, c), ptr(conv.att_src),
                                        ptr(conv.att_dst), _off(B["a_s"], mrow), _off(B["a_d"], mrow),
                                        _off(B["alpha"], 2 * E), ctypes.byref(gn), ptr(dO),
                                        float(conv.negative_slope), dH, None, None, None, 0, None, 0, ptr(ws), None,
                                        None, st), "vg_gat_bwd_gn")
            else:
                gn_bwd(b, True, tp, dY, dO, False)
                check(LIB.vg_gat_bwd_ex(ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot),
                                        ptr(csr.csc_dst), n, E, c, rows(B["H"], mrow, c), ptr(conv.att_src),
                                        ptr(conv.att_dst), _off(B["a_s"], mrow), _off(B["a_d"], mrow),
                                        _off(B["alpha"], 2 * E), ptr(dO), float(conv.negative_slope), dH, None, None,
                                        None, 0, None, 0, ptr(ws), st), "vg_gat_bwd_ex")
            dO_b[b] = dO
            cin = B["xw"]
            if b > 0:
                dX = _f(n, cin, dev=dev)
                tp = gemm_dy(dH, c, ptr(conv.lin.weight), cin, ptr(dX), n, cin, c, b - 1, True)
                dY = dX
            else:
                self._gemm(st, dH, c, ptr(conv.lin.weight), cin, 0, rows(adj_mlp[-1], trow, cin), cin, n, cin, c,
                           None, ACT_MASK, rows(mlp_out[-1], mrow, cin), cin)
        for i in range(nm - 1, 0, -1):
            Wt = self.mlp[i].weight
            o, m = Wt.shape
            self._gemm(st, rows(adj_mlp[i], trow, o), o, ptr(Wt), m, 0, rows(adj_mlp[i - 1], trow, m), m, n, m, o,
                       None, ACT_MASK, rows(mlp_out[i - 1], mrow, m), m)
        W = self.mlp[0].weight
        hd = W.shape[0]
        g = _f(n, K, dev=dev)
        self._gemm(st, rows(adj_mlp[0], trow, hd), hd, _off(W, F), W0, 0, ptr(g), K, n, K, hd)
        out = _f(2, dev=dev)
        gws = _f(int(LIB.vg_gp_head_ws_floats(n)), dev=dev)
        gcnt = self._const(("gp_counter", dev), lambda: torch.zeros(1, dtype=torch.int32, device=dev))
        u0 = _off(X0, trow * W0 + F)  # dGP/dg written into the label columns of X0's tangent rows
        check(LIB.vg_gp_head(ptr(g), n, K, ptr(scores), self.lam, u0, W0, ptr(out), ptr(gws), ptr(gcnt), st),
              "vg_gp_head")

        # ---------------------------------------------------------- pass C
        self._gemm(st, u0, W0, _off(W, F), W0, 1, rows(mlp_out[0], trow, hd), hd, n, hd, K, None, ACT_MASK,
                   rows(mlp_out[0], mrow, hd), hd)
        uw = hd
        for i in range(1, nm):
            lin = self.mlp[i]
            o = lin.out_features
            self._gemm(st, rows(mlp_out[i - 1], trow, uw), uw, ptr(lin.weight), uw, 1, rows(mlp_out[i], trow, o), o, n,
                       o, uw, None, ACT_MASK, rows(mlp_out[i], mrow, o), o)
            uw = o
        u_in = rows(mlp_out[-1], trow, uw)
        hinj_b, oinj_b = [None] * nb, [None] * nb
        for b in range(nb):
            (conv, norm), B = self.blocks[b], blk[b]
            c, cin = B["c"], B["xw"]
            # tangent of the projection with its attention projections in the epilogue
            uH, up_s, up_d = _f(n, c, dev=dev), _f(n, dev=dev), _f(n, dev=dev)
            check(dense("vg_gat_lin_att")(u_in, cin, ptr(conv.lin.weight), n, cin, c, ptr(conv.att_src),
                                     ptr(conv.att_dst), ptr(uH), ptr(up_s), ptr(up_d), st), "vg_gat_lin_att")
            uO, hinj = _f(n, c, dev=dev), _f(n, c, dev=dev)
            ws = _f(int(LIB.vg_gat_jvp2_ws_floats(n, E, c)), dev=dev)
            # the source pass (hinj, read in pass D) joins one grouped launch after the sweep
            jargs = (ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot), ptr(csr.csc_dst), n, E,
                     c, rows(B["H"], mrow, c), ptr(uH), ptr(dO_b[b]), ptr(conv.att_src), ptr(conv.att_dst),
                     _off(B["a_s"], mrow), _off(B["a_d"], mrow), _off(B["alpha"], 2 * E),
                     float(conv.negative_slope), ptr(uO), ptr(hinj), ptr(conv.att_src.grad),
                     ptr(conv.att_dst.grad), ptr(up_s), ptr(up_d), ptr(ws))
            gx, gkeep = rows(B["O"], mrow, c), rows(B["keep"], mrow, c) if B["keep"] is not None else None
            gstats = _off(B["stats"], 2 * 2 * c)
            oinj = _f(n, c, dev=dev)
            gws = _f(int(LIB.vg_graphnorm_seg_ws_floats(1, n, c)), dev=dev)
            if _lib._GN_JVP_FUSE:  # the GraphNorm tangent sums from the GAT tangent pass
                nblk = int(LIB.vg_gat_jvp2_blocks(n, c))
                gpart = _f(nblk * 5 * c, dev=dev)
                gn = VgGnJvp(x=gx, keep=gkeep, g_y=dY_b[b].data_ptr(),
                             stats=gstats, weight=norm.weight.data_ptr(), bias=norm.bias.data_ptr(),
                             mean_scale=norm.mean_scale.data_ptr(), eps=float(norm.eps), part=gpart.data_ptr())
                folds.jvp_gn(jargs, gn, st, keep=(ws, uH, gpart))
                check(LIB.vg_graphnorm_jvp2_part(gx, n, c, ptr(norm.weight), ptr(norm.bias), ptr(norm.mean_scale),
                                                 gkeep, float(norm.eps), gstats, ptr(uO), ptr(dY_b[b]),
                                                 rows(B["Y"], trow, c), ptr(oinj), ptr(norm.weight.grad),
                                                 ptr(norm.mean_scale.grad), ptr(gpart), nblk, ptr(gws), st),
                      "vg_graphnorm_jvp2_part")
            else:
                folds.jvp(jargs, st, keep=(ws, uH))
                check(LIB.vg_graphnorm_jvp2(gx, n, c, ptr(norm.weight), ptr(norm.bias), ptr(norm.mean_scale), gkeep,
                                            float(norm.eps), gstats, ptr(uO), ptr(dY_b[b]), rows(B["Y"], trow, c),
                                            ptr(oinj), ptr(norm.weight.grad), ptr(norm.mean_scale.grad), ptr(gws), sy,
                                            st), "vg_graphnorm_jvp2")
            hinj_b[b], oinj_b[b] = hinj, oinj
            u_in, uw = rows(B["Y"], trow, c), c
        # the tangent chain (VGAN_CHAIN_TANGENT=0: per-layer GEMMs): 14.3 vs
        # 16.7 us at 12.7k rows (profiles/r02_chain_probe_v3.json,
        # profiles/r02_ab_chain.txt)
        tan_w = [uw] + [lin.out_features for lin in self.dec[:-1]]
        if not _CHAIN_TANGENT or not linear_chain(u_in, uw, n, tan_w,
                            [dict(weight=lin.weight.data_ptr(), act=ACT_MASK,
                                  aux=rows(dec_out[i], mrow, lin.out_features), ld_aux=lin.out_features,
                                  out=rows(dec_out[i], trow, lin.out_features), ld_out=lin.out_features)
                             for i, lin in enumerate(self.dec[:-1])], st):
            for i, lin in enumerate(self.dec[:-1]):
                o = lin.out_features
                self._gemm(st, u_in, uw, ptr(lin.weight), uw, 1, rows(dec_out[i], trow, o), o, n, o, uw, None,
                           ACT_MASK, rows(dec_out[i], mrow, o), o)
                u_in, uw = rows(dec_out[i], trow, o), o

        folds.run_jvp_src(st)  # every block's dQ/dh injection, one launch

        # ---------------------------------------------------------- pass D
        # weight gradients over 4N rows: [pass-D adjoint ; pass-B adjoint]^T [activation ; tangent]
        dec_in = [blk[-1]["Y"] if blk else mlp_out[-1]] + dec_out[:-1]
        chained = adj_chain(0, R, 0)  # the adjoint chain first; the weight-gradient products are deferred
        for i in range(nd - 1, -1, -1):
            lin = self.dec[i]
            aw, m = lin.weight.shape
            self._gemm_tn(folds, st, dev, ptr(adj_dec[i]), aw, ptr(dec_in[i]), m, X4, aw, m, ptr(lin.weight.grad), m,
                          ptr(lin.bias.grad), R)
            if i > 0:
                if not chained:
                    self._gemm(st, ptr(adj_dec[i]), aw, ptr(lin.weight), m, 0, ptr(adj_dec[i - 1]), m, R, m, aw, None,
                               ACT_MASK, ptr(dec_out[i - 1]), m)
            else:
                dY = _f(R, m, dev=dev)
                tp = gemm_dy(ptr(adj_dec[0]), aw, ptr(lin.weight), m, ptr(dY), R, m, aw, nb - 1, False)
        for b in range(nb - 1, -1, -1):
            (conv, norm), B = self.blocks[b], blk[b]
            c, cin = B["c"], B["xw"]
            dO = _f(R, c, dev=dev)
            ws = _f(int(LIB.vg_gat_bwd_ws_floats(R, 3 * E, c)), dev=dev)
            gat_args = (ptr(csr3.row_ptr), ptr(csr3.col), ptr(csr3.csc_ptr), ptr(csr3.csc_slot), ptr(csr3.csc_dst), R,
                        3 * E, c, ptr(B["H"]), ptr(conv.att_src), ptr(conv.att_dst), ptr(B["a_s"]), ptr(B["a_d"]),
                        ptr(B["alpha"]))
            gat_tail = (float(conv.negative_slope), ptr(adj_H[b]), ptr(conv.att_src.grad), ptr(conv.att_dst.grad),
                        ptr(conv.bias.grad), 1, ptr(hinj_b[b]), mrow, ptr(ws))
            if _GN_ROWS:
                gn, gws = gn_bwd(b, False, tp, dY, None, True, ptr(oinj_b[b]), mrow * c)
                folds.call(LIB.vg_gat_bwd_gn, gat_args + (ctypes.byref(gn), ptr(dO)) + gat_tail, st,
                           keep=(ws, gws), name="vg_gat_bwd_gn")
            else:
                gn_bwd(b, False, tp, dY, dO, True, ptr(oinj_b[b]), mrow * c)
                folds.call(LIB.vg_gat_bwd_deferred, gat_args + (ptr(dO),) + gat_tail, st, keep=(ws,),
                           name="vg_gat_bwd_deferred")
            self._gemm_tn(folds, st, dev, ptr(adj_H[b]), c, ptr(B["X"]), cin, X4, c, cin, ptr(conv.lin.weight.grad), cin)
            if b > 0:
                dY = _f(R, cin, dev=dev)
                tp = gemm_dy(ptr(adj_H[b]), c, ptr(conv.lin.weight), cin, ptr(dY), R, cin, c, b - 1, False)
            else:
                self._gemm(st, ptr(adj_H[b]), c, ptr(conv.lin.weight), cin, 0, ptr(adj_mlp[-1]), cin, R, cin, c,
                           None, ACT_MASK, ptr(mlp_out[-1]), cin)
        for i in range(nm - 1, -1, -1):
            lin = self.mlp[i]
            o, m = lin.weight.shape
            xin = X0 if i == 0 else mlp_out[i - 1]
            self._gemm_tn(folds, st, dev, ptr(adj_mlp[i]), o, ptr(xin), m, X4, o, m, ptr(lin.weight.grad), m,
                          ptr(lin.bias.grad), R)
            if i > 0:
                self._gemm(st, ptr(adj_mlp[i]), o, ptr(lin.weight), m, 0, ptr(adj_mlp[i - 1]), m, R, m, o, None,
                           ACT_MASK, ptr(mlp_out[i - 1]), m)
        folds.flush(st)
        self.last_gp = out[1]
        return out[0]
