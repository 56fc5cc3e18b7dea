"""Explicit generator iteration: loss and generator gradient without autograd.

Replaces the generator half of the training step (``trainer.py:483-491``):
G(z) -> Gumbel-softmax labels -> D(label_hard) -> ``_compute_generator_loss``
(``trainer.py:334-385``) -> ``g_loss.backward()`` with the discriminator's
parameters frozen (their gradients are zeroed before every critic iteration
and never read, so they are not formed).  Under autograd that backward is
~120 Python-side Function backwards and ~3.5 ms of host time per iteration at
batch 32 (profiles/r03_host_profile_eager_step.txt), which a fresh batch -- no
captured graph to replay -- pays in full.  Here the same kernels run from one
straight-line schedule:

  forward   the matched-features encoder and the MLP encoder
            (vg_gemm_ln_act, row statistics saved), the 14 GATConv blocks
            (vg_gat_lin_att, the aggregation with the GraphNorm partials in its
            epilogue, vg_graphnorm_fwd_gnp with the dropout mask drawn and
            stored in-kernel), the decoder, the Gumbel head; then D(label_hard)
            in train mode and the fused loss head;
  backward  the loss head's seeds; D's INPUT VJP only (adjoint chain, GraphNorm
            and GAT backwards without parameter gradients, label columns of
            D's first layer); the Gumbel backward; G's backward with every
            GraphNorm's column partials from the epilogue of the GEMM that
            forms its output gradient, the GraphNorm's elementwise backward in
            the GAT backward's row pass, and every parameter-gradient fold and
            weight-gradient product deferred to ONE grouped flush.

Randomness is drawn in the autograd path's order (z, the generator's 14 masks,
the Gumbel noise, the discriminator's 6 masks), so both paths see the same
numbers from the same RNG state; the forward runs the very kernels the
autograd path runs, so labels and loss are bit-identical, and the gradient
differs only in the summation grouping of fused reductions
(tests/test_genstep_gpu.py).  Gradients are ACCUMULATED into the generator's
``.grad`` (views into its flat buffer), like ``backward()``.
"""
from __future__ import annotations

import ctypes
import os
from typing import List

import torch
import torch.nn as nn

from . import _lib
from . import data as vdata
from . import ops
from ._lib import (_GN_ROWS, LIB, FoldCollector, VgGnBwdIn, check, dense, gemm_precision, linear_chain, ptr,
                   stream_handle, sync_counter)
from .critic import _GN_FUSE, ACT_ADD, ACT_MASK, ACT_NONE, ACT_RELU, CriticEngine, _f, _off

# VGAN_GEN_ADD_FUSE=0: the summed adjoints (label_hard, x, em) as a product
# then a torch add_ instead of the product's add epilogue (A/B knob)
_ADD_FUSE = os.environ.get("VGAN_GEN_ADD_FUSE", "1") == "1"
# VGAN_GEN_NATIVE=0: the iteration issued from Python (the A/B leg of
# vg_gen_loss_and_grad, which is bit-identical)
_NATIVE = os.environ.get("VGAN_GEN_NATIVE", "1") == "1"


class GeneratorEngine:
    def __init__(self, generator: nn.Module, discriminator: nn.Module, configuration):
        G, D, cfg = generator, discriminator, configuration
        self.G, self.D = G, D
        self.n_classes = int(cfg.NUM_CLASSES)
        self.z_dim = int(cfg.Z_DIM)
        self.lambdas = tuple(float(v) for v in (cfg.LAMBDA_ADV, cfg.LAMBDA_LABEL, cfg.LAMBDA_RATIO,
                                                 cfg.LAMBDA_RATIO_VOID, cfg.LAMBDA_FAR))
        self.dim_scale = float(cfg.NORMALIZATION_FACTOR_DIMENSION)
        self.void_class = int(cfg.VOID)
        self.mfe = G._mlp_blocks(G.matched_features_encoder)
        self.mlp = G._mlp_blocks(G.mlp_encoder)
        dec_mods = list(G.decoder.children())
        self.dec = G._mlp_blocks(nn.Sequential(*dec_mods[:-1]))
        self.dec_last = dec_mods[-1]
        self.gblocks = [(getattr(G.encoder, f"module_{4 * b}"), getattr(G.encoder, f"module_{4 * b + 1}"))
                        for b in range(G.encoder.num_blocks)]
        self.d_mlp: List[nn.Linear] = [m for m in D.mlp_encoder if isinstance(m, nn.Linear)]
        self.d_dec: List[nn.Linear] = [m for m in D.decoder if isinstance(m, nn.Linear)]
        self.dblocks = [(getattr(D.encoder, f"module_{4 * b}"), getattr(D.encoder, f"module_{4 * b + 1}"))
                        for b in range(D.encoder.num_blocks)]
        self._consts = {}
        self.supported = self._supported(cfg, G, D, dec_mods)

    def _supported(self, cfg, G, D, dec_mods) -> bool:
        """The layer pattern this schedule is written for: the reference's
        models (models.py:14-155, 158-245) with the WGAN-GP loss head."""
        if not getattr(cfg, "USE_WGANGP", True) or self.n_classes <= 2:
            return False
        mlps = ((self.mfe, G.matched_features_encoder), (self.mlp, G.mlp_encoder))
        if any(not blocks or 3 * len(blocks) != len(list(m.children())) for blocks, m in mlps):
            return False
        if not self.dec or 3 * len(self.dec) + 1 != len(dec_mods) or not isinstance(self.dec_last, nn.Linear):
            return False
        if any(b[0].out_features > 128 for b in self.mfe + self.mlp + self.dec):
            return False
        d_mlp_mods = list(D.mlp_encoder.children())
        d_dec_mods = list(D.decoder.children())
        pairs_ok = all(isinstance(d_mlp_mods[i], nn.Linear) and isinstance(d_mlp_mods[i + 1], nn.ReLU)
                       for i in range(0, len(d_mlp_mods), 2)) and len(d_mlp_mods) == 2 * len(self.d_mlp)
        dec_ok = len(d_dec_mods) == 2 * len(self.d_dec) - 1 and all(
            isinstance(m, nn.ReLU) for m in d_dec_mods[1::2]) and self.d_dec[-1].out_features == 1
        return bool(pairs_ok and dec_ok and self.dblocks and self.gblocks)

    def _const(self, key, make):
        t = self._consts.get(key)
        if t is None:
            t = self._consts[key] = make()
        return t

    # ---------------------------------------------------------- helpers
    @staticmethod
    def _gemm(st, A, lda, B, ldb, bt, C, ldc, n, m, k, bias=None, act=ACT_NONE, aux=None, ldaux=0):
        check(dense("vg_gemm")(A, lda, B, ldb, bt, bias, act, aux, ldaux, C, ldc, n, m, k, st), "vg_gemm")

    def _gemm_sum(self, st, A, lda, B, ldb, C, ldc, n, m, k, other, col):
        """C [n, m] = A B + other[:, col:col + m]: the sum of a tensor's two
        adjoints, added in the product's epilogue (act 4) -- bit-identical to
        the product then torch's add_ (VGAN_GEN_ADD_FUSE=0, the A/B leg)."""
        if _ADD_FUSE:
            self._gemm(st, A, lda, B, ldb, 0, ptr(C), ldc, n, m, k, None, ACT_ADD, _off(other, col), other.shape[1])
        else:
            self._gemm(st, A, lda, B, ldb, 0, ptr(C), ldc, n, m, k)
            C.add_(other[:, col:col + m])

    @staticmethod
    def _tn(folds, st, dev, A, lda, B, ldb, n, m, k, C, ldc, db=None):
        """C += A^T B (and db += column sums of A) for tensors A, B, deferred
        to the flush (which keeps A and B alive until then)."""
        ws = _f(max(1, int(LIB.vg_gemm_tn_ws_floats(n, m, k))), dev=dev)
        folds.tn((ptr(A), lda, ptr(B), ldb, n, m, k, C, ldc, db, n, 1, ptr(ws)), st, keep=(ws, A, B))

    @staticmethod
    def _ln_fwd(st, dev, x, ldx, blk, n):
        """[Linear -> LayerNorm -> LeakyReLU] with the pre-norm output and row
        statistics kept for the backward (as _LinearLNActFn saves them)."""
        lin, ln, act = blk
        m, k = lin.weight.shape
        h, y, mean, rstd = _f(n, m, dev=dev), _f(n, m, dev=dev), _f(n, dev=dev), _f(n, dev=dev)
        check(dense("vg_gemm_ln_act")(ptr(x), ldx, ptr(lin.weight), n, m, k, ptr(lin.bias), ptr(ln.weight),
                                      ptr(ln.bias), float(ln.eps), float(act.negative_slope), ptr(h), ptr(y),
                                      ptr(mean), ptr(rstd), st), "vg_gemm_ln_act")
        return dict(blk=blk, x=x, ldx=ldx, h=h, y=y, mean=mean, rstd=rstd, m=m, k=k)

    def _ln_bwd(self, folds, st, dev, S, g_y, n):
        """g_h = d(pre-norm) from g_y; gamma / beta and weight / bias
        gradients accumulated (deferred)."""
        lin, ln, act = S["blk"]
        m, k = S["m"], S["k"]
        g_h = _f(n, m, dev=dev)
        ws = _f(int(LIB.vg_ln_act_bwd_ws_floats(m)), dev=dev)
        folds.call(LIB.vg_ln_act_bwd_deferred, (ptr(S["h"]), n, m, ptr(ln.weight), ptr(ln.bias),
                                                float(act.negative_slope), ptr(S["mean"]), ptr(S["rstd"]), ptr(g_y),
                                                ptr(g_h), ptr(ln.weight.grad), ptr(ln.bias.grad), 1, ptr(ws)),
                   st, keep=(ws,), name="vg_ln_act_bwd_deferred")
        self._tn(folds, st, dev, g_h, m, S["x"], S["ldx"], n, m, k, ptr(lin.weight.grad), k,
                 ptr(lin.bias.grad))
        return g_h

    @staticmethod
    def _gat_fwd(st, sy, dev, csr, x, xw, conv, norm, keep, n):
        """GATConv -> GraphNorm -> ReLU -> Dropout (models.py:73-75); the
        dropout mask, when drawn in-kernel, is stored for the backward."""
        c = conv.out_channels
        E = csr.num_edges
        H, a_s, a_d = _f(n, c, dev=dev), _f(n, dev=dev), _f(n, dev=dev)
        check(dense("vg_gat_lin_att")(ptr(x), xw, ptr(conv.lin.weight), n, xw, c, ptr(conv.att_src),
                                      ptr(conv.att_dst), ptr(H), ptr(a_s), ptr(a_d), st), "vg_gat_lin_att")
        O, alpha = _f(n, c, dev=dev), _f(E, dev=dev)
        gnp, g = ops.gnp_buffer(csr, c, dev)
        ops.aggregate_fwd_raw(csr, c, ptr(H), ptr(a_s), ptr(a_d), ptr(conv.bias), float(conv.negative_slope), ptr(O),
                              ptr(alpha), st, gnp)
        Y, stats = _f(n, c, dev=dev), _f(2 * c, dev=dev)
        spec = keep if keep is not None and not isinstance(keep, torch.Tensor) else None
        if spec is not None:
            keep = _f(n, c, dev=dev)
        w, b, ms, eps = ptr(norm.weight), ptr(norm.bias), ptr(norm.mean_scale), float(norm.eps)
        if gnp is not None:
            args = ((None, float(spec.p), int(spec.seed), ptr(spec.iter), int(spec.salt) & 0xFFFFFFFF)
                    if spec is not None else (ptr(keep), 0.0, 0, None, 0))
            check(LIB.vg_graphnorm_fwd_gnp(ptr(O), 1, n, c, w, b, ms, *args, eps, ptr(Y),
                                           ptr(keep) if spec is not None else None, ptr(stats), ptr(gnp), g, st),
                  "vg_graphnorm_fwd_gnp")
        else:
            ws = _f(int(LIB.vg_graphnorm_seg_ws_floats(1, n, c)), dev=dev)
            if spec is not None:
                check(LIB.vg_graphnorm_fwd_drop(ptr(O), 1, n, c, w, b, ms, float(spec.p), int(spec.seed),
                                                ptr(spec.iter), int(spec.salt) & 0xFFFFFFFF, eps, ptr(Y), ptr(keep),
                                                ptr(stats), ptr(ws), sy, st), "vg_graphnorm_fwd_drop")
            else:
                check(LIB.vg_graphnorm_fwd_seg(ptr(O), 1, n, c, w, b, ms, ptr(keep), eps, ptr(Y), ptr(stats),
                                               ptr(ws), sy, st), "vg_graphnorm_fwd_seg")
        return dict(X=x, xw=xw, H=H, O=O, alpha=alpha, a_s=a_s, a_d=a_d, Y=Y, stats=stats, keep=keep, c=c,
                    conv=conv, norm=norm)

    def _gemm_dy(self, st, dev, A, lda, B, ldb, out, n, m, k, blk):
        """out [n, m] = A B, the output gradient of ``blk``'s GraphNorm; returns
        that backward's column partials from the GEMM epilogue (as the
        autograd path's GraphNorm hint) or None."""
        norm = blk["norm"]
        if not (_GN_FUSE and n >= 64 and m % 4 == 0):
            self._gemm(st, A, lda, B, ldb, 0, ptr(out), m, n, m, k)
            return None
        tp = _f(int(LIB.vg_gemm_gn_tpart_floats(n, m)), dev=dev)
        check(dense("vg_gemm_gn_bwd")(A, lda, B, ldb, n, m, k, ptr(out), m, ptr(blk["O"]), ptr(blk["keep"]), n,
                                      ptr(norm.weight), ptr(norm.bias), ptr(norm.mean_scale), float(norm.eps),
                                      ptr(blk["stats"]), ptr(tp), st), "vg_gemm_gn_bwd")
        return tp

    @staticmethod
    def _gat_bwd(folds, st, sy, dev, csr, B, g_y, tp, pgrads: bool):
        """GraphNorm(+ReLU+Dropout) and GATConv backward of one block: dH (the
        projection's output gradient); with ``pgrads`` the block's GraphNorm
        and attention / bias gradients are accumulated (folds deferred)."""
        conv, norm, c = B["conv"], B["norm"], B["c"]
        n, E = csr.num_nodes, csr.num_edges
        dO, dH = _f(n, c, dev=dev), _f(n, c, dev=dev)
        ws = _f(int(LIB.vg_gat_bwd_ws_floats(n, E, c)), dev=dev)
        gat_args = (ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot), ptr(csr.csc_dst), n, E, c,
                    ptr(B["H"]), ptr(conv.att_src), ptr(conv.att_dst), ptr(B["a_s"]), ptr(B["a_d"]), ptr(B["alpha"]))
        if pgrads:
            tail = (float(conv.negative_slope), ptr(dH), ptr(conv.att_src.grad), ptr(conv.att_dst.grad),
                    ptr(conv.bias.grad), 1, None, 0, ptr(ws))
            pg = (ptr(norm.weight.grad), ptr(norm.bias.grad), ptr(norm.mean_scale.grad))
        else:
            tail = (float(conv.negative_slope), ptr(dH), None, None, None, 0, None, 0, ptr(ws))
            pg = (None, None, None)
        gws = _f(int(LIB.vg_graphnorm_seg_ws_floats(1, n, c)), dev=dev)
        gn_in = (ptr(B["O"]), 1, n, c, ptr(norm.weight), ptr(norm.bias), ptr(norm.mean_scale), ptr(B["keep"]),
                 float(norm.eps), ptr(B["stats"]), ptr(g_y))
        g_x = None if _GN_ROWS else ptr(dO)  # None: the column sums only, g_x formed in the GAT row pass
        if tp is not None:
            check(LIB.vg_graphnorm_bwd_seg_tiles(*gn_in, ptr(tp), g_x, *pg, 1 if pgrads else 0, None, 0, ptr(gws), st),
                  "vg_graphnorm_bwd_seg_tiles")
        else:
            check(LIB.vg_graphnorm_bwd_seg(*gn_in, g_x, *pg, 1 if pgrads else 0, None, 0, ptr(gws), sy, st),
                  "vg_graphnorm_bwd_seg")
        if _GN_ROWS:
            gn = VgGnBwdIn(x=ptr(B["O"]), keep=ptr(B["keep"]), g_y=ptr(g_y), inj=None, weight=ptr(norm.weight),
                           bias=ptr(norm.bias), mean_scale=ptr(norm.mean_scale), stats=ptr(B["stats"]),
                           sums=_off(gws, int(LIB.vg_graphnorm_bwd_sums_offset(1, c))), eps=float(norm.eps),
                           segments=1, seg_rows=n, inj_offset=0)
            if pgrads:
                folds.call(LIB.vg_gat_bwd_gn, gat_args + (ctypes.byref(gn), ptr(dO)) + tail, st, keep=(ws, gws),
                           name="vg_gat_bwd_gn")
            else:
                check(LIB.vg_gat_bwd_gn(*gat_args, ctypes.byref(gn), ptr(dO), *tail, None, None, st), "vg_gat_bwd_gn")
        elif pgrads:
            folds.call(LIB.vg_gat_bwd_deferred, gat_args + (ptr(dO),) + tail, st, keep=(ws,),
                       name="vg_gat_bwd_deferred")
        else:
            check(LIB.vg_gat_bwd_ex(*gat_args, ptr(dO), *tail, st), "vg_gat_bwd_ex")
        return dH

    # --------------------------------------------------- native engine
    # vg_gen_loss_and_grad issues loss_and_grad's launches from C++ (same
    # kernels, order, arguments and draws: bit-identical) with every
    # temporary in one arena: ~1-2 us of host time per launch instead of ~10.
    # Used in loss_and_grad's default configuration (the knobs at their
    # defaults, device-drawn randomness, both models in train mode, no early
    # hook, no ring aggregation); anything else runs the Python schedule.
    def _native_config_ok(self, n: int, rng, early) -> bool:
        return (_NATIVE and early is None and getattr(rng, "mode", None) == "device" and hasattr(rng, "_salt")
                and _GN_FUSE and _ADD_FUSE and _GN_ROWS and _lib._CHAIN and _lib._TN_GROUP and _lib._FOLD_SPLIT
                and _lib._FOLD_BATCH == _lib.VG_FOLD_MAX and ops._GN_FWD_FUSE and n >= 64
                and self.G.encoder.training and self.D.encoder.training
                and max(len(self.mfe), len(self.mlp), len(self.dec), len(self.d_mlp),
                        len(self.d_dec)) <= _lib.VG_GEN_MAX_LAYERS
                and max(len(self.gblocks), len(self.dblocks)) <= _lib.VG_GEN_MAX_BLOCKS)

    def _native_model(self):
        """The vg_gen_model of G's parameters and gradient views and D's
        parameters (rebuilt when any address changes), or None."""
        G, D = self.G, self.D
        dparams = self.__dict__.get("_dparams")
        if dparams is None:
            dparams = self._dparams = list(D.parameters())
        key = (gemm_precision(),) + tuple(p.data_ptr() for p in self._params) + \
            tuple(p.grad.data_ptr() for p in self._params) + tuple(p.data_ptr() for p in dparams)
        if self.__dict__.get("_native_key") == key:
            return self._native_md
        m = _lib.VgGenModel()
        m.n_mfe, m.n_mlp, m.n_gblocks, m.n_dec = len(self.mfe), len(self.mlp), len(self.gblocks), len(self.dec)
        m.n_dmlp, m.n_dblocks, m.n_ddec = len(self.d_mlp), len(self.dblocks), len(self.d_dec)
        m.bf16 = 1 if gemm_precision() == "bf16" else 0
        m.tau, m.p_drop_g, m.p_drop_d = float(G.tau), float(G.encoder.dropout), float(D.encoder.dropout)
        (m.lambda_adv, m.lambda_label, m.lambda_ratio, m.lambda_void, m.lambda_far) = self.lambdas
        m.dim_scale, m.void_class = self.dim_scale, self.void_class

        def ln_layer(dst, blk):
            lin, ln, act = blk
            if lin.bias is None or ln.weight is None or ln.bias is None:
                return False
            dst.weight, dst.bias, dst.ln_weight, dst.ln_bias = (lin.weight.data_ptr(), lin.bias.data_ptr(),
                                                                ln.weight.data_ptr(), ln.bias.data_ptr())
            dst.g_weight, dst.g_bias = lin.weight.grad.data_ptr(), lin.bias.grad.data_ptr()
            dst.g_ln_weight, dst.g_ln_bias = ln.weight.grad.data_ptr(), ln.bias.grad.data_ptr()
            dst.ln_eps, dst.slope = float(ln.eps), float(act.negative_slope)
            dst.in_, dst.out = lin.in_features, lin.out_features
            return True

        def linear(dst, lin, grads):
            if lin.bias is None:
                return False
            dst.weight, dst.bias = lin.weight.data_ptr(), lin.bias.data_ptr()
            if grads:
                dst.g_weight, dst.g_bias = lin.weight.grad.data_ptr(), lin.bias.grad.data_ptr()
            dst.in_, dst.out = lin.in_features, lin.out_features
            return True

        def block(dst, conv, norm, grads):
            if getattr(conv.lin, "bias", None) is not None:  # (GATConv's lin has none)
                return False
            dst.lin_weight, dst.att_src, dst.att_dst, dst.bias = (conv.lin.weight.data_ptr(), conv.att_src.data_ptr(),
                                                                  conv.att_dst.data_ptr(), conv.bias.data_ptr())
            dst.gn_weight, dst.gn_bias, dst.gn_mean_scale = (norm.weight.data_ptr(), norm.bias.data_ptr(),
                                                             norm.mean_scale.data_ptr())
            if grads:
                dst.g_lin_weight, dst.g_att_src, dst.g_att_dst, dst.g_bias = (
                    conv.lin.weight.grad.data_ptr(), conv.att_src.grad.data_ptr(), conv.att_dst.grad.data_ptr(),
                    conv.bias.grad.data_ptr())
                dst.g_gn_weight, dst.g_gn_bias, dst.g_gn_mean_scale = (
                    norm.weight.grad.data_ptr(), norm.bias.grad.data_ptr(), norm.mean_scale.grad.data_ptr())
            dst.gn_eps, dst.slope = float(norm.eps), float(conv.negative_slope)
            dst.in_, dst.out = conv.in_channels, conv.out_channels
            return True

        ok = all(ln_layer(m.mfe[i], b) for i, b in enumerate(self.mfe))
        ok = ok and all(ln_layer(m.mlp[i], b) for i, b in enumerate(self.mlp))
        ok = ok and all(ln_layer(m.dec[i], b) for i, b in enumerate(self.dec))
        ok = ok and linear(m.dec_last, self.dec_last, True)
        ok = ok and all(block(m.gblock[i], c, nm, True) for i, (c, nm) in enumerate(self.gblocks))
        ok = ok and all(linear(m.dmlp[i], l, False) for i, l in enumerate(self.d_mlp))
        ok = ok and all(block(m.dblock[i], c, nm, False) for i, (c, nm) in enumerate(self.dblocks))
        ok = ok and all(linear(m.ddec[i], l, False) for i, l in enumerate(self.d_dec))
        if not ok:
            return None
        self._native_key, self._native_md = key, m
        return m

    def _arena_for(self, model, batch, dev):
        """(arena tensor, floats, 256-byte aligned base) for this batch, grown
        outside a capture (25 % ahead); a replaced arena is kept alive, since
        recorded graphs may still reference it.  None when it is too small and
        a capture is running, or the model / batch is not the engine's."""
        need = int(LIB.vg_gen_arena_floats(ctypes.byref(model), ctypes.byref(batch)))
        if need < 0:
            return None
        cur = self.__dict__.get("_arena")
        if cur is not None and cur[1] >= need and cur[0].device == dev:
            return cur
        if torch.cuda.is_current_stream_capturing():
            return None
        floats = (need * 5 // 4 + 63) // 64 * 64
        t = torch.empty(floats + 64, dtype=torch.float32, device=dev)
        off = (-t.data_ptr() % 256) // 4
        if cur is not None:
            self.__dict__.setdefault("_old_arenas", []).append(cur)
        self._arena = (t, floats, t.data_ptr() + 4 * off)
        return self._arena

    def _native(self, prep, voxel_graph, rng, dev, st, sy):
        """loss_and_grad through vg_gen_loss_and_grad, or None (this batch or
        model is not the native engine's: nothing drawn, nothing launched)."""
        csr = prep.csr
        if any(csr.ring_on(conv.out_channels) for conv, _ in self.gblocks + self.dblocks):
            return None
        mx, vx, mvx, oh = prep.matched_x, prep.voxel_x, prep.matched_voxel_x, prep.onehot_f
        if any(t.dtype != torch.float32 or not t.is_contiguous() or t.dim() != 2 for t in (mx, vx, mvx, oh)):
            return None
        vtype, gptr = voxel_graph.type, voxel_graph.ptr
        if vtype.dtype != torch.int64 or gptr.dtype != torch.int64:
            return None
        vtype, gptr = vtype.contiguous(), gptr.contiguous()
        sa = voxel_graph.site_area
        sa = sa if sa.dtype == torch.float32 and sa.is_contiguous() else sa.float().contiguous()
        model = self._native_model()
        if model is None:
            return None
        n, K = vx.shape[0], self.n_classes
        b = _lib.VgGenBatch()
        b.n, b.classes, b.mx_w, b.vx_w, b.mvx_w, b.z_dim = n, K, mx.shape[1], vx.shape[1], mvx.shape[1], self.z_dim
        b.mx, b.vx, b.mvx, b.onehot = mx.data_ptr(), vx.data_ptr(), mvx.data_ptr(), oh.data_ptr()
        b.type, b.graph_ptr, b.site_area = vtype.data_ptr(), gptr.data_ptr(), sa.data_ptr()
        b.num_graphs, b.far_col, b.dy_col, b.dx_col = gptr.numel() - 1, 9, 4, 5
        ell, w = csr.ell()
        CriticEngine._csr_ref(b.g, csr, ell, w)
        b.seg_rows, b.sync = csr.seg_rows, sy
        b.one = self._const(("one", dev), lambda: torch.ones(1, dtype=torch.float32, device=dev)).data_ptr()
        it = rng._iter(dev)
        b.seed, b.iter = int(rng.seed) & ((1 << 64) - 1), it.data_ptr()
        arena = self._arena_for(model, b, dev)
        if arena is None:
            return None
        # the draws of the Python schedule, in its order: z, G's masks, the
        # Gumbel noise, D's masks (RNG.normal / keep_mask / exponential salts)
        s, nbg, nbd = rng._salt, len(self.gblocks), len(self.dblocks)
        b.z_salt = (0x40000000 | (s + 1)) & 0xFFFFFFFF
        for i in range(nbg):
            b.g_keep_salt[i] = (s + 2 + i) & 0xFFFFFFFF
        b.noise_salt = (0x40000000 | (s + 2 + nbg)) & 0xFFFFFFFF
        for i in range(nbd):
            b.d_keep_salt[i] = (s + 3 + nbg + i) & 0xFFFFFFFF
        rng._salt = s + 2 + nbg + nbd
        out, hard = _f(K + 3, dev=dev), _f(n, K, dev=dev)
        check(LIB.vg_gen_loss_and_grad(ctypes.byref(model), ctypes.byref(b), arena[2], arena[1], ptr(out), ptr(hard),
                                       st), "vg_gen_loss_and_grad")
        self.native_calls = self.__dict__.get("native_calls", 0) + 1
        return out[0], hard.unsqueeze(0)

    # ------------------------------------------------------------ engine
    def loss_and_grad(self, local_graph, voxel_graph, rng, early=None):
        """(g_loss device scalar, label_hard [1, N, K]) of trainer.py:483-490;
        the generator's gradients are added to its .grad.  ``early``: called
        (no arguments) as soon as the decoder's gradient is complete -- its
        weight-gradient products and folds flushed right after the decoder's
        backward instead of with the rest -- while the encoders' backward is
        still to run (the data-parallel trainer starts the decoder bucket's
        all-reduce there, on a side stream).  Bit-identical either way."""
        G, D = self.G, self.D
        K = self.n_classes
        prep = vdata.prepared(local_graph, voxel_graph, K)
        mx, vx = prep.matched_x, prep.voxel_x
        n = vx.shape[0]
        dev = vx.device
        st, sy = stream_handle(dev), sync_counter(dev)
        csr = prep.csr
        params = self.__dict__.get("_params")
        if params is None:  # (a module walk per iteration cost ~20 us of host time)
            params = self._params = list(G.parameters())
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        if self._native_config_ok(n, rng, early):
            r = self._native(prep, voxel_graph, rng, dev, st, sy)
            if r is not None:
                return r
        folds = FoldCollector()
        z = rng.normal((1, n, self.z_dim), dev).reshape(n, self.z_dim)

        # ------------------------------------------------- generator forward
        mfe_s = []
        x, xw = mx, mx.shape[1]
        for blk in self.mfe:  # models.py:122-131 matched-features encoder
            S = self._ln_fwd(st, dev, x, xw, blk, n)
            mfe_s.append(S)
            x, xw = S["y"], S["m"]
        em = x
        hl = em.shape[1]
        mlp_in = torch.cat([em, vx, z], dim=-1)
        mlp_s = []
        x, xw = mlp_in, mlp_in.shape[1]
        for blk in self.mlp:
            S = self._ln_fwd(st, dev, x, xw, blk, n)
            mlp_s.append(S)
            x, xw = S["y"], S["m"]
        xm, hg = x, xw
        genc = []
        training = G.encoder.training
        for conv, norm in self.gblocks:
            keep = rng.keep_mask((n, conv.out_channels), G.encoder.dropout, dev) if training else None
            B = self._gat_fwd(st, sy, dev, csr, x, xw, conv, norm, keep, n)
            genc.append(B)
            x, xw = B["Y"], B["c"]
        enc, ec = x, xw
        dec_in = torch.cat([enc, xm, em, vx, z], dim=-1)  # models.py:145
        dec_s = []
        x, xw = dec_in, dec_in.shape[1]
        for blk in self.dec:
            S = self._ln_fwd(st, dev, x, xw, blk, n)
            dec_s.append(S)
            x, xw = S["y"], S["m"]
        last = self.dec_last
        logits = _f(n, K, dev=dev)
        self._gemm(st, ptr(x), xw, ptr(last.weight), xw, 1, ptr(logits), K, n, K, xw, ptr(last.bias))
        a_last, a_last_w = x, xw
        noise = rng.exponential((n, K), dev)
        soft, hard = _f(n, K, dev=dev), _f(n, K, dev=dev)
        check(LIB.vg_gumbel_fwd(ptr(logits), ptr(noise.reshape(n, K)), n, K, float(G.tau), ptr(soft), ptr(hard), None,
                                st), "vg_gumbel_fwd")

        # ------------------------------------------- discriminator forward
        X0 = torch.cat([prep.matched_voxel_x, hard], dim=-1)
        F = prep.matched_voxel_x.shape[1]
        d_mlp_out = []
        x, xw = X0, X0.shape[1]
        for lin in self.d_mlp:
            o = lin.out_features
            y = _f(n, o, dev=dev)
            self._gemm(st, ptr(x), xw, ptr(lin.weight), xw, 1, ptr(y), o, n, o, xw, ptr(lin.bias), ACT_RELU)
            d_mlp_out.append(y)
            x, xw = y, o
        denc = []
        d_training = D.encoder.training
        for conv, norm in self.dblocks:
            keep = rng.keep_mask((n, conv.out_channels), D.encoder.dropout, dev) if d_training else None
            B = self._gat_fwd(st, sy, dev, csr, x, xw, conv, norm, keep, n)
            denc.append(B)
            x, xw = B["Y"], B["c"]
        nd = len(self.d_dec)
        dec_out = [_f(n, lin.out_features, dev=dev) for lin in self.d_dec]
        if not linear_chain(ptr(x), xw, n, [xw] + [lin.out_features for lin in self.d_dec],
                            [dict(weight=lin.weight.data_ptr(), bias=lin.bias.data_ptr(), out=o.data_ptr(),
                                  ld_out=lin.out_features, act=ACT_NONE if i == nd - 1 else ACT_RELU)
                             for i, (lin, o) in enumerate(zip(self.d_dec, dec_out))], st):
            for i, lin in enumerate(self.d_dec):
                o = lin.out_features
                self._gemm(st, ptr(x), xw, ptr(lin.weight), xw, 1, ptr(dec_out[i]), o, n, o, xw, ptr(lin.bias),
                           ACT_NONE if i == nd - 1 else ACT_RELU)
                x, xw = dec_out[i], o
        d_fake = dec_out[-1]

        # ------------------------------------------------------- loss head
        vtype = voxel_graph.type.contiguous()
        far_gen, far_ref = ops.far_per_graph(vx, hard, voxel_graph.ptr, voxel_graph.site_area, far_col=9, dy_col=4,
                                             dx_col=5, dim_scale=self.dim_scale, void_class=self.void_class)
        out = _f(K + 3, dev=dev)
        lws = _f(int(LIB.vg_gen_loss_ws_floats(n, K)), dev=dev)
        check(LIB.vg_gen_loss_fwd(ptr(d_fake), ptr(hard), ptr(logits), ptr(prep.onehot_f), ptr(vtype), n, K,
                                  ptr(far_gen), ptr(far_ref), far_gen.numel(), *self.lambdas, ptr(out), ptr(lws), st),
              "vg_gen_loss_fwd")
        one = self._const(("one", dev), lambda: torch.ones(1, dtype=torch.float32, device=dev))
        g_d, g_hard = _f(n, 1, dev=dev), _f(n, K, dev=dev)
        g_l = _f(n, K, dev=dev) if self.lambdas[1] != 0.0 else None
        check(LIB.vg_gen_loss_bwd(ptr(one), ptr(out), ptr(logits), ptr(vtype), n, K, ptr(g_d), ptr(g_hard), ptr(g_l),
                                  st), "vg_gen_loss_bwd")

        # ------------------------- discriminator input VJP (no parameter grads)
        adj = [_f(n, lin.out_features, dev=dev) for lin in self.d_dec[:-1]] + [g_d]
        widths = [self.d_dec[i].weight.shape[0] for i in range(nd - 1, 0, -1)] + [self.d_dec[0].weight.shape[0]]
        if not linear_chain(ptr(g_d), 1, n, widths,
                            [dict(weight=self.d_dec[i].weight.data_ptr(), w_trans=1, act=ACT_MASK,
                                  aux=dec_out[i - 1].data_ptr(), ld_aux=self.d_dec[i].weight.shape[1],
                                  out=adj[i - 1].data_ptr(), ld_out=self.d_dec[i].weight.shape[1])
                             for i in range(nd - 1, 0, -1)], st):
            for i in range(nd - 1, 0, -1):
                aw, m = self.d_dec[i].weight.shape
                self._gemm(st, ptr(adj[i]), aw, ptr(self.d_dec[i].weight), m, 0, ptr(adj[i - 1]), m, n, m, aw, None,
                           ACT_MASK, ptr(dec_out[i - 1]), m)
        W = self.d_dec[0].weight
        dY = _f(n, W.shape[1], dev=dev)
        tp = self._gemm_dy(st, dev, ptr(adj[0]), W.shape[0], ptr(W), W.shape[1], dY, n, W.shape[1], W.shape[0],
                           denc[-1])
        adj_m = [_f(n, lin.out_features, dev=dev) for lin in self.d_mlp]
        for b in range(len(denc) - 1, -1, -1):
            B = denc[b]
            c, cin = B["c"], B["xw"]
            dH = self._gat_bwd(folds, st, sy, dev, csr, B, dY, tp, False)
            Wl = B["conv"].lin.weight
            if b > 0:
                dY = _f(n, cin, dev=dev)
                tp = self._gemm_dy(st, dev, ptr(dH), c, ptr(Wl), cin, dY, n, cin, c, denc[b - 1])
            else:
                self._gemm(st, ptr(dH), c, ptr(Wl), cin, 0, ptr(adj_m[-1]), cin, n, cin, c, None, ACT_MASK,
                           ptr(d_mlp_out[-1]), cin)
        for i in range(len(self.d_mlp) - 1, 0, -1):
            o, m = self.d_mlp[i].weight.shape
            self._gemm(st, ptr(adj_m[i]), o, ptr(self.d_mlp[i].weight), m, 0, ptr(adj_m[i - 1]), m, n, m, o, None,
                       ACT_MASK, ptr(d_mlp_out[i - 1]), m)
        W0 = self.d_mlp[0].weight
        g_lab = _f(n, K, dev=dev)  # label_hard feeds the loss head and D (models.py:229-239): both adjoints summed
        self._gemm_sum(st, ptr(adj_m[0]), W0.shape[0], _off(W0, F), W0.shape[1], g_lab, K, n, K, W0.shape[0],
                       g_hard, 0)
        g_hard = g_lab

        # --------------------------------------------------- Gumbel backward
        g_logits = _f(n, K, dev=dev)
        check(LIB.vg_gumbel_bwd(ptr(soft), ptr(g_hard), None, n, K, float(G.tau), ptr(g_logits), st), "vg_gumbel_bwd")
        if g_l is not None:
            g_logits.add_(g_l)

        # ------------------------------------------------ generator backward
        self._tn(folds, st, dev, g_logits, K, a_last, a_last_w, n, K, a_last_w, ptr(last.weight.grad),
                 a_last_w, ptr(last.bias.grad))
        g = _f(n, a_last_w, dev=dev)
        self._gemm(st, ptr(g_logits), K, ptr(last.weight), a_last_w, 0, ptr(g), a_last_w, n, a_last_w, K)
        for i in range(len(dec_s) - 1, 0, -1):
            S = dec_s[i]
            g_h = self._ln_bwd(folds, st, dev, S, g, n)
            g = _f(n, S["k"], dev=dev)
            self._gemm(st, ptr(g_h), S["m"], ptr(S["blk"][0].weight), S["k"], 0, ptr(g), S["k"], n, S["k"], S["m"])
        S = dec_s[0]
        g_h = self._ln_bwd(folds, st, dev, S, g, n)
        Wd, m, kd = S["blk"][0].weight, S["m"], S["k"]
        g_enc = _f(n, ec, dev=dev)
        tp = self._gemm_dy(st, dev, ptr(g_h), m, ptr(Wd), kd, g_enc, n, ec, m, genc[-1])
        g_xem = _f(n, hg + hl, dev=dev)  # [x | em] columns of the decoder input (enc taken above)
        self._gemm(st, ptr(g_h), m, _off(Wd, ec), kd, 0, ptr(g_xem), hg + hl, n, hg + hl, m)
        if early is not None:  # the decoder's gradient complete: its bucket can go
            folds.flush(st)
            early()
        g_y = g_enc
        g_x = None
        for b in range(len(genc) - 1, -1, -1):
            B = genc[b]
            c, cin = B["c"], B["xw"]
            dH = self._gat_bwd(folds, st, sy, dev, csr, B, g_y, tp, True)
            Wl = B["conv"].lin.weight
            self._tn(folds, st, dev, dH, c, B["X"], cin, n, c, cin, ptr(Wl.grad), cin)
            if b > 0:
                g_y = _f(n, cin, dev=dev)
                tp = self._gemm_dy(st, dev, ptr(dH), c, ptr(Wl), cin, g_y, n, cin, c, genc[b - 1])
            else:
                g_x = _f(n, cin, dev=dev)  # x feeds the encoder and the decoder (models.py:132-145)
                self._gemm_sum(st, ptr(dH), c, ptr(Wl), cin, g_x, cin, n, cin, c, g_xem, 0)
        g = g_x
        for i in range(len(mlp_s) - 1, -1, -1):
            S = mlp_s[i]
            g_h = self._ln_bwd(folds, st, dev, S, g, n)
            W_, m, k = S["blk"][0].weight, S["m"], S["k"]
            if i > 0:
                g = _f(n, k, dev=dev)
                self._gemm(st, ptr(g_h), m, ptr(W_), k, 0, ptr(g), k, n, k, m)
            else:  # the em columns of [em | voxel.x | z]
                g = _f(n, hl, dev=dev)  # em feeds the MLP encoder and the decoder
                self._gemm_sum(st, ptr(g_h), m, ptr(W_), k, g, hl, n, hl, m, g_xem, hg)
        for i in range(len(mfe_s) - 1, -1, -1):
            S = mfe_s[i]
            g_h = self._ln_bwd(folds, st, dev, S, g, n)
            if i > 0:
                W_, m, k = S["blk"][0].weight, S["m"], S["k"]
                g = _f(n, k, dev=dev)
                self._gemm(st, ptr(g_h), m, ptr(W_), k, 0, ptr(g), k, n, k, m)
        folds.flush(st)
        return out[0], hard.unsqueeze(0)
