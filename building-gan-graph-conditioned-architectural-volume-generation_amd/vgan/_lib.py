"""ctypes binding of ``libvgan_hip.so`` (the C ABI declared in ``include/vgan.h``).

The library is REQUIRED: importing this module raises if it was not built, and
every wrapper refuses non-CUDA tensors.  There is no CPU or eager-torch fallback
for the message-passing core.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

# VGAN_LIB: an alternative build of the same ABI (A/B timing of kernel variants)
LIB_PATH = os.environ.get("VGAN_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvgan_hip.so")
VG_EINVAL = -1

_c_i32, _c_i64, _c_f32, _c_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p



class VgFoldSrc(ctypes.Structure):
    """vg_fold_src (include/vgan.h)."""
    _fields_ = [("part", _c_p), ("rows", _c_i32), ("ld", _c_i32)]


class VgFold(ctypes.Structure):
    """vg_fold (include/vgan.h): one deferred parameter-gradient fold."""
    _fields_ = [("out", _c_p), ("width", _c_i32), ("k", _c_i32), ("ldo", _c_i32), ("accumulate", _c_i32),
                ("nsrc", _c_i32), ("src", VgFoldSrc * 2)]


VG_FOLD_MAX = 120
# VGAN_FOLD_BATCH: folds per vg_fold_batch launch (<= VG_FOLD_MAX; 40 was the round-4 limit, A/B knob)
_FOLD_BATCH = max(1, min(int(os.environ.get("VGAN_FOLD_BATCH", str(VG_FOLD_MAX))), VG_FOLD_MAX))


class VgTn(ctypes.Structure):
    """vg_tn (include/vgan.h): one planned weight-gradient product."""
    _fields_ = [("A", _c_p), ("B", _c_p), ("part", _c_p), ("pdb", _c_p), ("lda", _c_i32), ("ldb", _c_i32),
                ("N", _c_i32), ("M", _c_i32), ("K", _c_i32), ("rows", _c_i32), ("chunks", _c_i32),
                ("db_rows", _c_i32), ("bf16", _c_i32)]


VG_TN_GROUP_MAX = 32
# VGAN_TN_GROUP=0: launch every weight-gradient product where the backward
# forms it (one launch per layer) instead of grouping them (A/B knob)
_TN_GROUP = os.environ.get("VGAN_TN_GROUP", "1") == "1"


class VgJvpSrc(ctypes.Structure):
    """vg_jvp_src (include/vgan.h): one described source pass of vg_gat_jvp2."""
    _fields_ = [(k, _c_p) for k in ("csc_ptr", "csc_slot", "csc_dst", "h", "u", "g_out", "att_src", "att_dst",
                                     "e_gz", "e_gzp", "e_alp", "n_gad", "h_inj", "part")] + \
               [("N", _c_i32), ("C", _c_i32), ("blocks", _c_i32), ("shape", _c_i32)]


VG_JVP_GROUP_MAX = 16
# VGAN_JVP_GROUP=1: the tangent sweep's source passes as one grouped launch
# before pass D.  Off: measured 0.07 ms per step slower than one launch per
# block right after its destination-row pass
_JVP_GROUP = os.environ.get("VGAN_JVP_GROUP", "0") == "1"
# folds of more than 768 partial rows in two levels (vg_fold_batch_split),
# as the critic engine does; 0: vg_fold_batch
_FOLD_SPLIT = os.environ.get("VGAN_FOLD_SPLIT", "1") == "1"


class VgGnBwdIn(ctypes.Structure):
    """vg_gn_bwd_in (include/vgan.h): the GraphNorm backward a GAT backward
    row pass forms in its prologue (vg_gat_bwd_gn)."""
    _fields_ = [(k, _c_p) for k in ("x", "keep", "g_y", "inj", "weight", "bias", "mean_scale", "stats", "sums")] + \
               [("eps", _c_f32), ("segments", _c_i32), ("seg_rows", _c_i32), ("inj_offset", _c_i64)]


# VGAN_GN_ROWS=0: the GraphNorm backward's elementwise pass as its own launch
# instead of in the GAT backward's destination-row pass (A/B knob)
_GN_ROWS = os.environ.get("VGAN_GN_ROWS", "1") == "1"


class VgGnApply(ctypes.Structure):
    """vg_gn_apply (include/vgan.h): the GraphNorm + ReLU + Dropout that
    vg_gat_lin_att_gn applies to its operand as it loads."""
    _fields_ = [(k, _c_p) for k in ("stats", "weight", "bias", "mean_scale", "keep")] + \
               [("eps", _c_f32), ("p_drop", _c_f32), ("seg_rows", _c_i32), ("salt", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("iter", _c_p), ("y", _c_p), ("keep_out", _c_p)]


# VGAN_GN_APPLY_GEMM=1: the GraphNorm that ends a critic-engine block applied
# in the next block's projection GEMM (vg_gat_lin_att_gn) instead of by its own
# launch.  Off: measured slower (profiles/r02_ab_gn_apply_gemm.txt).
_GN_APPLY_GEMM = os.environ.get("VGAN_GN_APPLY_GEMM", "0") == "1"


class VgGnJvp(ctypes.Structure):
    """vg_gn_jvp (include/vgan.h): the GraphNorm whose tangent sums the GAT
    tangent pass forms (vg_gat_jvp2_gn_deferred)."""
    _fields_ = [(k, _c_p) for k in ("x", "keep", "g_y", "stats", "weight", "bias", "mean_scale")] + \
               [("eps", _c_f32), ("part", _c_p)]


# VGAN_GN_JVP_FUSE=1: the tangent sweep's GraphNorm sums formed in the GAT
# tangent pass (vg_gat_jvp2_gn_deferred) instead of their own pass.  Off:
# measured slower (k_jvp_rows 94 -> 154 VGPRs; profiles/r02_rejected_gn_jvp_fuse.txt)
_GN_JVP_FUSE = os.environ.get("VGAN_GN_JVP_FUSE", "0") == "1"


class VgChainLayer(ctypes.Structure):
    """vg_chain_layer (include/vgan.h): one layer of vg_linear_chain."""
    _fields_ = [(k, _c_p) for k in ("weight", "bias", "aux", "out")] + \
               [(k, _c_i32) for k in ("ld_aux", "ld_out", "w_trans", "act")]


# VGAN_CHAIN=0: the critic's decoder chains as one vg_gemm launch per layer
# instead of one vg_linear_chain launch per pass (A/B knob)
_CHAIN = os.environ.get("VGAN_CHAIN", "1") == "1"


def linear_chain(x, ldx: int, rows: int, widths, layers, stream) -> bool:
    """vg_linear_chain over ``layers`` (dicts of VgChainLayer fields; device
    pointers as ints / c_void_p); False when the width chain has no kernel
    (the caller runs its per-layer GEMMs).  Only VG_EINVAL (no kernel for
    this width chain / alignment) falls back; a launch error raises."""
    if not _CHAIN:
        return False
    n = len(layers)
    arr = (VgChainLayer * n)()
    for i, l in enumerate(layers):
        for k, v in l.items():
            setattr(arr[i], k, v.value if isinstance(v, ctypes.c_void_p) else v)
    w = (ctypes.c_int32 * (n + 1))(*widths)
    name = "vg_linear_chain_bf16" if _precision == "bf16" else "vg_linear_chain"
    rc = getattr(LIB, name)(x, ldx, rows, w, n, arr, stream)
    if rc == VG_EINVAL:
        return False
    check(rc, name)
    return True


class VgASrc(ctypes.Structure):
    """vg_asrc (include/vgan.h): one column block of vg_gemm_ln_act_ms's A."""
    _fields_ = [("ptr", _c_p), ("ld", _c_i32), ("cols", _c_i32), ("w_col0", _c_i32), ("rows_mod", _c_i32)]


VG_CRITIC_MAX_LAYERS = 8


class VgCriticLinear(ctypes.Structure):
    """vg_critic_linear (include/vgan.h)."""
    _fields_ = [(k, _c_p) for k in ("weight", "bias", "g_weight", "g_bias")] + [("in_", _c_i32), ("out", _c_i32)]


class VgCriticBlock(ctypes.Structure):
    """vg_critic_block (include/vgan.h): one GATConv + GraphNorm block."""
    _fields_ = [(k, _c_p) for k in ("lin_weight", "att_src", "att_dst", "bias", "g_lin_weight", "g_att_src",
                                    "g_att_dst", "g_bias", "gn_weight", "gn_bias", "gn_mean_scale", "g_gn_weight",
                                    "g_gn_bias", "g_gn_mean_scale")] + \
               [("gn_eps", _c_f32), ("slope", _c_f32), ("in_", _c_i32), ("out", _c_i32)]


class VgCriticModel(ctypes.Structure):
    """vg_critic_model (include/vgan.h)."""
    _fields_ = [("n_mlp", _c_i32), ("n_blocks", _c_i32), ("n_dec", _c_i32), ("bf16", _c_i32),
                ("lambda_gp", _c_f32), ("p_drop", _c_f32), ("mlp", VgCriticLinear * VG_CRITIC_MAX_LAYERS),
                ("block", VgCriticBlock * VG_CRITIC_MAX_LAYERS), ("dec", VgCriticLinear * VG_CRITIC_MAX_LAYERS)]


class VgCsrRef(ctypes.Structure):
    """vg_csr_ref (include/vgan.h)."""
    _fields_ = [(k, _c_p) for k in ("row_ptr", "col", "csc_ptr", "csc_slot", "csc_dst", "ell")] + \
               [("num_nodes", _c_i32), ("num_edges", _c_i32), ("ell_width", _c_i32)]


class VgCriticBatch(ctypes.Structure):
    """vg_critic_batch (include/vgan.h)."""
    _fields_ = [("n", _c_i32), ("feat", _c_i32), ("classes", _c_i32)] + \
               [(k, _c_p) for k in ("mvx", "real", "hard", "soft", "seeds4")] + \
               [("g1", VgCsrRef), ("g3", VgCsrRef), ("seed", ctypes.c_uint64), ("iter", _c_p),
                ("eps_salt", ctypes.c_uint32), ("keep_salt", ctypes.c_uint32 * VG_CRITIC_MAX_LAYERS),
                ("gp_counter", _c_p)]


VG_GEN_MAX_LAYERS = 8
VG_GEN_MAX_BLOCKS = 32


class VgGenLnLayer(ctypes.Structure):
    """vg_gen_ln_layer (include/vgan.h): Linear -> LayerNorm -> LeakyReLU."""
    _fields_ = [(k, _c_p) for k in ("weight", "bias", "ln_weight", "ln_bias", "g_weight", "g_bias", "g_ln_weight",
                                    "g_ln_bias")] + [("ln_eps", _c_f32), ("slope", _c_f32), ("in_", _c_i32),
                                                     ("out", _c_i32)]


class VgGenModel(ctypes.Structure):
    """vg_gen_model (include/vgan.h)."""
    _fields_ = [(k, _c_i32) for k in ("n_mfe", "n_mlp", "n_gblocks", "n_dec", "n_dmlp", "n_dblocks", "n_ddec",
                                      "bf16")] + \
               [(k, _c_f32) for k in ("tau", "p_drop_g", "p_drop_d", "lambda_adv", "lambda_label", "lambda_ratio",
                                      "lambda_void", "lambda_far", "dim_scale")] + \
               [("void_class", _c_i32), ("mfe", VgGenLnLayer * VG_GEN_MAX_LAYERS),
                ("mlp", VgGenLnLayer * VG_GEN_MAX_LAYERS), ("gblock", VgCriticBlock * VG_GEN_MAX_BLOCKS),
                ("dec", VgGenLnLayer * VG_GEN_MAX_LAYERS), ("dec_last", VgCriticLinear),
                ("dmlp", VgCriticLinear * VG_GEN_MAX_LAYERS), ("dblock", VgCriticBlock * VG_GEN_MAX_BLOCKS),
                ("ddec", VgCriticLinear * VG_GEN_MAX_LAYERS)]


class VgGenBatch(ctypes.Structure):
    """vg_gen_batch (include/vgan.h)."""
    _fields_ = [(k, _c_i32) for k in ("n", "classes", "mx_w", "vx_w", "mvx_w", "z_dim")] + \
               [(k, _c_p) for k in ("mx", "vx", "mvx", "onehot", "type", "graph_ptr", "site_area")] + \
               [(k, _c_i32) for k in ("num_graphs", "far_col", "dy_col", "dx_col")] + \
               [("g", VgCsrRef), ("seg_rows", _c_i32), ("sync", _c_p), ("one", _c_p), ("seed", ctypes.c_uint64),
                ("iter", _c_p), ("z_salt", ctypes.c_uint32), ("noise_salt", ctypes.c_uint32),
                ("g_keep_salt", ctypes.c_uint32 * VG_GEN_MAX_BLOCKS),
                ("d_keep_salt", ctypes.c_uint32 * VG_GEN_MAX_BLOCKS)]


VG_HGEN_MAX_LAYERS = 8
VG_HGEN_MAX_BLOCKS = 32


class VgHgenLinear(ctypes.Structure):
    """vg_hgen_linear (include/vgan.h): an f16 [Linear, LayerNorm, LeakyReLU] block (or the head)."""
    _fields_ = [("weight", _c_p), ("ldw", _c_i32), ("bias", _c_p), ("gamma", _c_p), ("beta", _c_p),
                ("eps", _c_f32), ("slope", _c_f32), ("in_", _c_i32), ("out", _c_i32)]


class VgHgenBlock(ctypes.Structure):
    """vg_hgen_block (include/vgan.h): an f16 GATConv + GraphNorm block."""
    _fields_ = [("lin_weight", _c_p), ("ldw", _c_i32), ("att_src", _c_p), ("att_dst", _c_p), ("bias", _c_p),
                ("slope", _c_f32), ("gn_weight", _c_p), ("gn_bias", _c_p), ("gn_mean_scale", _c_p),
                ("gn_eps", _c_f32), ("in_", _c_i32), ("out", _c_i32)]


class VgHgenModel(ctypes.Structure):
    """vg_hgen_model (include/vgan.h)."""
    _fields_ = [("n_matched", _c_i32), ("n_mlp", _c_i32), ("n_blocks", _c_i32), ("n_dec", _c_i32),
                ("matched", VgHgenLinear * VG_HGEN_MAX_LAYERS), ("mlp", VgHgenLinear * VG_HGEN_MAX_LAYERS),
                ("block", VgHgenBlock * VG_HGEN_MAX_BLOCKS), ("dec", VgHgenLinear * VG_HGEN_MAX_LAYERS),
                ("head", VgHgenLinear)]


class VgHgenBatch(ctypes.Structure):
    """vg_hgen_batch (include/vgan.h)."""
    _fields_ = [("n", _c_i32), ("copies", _c_i32), ("voxel_dim", _c_i32), ("matched_dim", _c_i32),
                ("z_dim", _c_i32), ("num_edges", _c_i32)] + \
               [(k, _c_p) for k in ("voxel_x", "matched_x", "row_ptr", "col", "taus")] + \
               [("seed", ctypes.c_uint64), ("iter", _c_p), ("advance_iter", _c_i32), ("z_salt", ctypes.c_uint32),
                ("noise_salt", ctypes.c_uint32)]


# name -> (restype, argtypes); every function listed here is declared in include/vgan.h
SIGNATURES = {
    "vg_fold_batch": (ctypes.c_int, [_c_p, _c_i32, _c_p]),
    "vg_fold_split_ws_floats": (_c_i64, [_c_p, _c_i32]),
    "vg_fold_batch_split": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i64, _c_p]),
    "vg_gemm_tn_plan": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_i32, _c_p,
                                       _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_gemm_tn_group": (ctypes.c_int, [_c_p, _c_i32, _c_p]),
    "vg_gat_tile_plan_ints": (_c_i64, [_c_i32, _c_i32]),
    "vg_gat_tile_plan": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p]),
    "vg_build_stamp": (ctypes.c_char_p, []),
    "vg_gat_stage_plan_ints": (_c_i64, [_c_i32, _c_i32]),
    "vg_gat_stage_plan": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p]),
    "vg_gat_aggregate_fwd_staged": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p,
                                                   _c_p, _c_p, _c_p]),
    "vg_gat_ring_plan_ints": (_c_i64, [_c_i32, _c_i32]),
    "vg_gat_ring_plan": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p]),
    "vg_gat_aggregate_fwd_ring": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p,
                                                 _c_p, _c_p, _c_p, _c_p]),
    "vg_gat_ring_tile_rows": (_c_i32, []),
    "vg_gat_ring_gnp_floats": (_c_i64, [_c_i32, _c_i32]),
    "vg_gat_aggregate_fwd_ring_gnp": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32,
                                                     _c_p, _c_p, _c_p, _c_i32, _c_p, _c_p, _c_p]),
    "vg_gat_aggregate_fwd_lds": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p,
                                                _c_p, _c_p, _c_i32, _c_p]),
    "vg_gat_jvp2_plan": (ctypes.c_int, [_c_p] * 5 + [_c_i32] * 3 + [_c_p] * 8 + [_c_f32] + [_c_p] * 7 + [_c_p] * 4),
    "vg_gat_jvp_src_group": (ctypes.c_int, [_c_p, _c_i32, _c_p]),
    "vg_graphnorm_jvp2_sums": (ctypes.c_int, [_c_p, _c_i32, _c_i32] + [_c_p] * 4 + [_c_f32] + [_c_p] * 5),
    "vg_graphnorm_jvp2_fold_src": (ctypes.c_int, [_c_i32, _c_i32] + [_c_p] * 8),
    "vg_graphnorm_jvp2_apply": (ctypes.c_int, [_c_p, _c_i32, _c_i32] + [_c_p] * 4 + [_c_f32] + [_c_p] * 7),
    "vg_gemm_gn_tpart_floats": (_c_i64, [_c_i32, _c_i32]),
    "vg_gemm_gn_bwd": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p,
                                      _c_i32, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p]),
    "vg_graphnorm_bwd_seg_tiles": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p,
                                                  _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_i64, _c_p,
                                                  _c_p]),
    "vg_graphnorm_bwd_sums_offset": (_c_i64, [_c_i32, _c_i32]),
    "vg_gat_bwd_gn": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p,
                                     _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_i32, _c_p, _c_p,
                                     _c_p, _c_p]),
    "vg_gemm_tn_deferred": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_i32, _c_p,
                                           _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_gat_bwd_deferred": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p,
                                           _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p,
                                           _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_ln_act_bwd_deferred": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_p,
                                              _c_p, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_gat_jvp2_deferred": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p,
                                            _c_p, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                            _c_p, _c_p, _c_p, _c_p]),
    "vg_hgemm": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_i32, _c_f32, _c_p,
                                _c_i32, _c_i32, _c_p]),
    "vg_hgemm_ln_act": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_f32,
                                       _c_f32, _c_p, _c_i32, _c_p]),
    "vg_hgat_lin_att": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_i32,
                                       _c_p, _c_p, _c_p]),
    "vg_hgat_gna_max_segments": (_c_i32, []),
    "vg_hgat_lin_att_gn": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p,
                                          _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p]),
    "vg_hgat_fwd": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_i32,
                                   _c_p]),
    "vg_graphnorm_fwd_h": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_f32, _c_p,
                                          _c_i32, _c_p, _c_p, _c_p]),
    "vg_hgat_gnp_rows": (_c_i32, [_c_i32, _c_i32]),
    "vg_hgat_gnp_floats": (_c_i64, [_c_i32, _c_i32]),
    "vg_hgat_fwd_gnp": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p,
                                       _c_i32, _c_i32, _c_p, _c_p]),
    "vg_graphnorm_fwd_h_gnp": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_f32, _c_p,
                                              _c_i32, _c_p, _c_p, _c_i32, _c_p]),
    "vg_rng_fill": (ctypes.c_int, [_c_p, _c_i64, _c_i32, ctypes.c_uint64, _c_p, ctypes.c_uint32, _c_p]),
    "vg_gemm_ln_act_ms": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_i32, _c_p,
                                         _c_p, _c_f32, _c_f32, _c_p, _c_i32, _c_p]),
    "vg_csr_ws_ints": (_c_i64, [_c_i64, _c_i32]),
    "vg_csr_build": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "vg_gat_fwd": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p,
                                  _c_p, _c_p]),
    "vg_gat_att": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "vg_gat_lin_att": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p,
                                      _c_p]),
    "vg_csr_ell": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p]),
    "vg_gat_aggregate_fwd_ell": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p,
                                                _c_f32, _c_p, _c_p, _c_p]),
    "vg_gat_lin_att_gn": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p,
                                         ctypes.POINTER(VgGnApply), _c_p]),
    "vg_graphnorm_stats_gnp": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_f32, _c_p, _c_p]),
    "vg_graphnorm_stats": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_f32, _c_p, _c_p, _c_p]),
    "vg_gat_jvp2_blocks": (_c_i32, [_c_i32, _c_i32]),
    "vg_gat_jvp2_gn_deferred": (ctypes.c_int, [_c_p] * 5 + [_c_i32] * 3 + [_c_p] * 8 + [_c_f32] + [_c_p] * 7 +
                                [ctypes.POINTER(VgGnJvp), _c_p, _c_p, _c_p]),
    "vg_graphnorm_jvp2_part": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p,
                                              _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_p]),
    "vg_linear_chain": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p]),
    "vg_graph_exec_update": (ctypes.c_int, [_c_p, _c_p]),
    "vg_graph_launch": (ctypes.c_int, [_c_p, _c_p]),
    "vg_hgen_arena_bytes": (ctypes.c_int64, [ctypes.POINTER(VgHgenModel), ctypes.POINTER(VgHgenBatch)]),
    "vg_hgen_sweep": (ctypes.c_int, [ctypes.POINTER(VgHgenModel), ctypes.POINTER(VgHgenBatch), _c_p, ctypes.c_int64,
                                     _c_p, _c_p, _c_p]),
    "vg_hgen_graph_create": (_c_p, []),
    "vg_hgen_graph_destroy": (None, [_c_p]),
    "vg_hgen_graph_stats": (ctypes.c_int, [_c_p, ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i32)]),
    "vg_hgen_sweep_graphed": (ctypes.c_int, [_c_p, ctypes.POINTER(VgHgenModel), ctypes.POINTER(VgHgenBatch), _c_p,
                                             ctypes.c_int64, _c_p, _c_p, _c_p]),
    "vg_critic_arena_floats": (ctypes.c_int64, [ctypes.POINTER(VgCriticModel), ctypes.POINTER(VgCriticBatch)]),
    "vg_critic_loss_and_grad": (ctypes.c_int, [ctypes.POINTER(VgCriticModel), ctypes.POINTER(VgCriticBatch), _c_p,
                                               _c_i64, _c_p, _c_p]),
    "vg_gen_arena_floats": (ctypes.c_int64, [ctypes.POINTER(VgGenModel), ctypes.POINTER(VgGenBatch)]),
    "vg_gen_loss_and_grad": (ctypes.c_int, [ctypes.POINTER(VgGenModel), ctypes.POINTER(VgGenBatch), _c_p, _c_i64,
                                            _c_p, _c_p, _c_p]),
    "vg_linear_chain_bf16": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p]),
    "vg_gat_gnp_rows": (_c_i32, [_c_i32, _c_i32]),
    "vg_graphnorm_fwd_gnp_fused": (_c_i32, [_c_i32, _c_i32, _c_i32]),
    "vg_gat_gnp_floats": (_c_i64, [_c_i32, _c_i32]),
    "vg_gat_aggregate_fwd_gnp": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p,
                                                _c_f32, _c_p, _c_p, _c_i32, _c_p, _c_p]),
    "vg_graphnorm_fwd_gnp": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32,
                                            ctypes.c_uint64, _c_p, ctypes.c_uint32, _c_f32, _c_p, _c_p, _c_p, _c_p,
                                            _c_i32, _c_p]),
    "vg_gat_aggregate_fwd": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p,
                                            _c_p]),
    "vg_gat_bwd_ws_floats": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "vg_gat_bwd": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p,
                                  _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "vg_spmm": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_spmm_t": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_sddmm": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_seg_sum": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_p, _c_p]),
    "vg_seg_max": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_p, _c_p]),
    "vg_gather": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p]),
    "vg_scatter_src": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_p, _c_p, _c_p]),
    "vg_graphnorm_ws_floats": (_c_i64, [_c_i32, _c_i32]),
    "vg_graphnorm_fwd": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p]),
    "vg_graphnorm_bwd": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p,
                                        _c_p, _c_p, _c_p, _c_p, _c_p]),
    "vg_type_mean": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_i32, _c_p, _c_p]),
    "vg_gumbel_fwd": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_f32, _c_p, _c_p, _c_p, _c_p]),
    "vg_gumbel_fwd_dev": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_gumbel_bwd": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_i32, _c_i32, _c_f32, _c_p, _c_p]),
    "vg_far_per_graph": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32,
                                        _c_f32, _c_i32, _c_p, _c_p, _c_p]),
    "vg_gen_loss_ws_floats": (_c_i64, [_c_i32, _c_i32]),
    "vg_gen_loss_fwd": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_f32, _c_f32,
                                       _c_f32, _c_f32, _c_f32, _c_p, _c_p, _c_p]),
    "vg_gen_loss_bwd": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_confusion": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_p]),
    "vg_gemm": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_i32, _c_p, _c_i32, _c_i32,
                               _c_i32, _c_i32, _c_p]),
    "vg_gemm_tn_ws_floats": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "vg_gemm_tn": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_i32, _c_p,
                                  _c_p]),
    "vg_gemm_tn_ex": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_i32,
                                     _c_i32, _c_p, _c_p]),
    "vg_gat_bwd_ex": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p,
                                     _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_i32, _c_p,
                                     _c_p]),
    "vg_gat_jvp2_ws_floats": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "vg_gat_jvp2": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p,
                                   _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "vg_gat_jvp2_ex": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p,
                                      _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                      _c_p]),
    "vg_graphnorm_seg_ws_floats": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "vg_graphnorm_fwd_seg": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p,
                                            _c_p, _c_p, _c_p]),
    "vg_graphnorm_fwd_drop": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_f32, ctypes.c_uint64,
                                             _c_p, ctypes.c_uint32, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "vg_graphnorm_bwd_seg": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p,
                                            _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_i64, _c_p, _c_p, _c_p]),
    "vg_graphnorm_jvp2": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p,
                                         _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "vg_gemm_ln_act": (ctypes.c_int, [_c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_f32, _c_f32,
                                      _c_p, _c_p, _c_p, _c_p, _c_p]),
    "vg_ln_act_fwd": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_f32, _c_f32, _c_p, _c_p, _c_p, _c_p]),
    "vg_ln_act_bwd_ws_floats": (_c_i64, [_c_i32]),
    "vg_ln_act_bwd": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_f32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                     _c_i32, _c_p, _c_p]),
    "vg_critic_input": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p]),
    "vg_critic_input_drawn": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_p, _c_p, ctypes.c_uint64, _c_p,
                                             ctypes.c_uint32, _c_i32, _c_i32, _c_p, _c_p]),
    "vg_iter_begin": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_i64, _c_p]),
    "vg_gp_head_ws_floats": (_c_i64, [_c_i32]),
    "vg_gp_head": (ctypes.c_int, [_c_p, _c_i32, _c_i32, _c_p, _c_f32, _c_p, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "vg_adam_dev": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_i64, ctypes.c_double, ctypes.c_double, _c_f32, _c_f32,
                                   _c_p, _c_p, _c_p]),
    "vg_adam": (ctypes.c_int, [_c_p, _c_p, _c_p, _c_p, _c_i64, _c_f32, _c_f32, _c_f32, _c_f32, _c_f32, _c_f32,
                               _c_f32, _c_p]),
}

# the dense products of the path, each also exported with bf16 operands
# (include/vgan.h, "bf16 training"); same signatures
DENSE = ("vg_gemm", "vg_gemm_tn", "vg_gemm_tn_deferred", "vg_gemm_tn_plan", "vg_gemm_ln_act", "vg_gemm_ln_act_ms",
         "vg_gat_lin_att", "vg_gemm_gn_bwd")
for _name in DENSE:
    SIGNATURES[_name + "_bf16"] = SIGNATURES[_name]


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). The HIP library is required; there is no fallback."
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _check_stamp(lib)
    return lib


def source_hash(csrc: str) -> Optional[str]:
    """The hash csrc/Makefile stamps into the library: sha256 over csrc/*.hip,
    csrc/*.h and include/vgan.h concatenated in sorted path order (make's
    $(sort) of the relative paths), first 16 hex digits.  None when the
    sources are not in the tree."""
    import glob
    import hashlib

    if not os.path.isdir(csrc):
        return None
    rel = [os.path.basename(p) for p in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h"))]
    rel.append("../../include/vgan.h")
    h = hashlib.sha256()
    for r in sorted(rel):
        path = os.path.normpath(os.path.join(csrc, r))
        if not os.path.exists(path):
            return None
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _check_stamp(lib) -> None:
    """A library built from other sources than the tree's fails loudly (a
    stale prebuilt .so would otherwise run old kernels under new tests).
    An explicit VGAN_LIB (an A/B build of other sources, tools/ab_libs.sh)
    is exempt."""
    if os.environ.get("VGAN_LIB"):
        return
    stamp = lib.vg_build_stamp().decode()
    want = source_hash(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc"))
    if want is not None and stamp.split(" ")[0] != want:
        raise ImportError(f"{LIB_PATH} was built from other sources (stamp {stamp.split(' ')[0]}, tree {want}): "
                          "rebuild it (make -C building-gan-graph-conditioned-architectural-volume-generation_amd/csrc)")


def build_stamp() -> str:
    """'<source hash> <hipcc version>' of the loaded library."""
    return LIB.vg_build_stamp().decode()


LIB = _load()


# Operand precision of the dense products: "f32" (the reference's) or "bf16"
# (configs[2]: bf16 operands, f32 accumulation and outputs).  A process-wide
# setting rather than a thread-local one: autograd runs the backward of the
# HIP ops on its own device thread, which must see the same precision.
PRECISIONS = ("f32", "bf16")
_precision = "f32"


def gemm_precision() -> str:
    return _precision


def set_gemm_precision(p: str) -> None:
    global _precision
    if p not in PRECISIONS:
        raise ValueError(f"gemm precision must be one of {PRECISIONS}, not {p!r}")
    _precision = p


class gemm_precision_scope:
    """``with gemm_precision_scope("bf16"): ...`` -- set, then restore."""

    def __init__(self, p: str):
        self.p = p

    def __enter__(self):
        self.prev = _precision
        set_gemm_precision(self.p)
        return self

    def __exit__(self, *exc):
        set_gemm_precision(self.prev)
        return False


def dense(name: str):
    """Entry point of the dense product ``name`` (one of DENSE) in the current precision."""
    return getattr(LIB, name + "_bf16" if _precision == "bf16" else name)


def ptr(t: Optional[torch.Tensor]):
    """A tensor's device address for a c_void_p argument: a plain int (ctypes
    converts it itself; wrapping every pointer in a c_void_p object cost ~0.4
    us each, ~4 us per ABI call of the eager paths' ~10 pointers), None for NULL."""
    return None if t is None else t.data_ptr()


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


_SYNC = {}


# measured slower at batch 32 (16.1 vs 18.2 ms/step: one contended counter for
# ~640 blocks), so off unless VGAN_LAST_BLOCK_FOLD=1
_LAST_BLOCK = os.environ.get("VGAN_LAST_BLOCK_FOLD", "0") == "1"


def sync_counter(device: torch.device):
    """Persistent zeroed int32 device counter per (device, current stream) for
    the kernels' last-block fold (left at 0 by every launch); None (separate
    finalize launches) when VGAN_LAST_BLOCK_FOLD=0."""
    if not _LAST_BLOCK:
        return None
    key = (torch.device(device), torch.cuda.current_stream(device).cuda_stream)
    t = _SYNC.get(key)
    if t is None:
        t = _SYNC[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return ptr(t)


def check(rc: int, name: str) -> None:
    if rc != 0:
        what = "invalid argument" if rc == VG_EINVAL else f"hipError {rc}"
        raise RuntimeError(f"{name} failed: {what}")


def require_cuda(*tensors: Optional[torch.Tensor]) -> None:
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("vgan HIP ops require tensors on a ROCm device (no CPU fallback)")
        if not t.is_contiguous():
            raise RuntimeError("vgan HIP ops require contiguous tensors")


class FoldCollector:
    """Collects the parameter-gradient folds of one backward (the *_deferred
    ABI calls) and runs them in as few vg_fold_batch launches as possible.
    Folds into the same destination merge into one two-source fold, applied
    in call order ((out + first) + second, as the immediate folds would); the
    partial workspaces are kept alive until the batch is enqueued."""

    def __init__(self):
        self.folds = []
        self.keep = []
        self.products = []
        self.jvp_src = []

    def call(self, fn, args_before_stream, stream, keep=(), name="deferred"):
        arr = (VgFold * 3)()
        n = ctypes.c_int32(0)
        check(fn(*args_before_stream, arr, ctypes.byref(n), stream), name)
        for i in range(n.value):
            self.folds.append(VgFold.from_buffer_copy(arr[i]))
        self.keep.extend(keep)

    def tn(self, args_before_outputs, stream, keep=()):
        """A weight-gradient product (vg_gemm_tn_plan's arguments up to the
        workspace; accumulate into C / db).  It runs at flush() in one
        vg_gemm_tn_group launch with the backward's other products, before
        the folds; ``keep`` holds A, B and the workspace until then."""
        if not _TN_GROUP:
            self.call(dense("vg_gemm_tn_deferred"), args_before_outputs, stream, keep=keep, name="vg_gemm_tn_deferred")
            return
        prod = VgTn()
        arr = (VgFold * 2)()
        n = ctypes.c_int32(0)
        check(dense("vg_gemm_tn_plan")(*args_before_outputs, ctypes.byref(prod), arr, ctypes.byref(n)),
              "vg_gemm_tn_plan")
        self.products.append(prod)
        for i in range(n.value):
            self.folds.append(VgFold.from_buffer_copy(arr[i]))
        self.keep.extend(keep)

    def jvp(self, args_before_outputs, stream, keep=()):
        """vg_gat_jvp2 with its folds deferred and its source pass (dQ/dh
        injections) described for ONE grouped launch by run_jvp_src();
        ``keep`` holds h, u, g_out and the workspace until then."""
        arr = (VgFold * 2)()
        n = ctypes.c_int32(0)
        if not _JVP_GROUP:
            check(LIB.vg_gat_jvp2_deferred(*args_before_outputs, arr, ctypes.byref(n), stream), "vg_gat_jvp2_deferred")
        else:
            src = VgJvpSrc()
            check(LIB.vg_gat_jvp2_plan(*args_before_outputs, arr, ctypes.byref(n), ctypes.byref(src), stream),
                  "vg_gat_jvp2_plan")
            if src.shape >= 0:
                self.jvp_src.append(src)
        for i in range(n.value):
            self.folds.append(VgFold.from_buffer_copy(arr[i]))
        self.keep.extend(keep)

    def jvp_gn(self, args_before_outputs, gn: "VgGnJvp", stream, keep=()):
        """vg_gat_jvp2_gn_deferred: ``jvp`` (source pass run here) that also
        writes the GraphNorm tangent sums of ``gn`` into gn.part."""
        arr = (VgFold * 2)()
        n = ctypes.c_int32(0)
        check(LIB.vg_gat_jvp2_gn_deferred(*args_before_outputs, ctypes.byref(gn), arr, ctypes.byref(n), stream),
              "vg_gat_jvp2_gn_deferred")
        for i in range(n.value):
            self.folds.append(VgFold.from_buffer_copy(arr[i]))
        self.keep.extend(keep)

    def run_jvp_src(self, stream) -> None:
        """The described source passes, in one launch per VG_JVP_GROUP_MAX."""
        for i in range(0, len(self.jvp_src), VG_JVP_GROUP_MAX):
            part = self.jvp_src[i:i + VG_JVP_GROUP_MAX]
            arr = (VgJvpSrc * len(part))(*part)
            check(LIB.vg_gat_jvp_src_group(arr, len(part), stream), "vg_gat_jvp_src_group")
        self.jvp_src = []

    def _launch_products(self, stream) -> None:
        for bf in (0, 1):
            prods = [p for p in self.products if p.bf16 == bf]
            for i in range(0, len(prods), VG_TN_GROUP_MAX):
                part = prods[i:i + VG_TN_GROUP_MAX]
                arr = (VgTn * len(part))(*part)
                check(LIB.vg_gemm_tn_group(arr, len(part), stream), "vg_gemm_tn_group")
        self.products = []

    def flush(self, stream) -> None:
        self.run_jvp_src(stream)  # (their att_src partials feed folds)
        # the grouped products first: their partials feed the folds
        self._launch_products(stream)
        batches, cur, where = [], [], {}
        for f in self.folds:
            j = where.get(f.out)
            if j is not None:
                g = cur[j]
                if (g.nsrc == 1 and f.nsrc == 1 and f.accumulate and (g.width, g.k, g.ldo) == (f.width, f.k, f.ldo)):
                    g.src[1] = f.src[0]
                    g.nsrc = 2
                    continue
                batches.append(cur)  # cannot merge: later batch, so the two never race
                cur, where = [], {}
            if len(cur) == _FOLD_BATCH:
                batches.append(cur)
                cur, where = [], {}
            where[f.out] = len(cur)
            cur.append(f)
        if cur:
            batches.append(cur)
        for b in batches:
            arr = (VgFold * len(b))(*b)
            need = int(LIB.vg_fold_split_ws_floats(arr, len(b))) if _FOLD_SPLIT else 0
            if need > 0:  # the chunk sums' workspace, on the current stream (the folds' own: stream-ordered reuse)
                ws = torch.empty(need, dtype=torch.float32, device="cuda")
                check(LIB.vg_fold_batch_split(arr, len(b), ws.data_ptr(), need, stream), "vg_fold_batch_split")
            else:
                check(LIB.vg_fold_batch(arr, len(b), stream), "vg_fold_batch")
        self.folds, self.keep = [], []
