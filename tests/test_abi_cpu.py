"""The C-ABI library loads and exports exactly what include/vgan.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from parity_util import PKG_ROOT, ROOT

HEADER = os.path.join(ROOT, "include", "vgan.h")
LIB = os.path.join(PKG_ROOT, "vgan", "libvgan_hip.so")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vg_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_functions():
    syms = header_symbols()
    assert "vg_gat_fwd" in syms and "vg_csr_build" in syms and len(syms) >= 20


def test_library_exports_every_header_symbol():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (vg_[a-z0-9_]+)$", out, flags=re.M))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(LIB)
    for s in header_symbols():
        assert hasattr(lib, s)


def test_binding_table_matches_header():
    from vgan import _lib

    assert sorted(_lib.SIGNATURES) == header_symbols()


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", LIB], capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob


def test_workspace_queries_are_host_only():
    from vgan._lib import LIB as lib

    assert lib.vg_csr_ws_ints(100, 10) == 4 * 10 + 100 + 10
    assert lib.vg_graphnorm_ws_floats(1000, 16) >= 2 * 16
    # the one-launch GraphNorm forward: narrow layers at batch 32, not the wide ones
    assert lib.vg_graphnorm_fwd_gnp_fused(12600, 16, 64) == 1
    assert lib.vg_graphnorm_fwd_gnp_fused(12600, 128, 8) == 0
    assert lib.vg_graphnorm_fwd_gnp_fused(12600, 2, 32) == 0
    # the f16 aggregation's partial blocks: kBlock / lanes per row of the width
    assert [lib.vg_hgat_gnp_rows(1000, ld) for ld in (8, 16, 32, 64, 128)] == [128, 64, 128, 64, 32]
    assert lib.vg_hgat_gnp_rows(1000, 24) == 0 and lib.vg_hgat_gnp_floats(1000, 24) == 0
    assert lib.vg_hgat_gna_max_segments() == 16
    assert lib.vg_hgat_gnp_floats(1000, 128) >= (1000 // 32 + 1) * 2 * 128 * 3


def test_hgen_arena_sizing_is_host_only():
    """vg_hgen_arena_bytes runs the f16 sweep engine's orchestration dry (no
    launch, no device pointer read): a consistent generator description sizes
    a 256-byte-granular arena that grows with the batch; an MLP whose input
    width does not match the row buffer, or an empty batch, is refused."""
    import ctypes as ct

    from vgan._lib import LIB as lib, VgHgenBatch, VgHgenModel

    md = VgHgenModel()
    md.n_matched, md.n_mlp, md.n_blocks, md.n_dec = 1, 1, 2, 1
    fl, vd, zd, hl, hg = 17, 12, 128, 32, 64

    def lin(d, i, o, ln=True):
        d.weight, d.ldw, d.bias = 1, (i + 7) // 8 * 8, 1
        d.gamma = d.beta = 1 if ln else None
        d.eps, d.slope, d.in_, d.out = 1e-5, 0.2, i, o

    lin(md.matched[0], fl, hl)
    lin(md.mlp[0], hl + vd + zd, hg)
    for b, (i, o) in enumerate(((hg, 32), (32, 8))):
        d = md.block[b]
        d.lin_weight, d.ldw, d.att_src, d.att_dst, d.bias, d.slope = 1, (i + 7) // 8 * 8, 1, 1, 1, 0.2
        d.gn_weight = d.gn_bias = d.gn_mean_scale = 1
        d.gn_eps, d.in_, d.out = 1e-5, i, o
    lin(md.dec[0], 8 + hg + hl + vd + zd, 64)
    lin(md.head, 64, 7, ln=False)

    def size(n, copies):
        bt = VgHgenBatch()
        bt.n, bt.copies, bt.voxel_dim, bt.matched_dim, bt.z_dim, bt.num_edges = n, copies, vd, fl, zd, 9 * n
        return int(lib.vg_hgen_arena_bytes(ct.byref(md), ct.byref(bt)))

    a, b = size(1000, 1), size(1000, 10)
    assert a > 0 and b > a and a % 256 == 0 and b % 256 == 0
    assert size(0, 10) < 0
    md.mlp[0].in_ = hl + vd  # not the [em | voxel.x | z] width
    assert size(1000, 10) < 0


def test_gen_arena_sizing_is_host_only():
    """vg_gen_arena_floats runs the native generator iteration's schedule dry
    (no launch, no device pointer read): the reference's layer pattern sizes
    an arena that grows with the batch; a decoder input width that is not
    [enc | x | em | voxel.x | z], a batch under 64 nodes or segment rows
    other than the batch's are refused (the Python schedule runs them)."""
    import ctypes as ct

    from vgan._lib import LIB as lib, VgGenBatch, VgGenModel

    K, fl, vd, zd, h, F = 7, 17, 12, 128, 128, 29
    md = VgGenModel()
    md.n_mfe, md.n_mlp, md.n_gblocks, md.n_dec = 2, 2, 4, 2
    md.n_dmlp, md.n_dblocks, md.n_ddec = 2, 2, 2
    md.tau, md.p_drop_g, md.p_drop_d = 1.0, 0.2, 0.2

    def ln(d, i, o):
        d.in_, d.out, d.ln_eps, d.slope = i, o, 1e-5, 0.2

    def blk(d, i, o):
        d.in_, d.out, d.gn_eps, d.slope = i, o, 1e-5, 0.2

    ln(md.mfe[0], fl, h)
    ln(md.mfe[1], h, h)
    ln(md.mlp[0], h + vd + zd, h)
    ln(md.mlp[1], h, h)
    for b, (i, o) in enumerate(((h, 64), (64, 2), (2, 1), (1, 8))):
        blk(md.gblock[b], i, o)
    ln(md.dec[0], 8 + h + h + vd + zd, 64)
    ln(md.dec[1], 64, 16)
    md.dec_last.in_, md.dec_last.out = 16, K
    md.dmlp[0].in_, md.dmlp[0].out = F + K, 64
    md.dmlp[1].in_, md.dmlp[1].out = 64, 64
    blk(md.dblock[0], 64, 32)
    blk(md.dblock[1], 32, 16)
    md.ddec[0].in_, md.ddec[0].out = 16, 8
    md.ddec[1].in_, md.ddec[1].out = 8, 1

    def size(n):
        bt = VgGenBatch()
        bt.n, bt.classes, bt.mx_w, bt.vx_w, bt.mvx_w, bt.z_dim = n, K, fl, vd, F, zd
        bt.num_graphs, bt.seg_rows = 4, n
        bt.g.num_nodes, bt.g.num_edges = n, 9 * n
        return int(lib.vg_gen_arena_floats(ct.byref(md), ct.byref(bt))), bt

    (a, _), (b, bt) = size(1000), size(4000)
    assert a > 0 and b > a and a % 64 == 0
    assert size(32)[0] < 0
    bt.seg_rows = 2000
    assert int(lib.vg_gen_arena_floats(ct.byref(md), ct.byref(bt))) < 0
    md.dec[0].in_ = h + h + vd + zd  # not the [enc | x | em | voxel.x | z] width
    assert size(1000)[0] < 0
    VG_EINVAL = -1
    assert lib.vg_gen_loss_and_grad(ct.byref(md), ct.byref(bt), None, 0, None, None, None) == VG_EINVAL


def test_ops_refuse_cpu_tensors():
    import torch

    from vgan import ops

    with pytest.raises(RuntimeError, match="ROCm device"):
        ops.CSR(torch.zeros(2, 3, dtype=torch.long), 4)


def test_build_stamp_matches_tree_and_stale_library_is_refused():
    """libvgan_hip.so carries the hash of the sources it was built from; the
    binding recomputes it from the tree, and a library built from other
    sources (a stale prebuilt .so) is refused at import."""
    import vgan._lib as L

    stamp = L.build_stamp()
    assert stamp.split(" ")[0] == L.source_hash(os.path.join(os.path.dirname(L.__file__), "..", "csrc"))
    assert "HIP version" in stamp

    class Stale:
        @staticmethod
        def vg_build_stamp():
            return b"0123456789abcdef HIP version: 0"

    with pytest.raises(ImportError, match="other sources"):
        L._check_stamp(Stale())


def test_graphed_sweep_refuses_bad_arguments_host_only():
    """vg_hgen_sweep_graphed / vg_hgen_graph_stats check their arguments on
    the host before any runtime call: a NULL handle, model or arena is
    VG_EINVAL (no capture started, no device touched)."""
    import ctypes as ct

    from vgan._lib import LIB as lib, VgHgenBatch, VgHgenModel

    VG_EINVAL = -1
    md, bt = VgHgenModel(), VgHgenBatch()
    assert lib.vg_hgen_sweep_graphed(None, ct.byref(md), ct.byref(bt), None, 0, None, None, None) == VG_EINVAL
    assert lib.vg_hgen_sweep_graphed(1, None, ct.byref(bt), 256, 0, None, None, None) == VG_EINVAL
    assert lib.vg_hgen_sweep_graphed(1, ct.byref(md), ct.byref(bt), None, 0, None, None, None) == VG_EINVAL
    a, b = ct.c_int32(7), ct.c_int32(7)
    assert lib.vg_hgen_graph_stats(None, ct.byref(a), ct.byref(b)) == VG_EINVAL
    lib.vg_hgen_graph_destroy(None)  # a NULL handle is a no-op
    # the arena query's errors are negative, never a size a caller could allocate
    assert lib.vg_hgen_arena_bytes(None, ct.byref(bt)) == VG_EINVAL
    assert lib.vg_hgen_arena_bytes(ct.byref(md), None) == VG_EINVAL
    assert lib.vg_hgen_arena_bytes(ct.byref(md), ct.byref(bt)) < 0  # an empty model: n_matched = 0


def test_gemm_act_codes_checked_host_only():
    """vg_gemm refuses an act code outside 0-4, and act 3 / 4 (mask, add)
    without aux, before any launch."""
    from vgan._lib import LIB as lib

    VG_EINVAL = -1
    for act, aux in ((5, 1), (-1, 1), (3, None), (4, None)):
        assert lib.vg_gemm(1, 8, 1, 8, 1, None, act, aux, 8, 1, 8, 8, 8, 8, None) == VG_EINVAL, act


def test_fold_batch_limit_matches_header():
    """vgan._lib.VG_FOLD_MAX (the Python batcher's limit) is the header's."""
    import re

    from vgan import _lib

    hdr = open(os.path.join(ROOT, "include", "vgan.h")).read()
    assert int(re.search(r"#define VG_FOLD_MAX (\d+)", hdr).group(1)) == _lib.VG_FOLD_MAX
    assert 1 <= _lib._FOLD_BATCH <= _lib.VG_FOLD_MAX
