"""The explicit WGAN-GP critic engine (vgan/critic.py) and its kernels.

Kernels are checked against torch autograd on the oracle's ops in float64
(tests/critic_ref.py units); the engine against (i) the four-pass reference in
float64 and (ii) plain double backward of the oracle discriminator, both on the
engine's own dropout masks and eps.  Tolerances: kernels 1e-5 relative to the
output scale (f32 summation order), engine loss 1e-5, gradients grads_close
at 1e-3.
"""
import pytest
import torch

import critic_ref as CR
from oracle import pyg
from oracle import reference as R
from parity_util import grads_close, rel_err
from vgan import ops, synth
from vgan._lib import LIB, check, ptr, stream_handle, sync_counter
from vgan.config import Configuration
from vgan.graph import GraphBatch

pytestmark = pytest.mark.gpu


def _graph(numbers=(1, 2, 3), stress=False):
    items = [(synth.make_stress_building(777, n, F=3, Y=9, X=9) if stress else synth.make_building(777, n))
             for n in numbers]
    return (GraphBatch.from_data_list([l for l, _ in items]), GraphBatch.from_data_list([v for _, v in items]))


def _close(got, ref, tol=1e-5):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    scale = max(ref.abs().max().item(), 1e-12)
    return (got - ref).abs().max().item() <= tol * scale, (got - ref).abs().max().item() / scale


# ------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("sym", ["vg_gemm", "vg_gemm_bf16"])
@pytest.mark.parametrize("bt", [0, 1])
def test_gemm_add_epilogue_equals_product_then_add(cuda, sym, bt):
    """act 4 (C = A op(B) + aux, aux a strided column window): bit-exact with
    the act-0 product followed by torch's add_ -- the generator engine's
    summed adjoints (genstep.py) rely on it."""
    g = torch.Generator().manual_seed(1)
    n, k, m, ld = 1000, 96, 40, 72
    A = torch.randn(n, k, generator=g).to(cuda)
    W = torch.randn(*((m, k) if bt else (k, m)), generator=g).to(cuda)
    wide = torch.randn(n, ld, generator=g).to(cuda)  # aux = wide[:, 9:9+m]
    C0, C4 = torch.empty(n, m, device=cuda), torch.empty(n, m, device=cuda)
    st = stream_handle(cuda)
    fn = getattr(LIB, sym)
    ldb = k if bt else m
    check(fn(ptr(A), k, ptr(W), ldb, bt, None, 0, None, 0, ptr(C0), m, n, m, k, st), sym)
    check(fn(ptr(A), k, ptr(W), ldb, bt, None, 4, wide.data_ptr() + 4 * 9, ld, ptr(C4), m, n, m, k, st), sym)
    assert torch.equal(C4, C0.add_(wide[:, 9:9 + m]))
    assert fn(ptr(A), k, ptr(W), ldb, bt, None, 4, None, 0, ptr(C4), m, n, m, k, st) != 0  # aux required


def test_gemm_mask_epilogue_and_strided_accumulate(cuda):
    g = torch.Generator().manual_seed(0)
    n, k, m = 300, 37, 45
    A = torch.randn(n, k, generator=g, dtype=torch.float64)
    W = torch.randn(m, k, generator=g, dtype=torch.float64)
    aux = torch.randn(n, m, generator=g, dtype=torch.float64)
    Ad, Wd, auxd = (t.float().to(cuda) for t in (A, W, aux))
    C = torch.empty(n, m, device=cuda)
    st = stream_handle(cuda)
    check(LIB.vg_gemm(ptr(Ad), k, ptr(Wd), k, 1, None, 3, ptr(auxd), m, ptr(C), m, n, m, k, st), "vg_gemm")
    ok, err = _close(C, (A @ W.T) * (aux > 0))
    assert ok, err
    # C[:, 5:5+k] of a wider [m, 60] buffer += A2^T B, with column sums
    A2 = torch.randn(n, m, generator=g, dtype=torch.float64)
    B2 = torch.randn(n, k, generator=g, dtype=torch.float64)
    base = torch.randn(m, 60, generator=g, dtype=torch.float64)
    db0 = torch.randn(m, generator=g, dtype=torch.float64)
    out, db = base.float().to(cuda), db0.float().to(cuda)
    ws = torch.empty(int(LIB.vg_gemm_tn_ws_floats(n, m, k)), device=cuda)
    import ctypes
    A2d, B2d = A2.float().to(cuda), B2.float().to(cuda)  # keep alive: the kernel reads them
    check(LIB.vg_gemm_tn(ptr(A2d), m, ptr(B2d), k, n, m, k,
                         ctypes.c_void_p(out.data_ptr() + 4 * 5), 60, ptr(db), 1, ptr(ws), st), "vg_gemm_tn")
    exp = base.clone()
    exp[:, 5:5 + k] += A2.T @ B2
    ok, err = _close(out, exp)
    bad = ((out.cpu().double() - exp).abs() > 1e-3).nonzero()[:8].tolist()
    assert ok, (err, bad)
    ok, err = _close(db, db0 + A2.sum(0))
    assert ok, err


# ------------------------------------------------------------------- GAT
def _gat_inputs(C, stress, seed=0):
    _, vox = _graph(stress=stress)
    n = vox.num_nodes
    g = torch.Generator().manual_seed(seed)
    d = torch.float64
    h = torch.randn(n, C, generator=g, dtype=d)
    u = torch.randn(n, C, generator=g, dtype=d)
    go = torch.randn(n, C, generator=g, dtype=d)
    P = {"as": torch.randn(1, 1, C, generator=g, dtype=d), "ad": torch.randn(1, 1, C, generator=g, dtype=d),
         "bias": torch.randn(C, generator=g, dtype=d)}
    return vox.edge_index, n, h, u, go, P


@pytest.mark.parametrize("C", [1, 3, 8, 16, 32, 64, 100])
@pytest.mark.parametrize("stress", [False, True])
def test_gat_jvp2_matches_autograd(cuda, C, stress):
    ei, n, h, u, go, P = _gat_inputs(C, stress)
    ju, hinj, pg = CR.Unit("gat", CR.gat_fn(ei, n), ["as", "ad", "bias"]).jvp2(h, u, go, P)
    csr = ops.CSR(ei.to(cuda), n)
    hd, ud, god = (t.float().to(cuda).contiguous() for t in (h, u, go))
    vs, vd, b = (P[k].float().to(cuda).reshape(-1).contiguous() for k in ("as", "ad", "bias"))
    out = torch.empty(n, C, device=cuda)
    alpha = torch.empty(csr.num_edges, device=cuda)
    a_s, a_d = torch.empty(n, device=cuda), torch.empty(n, device=cuda)
    st = stream_handle(cuda)
    check(LIB.vg_gat_fwd(ptr(csr.row_ptr), ptr(csr.col), n, C, ptr(hd), ptr(vs), ptr(vd), ptr(b), 0.2, ptr(out),
                         ptr(alpha), ptr(a_s), ptr(a_d), st), "vg_gat_fwd")
    u_out, h_inj = torch.empty(n, C, device=cuda), torch.empty(n, C, device=cuda)
    gb0 = torch.Generator().manual_seed(21)
    g_as0, g_ad0 = (torch.randn(C, generator=gb0, dtype=torch.float64).float().double() for _ in range(2))
    g_as, g_ad = g_as0.float().to(cuda), g_ad0.float().to(cuda)
    ws = torch.empty(int(LIB.vg_gat_jvp2_ws_floats(n, csr.num_edges, C)), device=cuda)
    check(LIB.vg_gat_jvp2(ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot), ptr(csr.csc_dst), n,
                          csr.num_edges, C, ptr(hd), ptr(ud), ptr(god), ptr(vs), ptr(vd), ptr(a_s), ptr(a_d),
                          ptr(alpha), 0.2, ptr(u_out), ptr(h_inj), ptr(g_as), ptr(g_ad), ptr(ws), st), "vg_gat_jvp2")
    # parameter gradients: the accumulated increment at its own scale
    for got, ref in ((u_out, ju), (h_inj, hinj), (g_as.double().cpu() - g_as0, pg["as"].reshape(-1)),
                     (g_ad.double().cpu() - g_ad0, pg["ad"].reshape(-1))):
        ok, err = _close(got, ref, 2e-5)
        assert ok, err
    assert pg["bias"].abs().max().item() == 0.0


@pytest.mark.parametrize("C", [4, 16, 64])
def test_gat_bwd_ex_injection_and_accumulate(cuda, C):
    ei, n, h, _, go, P = _gat_inputs(C, False, seed=1)
    dx, pg = CR.Unit("gat", CR.gat_fn(ei, n), ["as", "ad", "bias"]).vjp(h, go, P)
    csr = ops.CSR(ei.to(cuda), n)
    hd, god = h.float().to(cuda), go.float().to(cuda)
    vs, vd, b = (P[k].float().to(cuda).reshape(-1).contiguous() for k in ("as", "ad", "bias"))
    out = torch.empty(n, C, device=cuda)
    alpha = torch.empty(csr.num_edges, device=cuda)
    a_s, a_d = torch.empty(n, device=cuda), torch.empty(n, device=cuda)
    st = stream_handle(cuda)
    check(LIB.vg_gat_fwd(ptr(csr.row_ptr), ptr(csr.col), n, C, ptr(hd), ptr(vs), ptr(vd), ptr(b), 0.2, ptr(out),
                         ptr(alpha), ptr(a_s), ptr(a_d), st), "vg_gat_fwd")
    row0 = n // 3
    inj = torch.randn(n - row0, C, dtype=torch.float64)
    gb0 = torch.Generator().manual_seed(22)
    base = [torch.randn(C, generator=gb0, dtype=torch.float64).float().double() for _ in range(3)]
    gs = [t.float().to(cuda) for t in base]
    g_h = torch.empty(n, C, device=cuda)
    ws = torch.empty(int(LIB.vg_gat_bwd_ws_floats(n, csr.num_edges, C)), device=cuda)
    injd = inj.float().to(cuda)
    check(LIB.vg_gat_bwd_ex(ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot), ptr(csr.csc_dst), n,
                            csr.num_edges, C, ptr(hd), ptr(vs), ptr(vd), ptr(a_s), ptr(a_d), ptr(alpha), ptr(god), 0.2,
                            ptr(g_h), ptr(gs[0]), ptr(gs[1]), ptr(gs[2]), 1, ptr(injd), row0, ptr(ws),
                            st), "vg_gat_bwd_ex")
    exp = dx.clone()
    exp[row0:] += inj
    assert _close(g_h, exp)[0]
    for got, b0, k in zip(gs, base, ("as", "ad", "bias")):
        assert _close(got.double().cpu() - b0, pg[k].reshape(-1), 2e-5)[0], k
    # no parameter gradients: only g_h
    g_h2 = torch.empty(n, C, device=cuda)
    check(LIB.vg_gat_bwd_ex(ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot), ptr(csr.csc_dst), n,
                            csr.num_edges, C, ptr(hd), ptr(vs), ptr(vd), ptr(a_s), ptr(a_d), ptr(alpha), ptr(god), 0.2,
                            ptr(g_h2), None, None, None, 0, None, 0, ptr(ws), st), "vg_gat_bwd_ex")
    assert _close(g_h2, dx)[0]


# ------------------------------------------------------------- GraphNorm
def _gn_inputs(n, C, seed=0):
    g = torch.Generator().manual_seed(seed)
    d = torch.float64
    x = torch.randn(n, C, generator=g, dtype=d) * 2 + 0.4
    P = {"w": torch.rand(C, generator=g, dtype=d) + 0.5, "b": torch.randn(C, generator=g, dtype=d) * 0.3,
         "s": torch.rand(C, generator=g, dtype=d)}
    keep = (torch.rand(n, C, generator=g) > 0.2).to(d) / 0.8
    return x, P, keep


@pytest.mark.parametrize("last_block_fold", [True, False])
@pytest.mark.parametrize("C", [1, 8, 32, 64, 128, 200])
def test_graphnorm_segments_fwd_bwd_injection(cuda, C, last_block_fold):
    S, n = 3, 700
    x, P, keep = _gn_inputs(S * n, C)
    gy = torch.randn(S * n, C, dtype=torch.float64)
    ys, gxs = [], []
    pgs = {k: torch.zeros_like(v) for k, v in P.items()}
    for s in range(S):
        rows = slice(s * n, (s + 1) * n)
        unit = CR.Unit("gn", CR.gnrd_fn(keep[rows]), ["w", "b", "s"])
        ys.append(unit.fwd(x[rows], P))
        gx, pg = unit.vjp(x[rows], gy[rows], P)
        gxs.append(gx)
        for k in pgs:
            pgs[k] += pg[k]
    dev = [t.float().to(cuda).contiguous() for t in (x, keep, gy, P["w"], P["b"], P["s"])]
    xd, kd, gyd, wd, bd, sd = dev
    st = stream_handle(cuda)
    y = torch.empty(S * n, C, device=cuda)
    stats = torch.empty(S * 2 * C, device=cuda)
    ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(S, n, C)), device=cuda)
    sy = sync_counter(cuda) if last_block_fold else None
    check(LIB.vg_graphnorm_fwd_seg(ptr(xd), S, n, C, ptr(wd), ptr(bd), ptr(sd), ptr(kd), 1e-5, ptr(y), ptr(stats),
                                   ptr(ws), sy, st), "vg_graphnorm_fwd_seg")
    assert _close(y, torch.cat(ys))[0]
    inj = torch.randn(n, C, dtype=torch.float64)
    gbase = torch.Generator().manual_seed(11)
    base = {k: torch.randn(C, generator=gbase, dtype=torch.float64) for k in P}
    gw, gb, gs = (base[k].float().to(cuda) for k in ("w", "b", "s"))
    gx = torch.empty(S * n, C, device=cuda)
    injd = inj.float().to(cuda)
    check(LIB.vg_graphnorm_bwd_seg(ptr(xd), S, n, C, ptr(wd), ptr(bd), ptr(sd), ptr(kd), 1e-5, ptr(stats), ptr(gyd),
                                   ptr(gx), ptr(gw), ptr(gb), ptr(gs), 1, ptr(injd), 2 * n * C, ptr(ws),
                                   sy, st), "vg_graphnorm_bwd_seg")
    exp = torch.cat(gxs)
    exp[2 * n:] += inj
    assert _close(gx, exp)[0]
    for got, k in ((gw, "w"), (gb, "b"), (gs, "s")):
        # compare the accumulated increment at its own scale (base + increment
        # can cancel to ~0 for C = 1)
        assert _close(got.double().cpu() - base[k].float().double(), pgs[k], 2e-5)[0], k
    if sy is not None:  # the in-kernel folds leave every counter at 0
        from vgan import _lib
        assert all(int(t.abs().sum().item()) == 0 for t in _lib._SYNC.values())


@pytest.mark.parametrize("last_block_fold", [True, False])
@pytest.mark.parametrize("C", [1, 8, 32, 64])
def test_graphnorm_jvp2_matches_autograd(cuda, C, last_block_fold):
    n = 900
    x, P, keep = _gn_inputs(n, C, seed=3)
    u = torch.randn(n, C, dtype=torch.float64)
    gy = torch.randn(n, C, dtype=torch.float64)
    ju, xinj, pg = CR.Unit("gn", CR.gnrd_fn(keep), ["w", "b", "s"]).jvp2(x, u, gy, P)
    xd, kd, ud, gyd, wd, bd, sd = (t.float().to(cuda).contiguous() for t in (x, keep, u, gy, P["w"], P["b"], P["s"]))
    st = stream_handle(cuda)
    y = torch.empty(n, C, device=cuda)
    stats = torch.empty(2 * C, device=cuda)
    ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(1, n, C)), device=cuda)
    sy = sync_counter(cuda) if last_block_fold else None
    check(LIB.vg_graphnorm_fwd_seg(ptr(xd), 1, n, C, ptr(wd), ptr(bd), ptr(sd), ptr(kd), 1e-5, ptr(y), ptr(stats),
                                   ptr(ws), sy, st), "vg_graphnorm_fwd_seg")
    u_out, x_inj = torch.empty(n, C, device=cuda), torch.empty(n, C, device=cuda)
    gb0 = torch.Generator().manual_seed(23)
    gw0, gs0 = (torch.randn(C, generator=gb0, dtype=torch.float64).float().double() for _ in range(2))
    gw, gs = gw0.float().to(cuda), gs0.float().to(cuda)
    check(LIB.vg_graphnorm_jvp2(ptr(xd), n, C, ptr(wd), ptr(bd), ptr(sd), ptr(kd), 1e-5, ptr(stats), ptr(ud), ptr(gyd),
                                ptr(u_out), ptr(x_inj), ptr(gw), ptr(gs), ptr(ws), sy, st), "vg_graphnorm_jvp2")
    if sy is not None:
        from vgan import _lib
        assert all(int(t.abs().sum().item()) == 0 for t in _lib._SYNC.values())  # counters left at 0
    for got, ref in ((u_out, ju), (x_inj, xinj), (gw.double().cpu() - gw0, pg["w"]), (gs.double().cpu() - gs0, pg["s"])):
        ok, err = _close(got, ref, 2e-5)
        assert ok, err


@pytest.mark.parametrize("C", [1, 8, 32, 64])
def test_graphnorm_jvp2_split_with_source_pass_bitwise(cuda, C):
    """vg_graphnorm_jvp2 as _sums / _fold_src / _apply (the native critic
    engine's pass C) with a GAT tangent source pass run inside the fold's
    launch: u_out, x_inj, the parameter gradients, the source pass's h_inj and
    att_src partials all bit-identical to vg_graphnorm_jvp2 + the source pass
    as its own launch (vg_gat_jvp2_deferred)."""
    import ctypes

    from vgan._lib import VgFold, VgJvpSrc

    n = 900
    x, P, keep = _gn_inputs(n, C, seed=5)
    g = torch.Generator().manual_seed(6)
    xd, kd, wd, bd, sd = (t.float().to(cuda).contiguous() for t in (x, keep, P["w"], P["b"], P["s"]))
    u, gy = (torch.randn(n, C, generator=g).to(cuda) for _ in range(2))
    st = stream_handle(cuda)
    y = torch.empty(n, C, device=cuda)
    stats = torch.empty(2 * C, device=cuda)
    ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(1, n, C)), device=cuda)
    check(LIB.vg_graphnorm_fwd_seg(ptr(xd), 1, n, C, ptr(wd), ptr(bd), ptr(sd), ptr(kd), 1e-5, ptr(y), ptr(stats),
                                   ptr(ws), None, st), "vg_graphnorm_fwd_seg")
    # a GAT tangent over a lattice of n nodes for the source pass
    _, vox = _graph((1, 2))
    csr = ops.CSR(vox.edge_index.to(cuda), vox.num_nodes)
    m, e = csr.num_nodes, csr.num_edges
    h, uh, go = (torch.randn(m, C, generator=g).to(cuda) for _ in range(3))
    att_s, att_d = (0.3 * torch.randn(C, generator=g)).to(cuda), (0.3 * torch.randn(C, generator=g)).to(cuda)
    a_s, a_d = h @ att_s, h @ att_d
    out, alpha = torch.empty(m, C, device=cuda), torch.empty(e, device=cuda)
    ops.aggregate_fwd_raw(csr, C, ptr(h), ptr(a_s), ptr(a_d), ptr(torch.zeros(C, device=cuda)), 0.2, ptr(out),
                          ptr(alpha), st)
    res = {}
    for split in (False, True):
        gw, gs = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
        u_out, x_inj = torch.empty(n, C, device=cuda), torch.empty(n, C, device=cuda)
        wsj = torch.zeros(int(LIB.vg_gat_jvp2_ws_floats(m, e, C)), device=cuda)
        uo2, hinj = torch.empty(m, C, device=cuda), torch.zeros(m, C, device=cuda)
        ga_s, ga_d = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
        folds = (VgFold * 2)()
        nf = ctypes.c_int32(0)
        args = (ptr(csr.row_ptr), ptr(csr.col), ptr(csr.csc_ptr), ptr(csr.csc_slot), ptr(csr.csc_dst), m, e, C,
                ptr(h), ptr(uh), ptr(go), ptr(att_s), ptr(att_d), ptr(a_s), ptr(a_d), ptr(alpha), 0.2, ptr(uo2),
                ptr(hinj), ptr(ga_s), ptr(ga_d), None, None, ptr(wsj), folds, ctypes.byref(nf))
        gws = torch.zeros_like(ws)
        if split:
            src = VgJvpSrc()
            check(LIB.vg_gat_jvp2_plan(*args, ctypes.byref(src), st), "vg_gat_jvp2_plan")
            check(LIB.vg_graphnorm_jvp2_sums(ptr(xd), n, C, ptr(wd), ptr(bd), ptr(sd), ptr(kd), 1e-5, ptr(stats), ptr(u),
                                             ptr(gy), ptr(gws), st), "vg_graphnorm_jvp2_sums")
            check(LIB.vg_graphnorm_jvp2_fold_src(n, C, ptr(wd), ptr(sd), ptr(stats), ptr(gws), ptr(gw), ptr(gs),
                                                 ctypes.byref(src), st), "vg_graphnorm_jvp2_fold_src")
            check(LIB.vg_graphnorm_jvp2_apply(ptr(xd), n, C, ptr(wd), ptr(bd), ptr(sd), ptr(kd), 1e-5, ptr(stats),
                                              ptr(u), ptr(gy), ptr(u_out), ptr(x_inj), ptr(gws), st),
                  "vg_graphnorm_jvp2_apply")
        else:
            check(LIB.vg_gat_jvp2_deferred(*args, st), "vg_gat_jvp2_deferred")
            check(LIB.vg_graphnorm_jvp2(ptr(xd), n, C, ptr(wd), ptr(bd), ptr(sd), ptr(kd), 1e-5, ptr(stats), ptr(u),
                                        ptr(gy), ptr(u_out), ptr(x_inj), ptr(gw), ptr(gs), ptr(gws), None, st),
                  "vg_graphnorm_jvp2")
        torch.cuda.synchronize()
        part_s = wsj[5 * e + 3 * m:].view(-1)  # both partial blocks (vg_gat_jvp2_ws_floats layout)
        res[split] = [t.clone() for t in (u_out, x_inj, gw, gs, uo2, hinj, part_s)]
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)


# -------------------------------------------------------------- helpers
@pytest.mark.parametrize("n", [333, 5000])
def test_critic_input_and_gp_head(cuda, n):
    g = torch.Generator().manual_seed(5)
    F, K = 29, 7
    mvx = torch.rand(n, F, generator=g)
    real = torch.nn.functional.one_hot(torch.randint(0, K, (n,), generator=g), K).float()
    hard = torch.nn.functional.one_hot(torch.randint(0, K, (n,), generator=g), K).float()
    soft = torch.softmax(torch.randn(n, K, generator=g), 1)
    eps = torch.rand(n, 1, generator=g)
    X = torch.empty(3 * n, F + K, device=cuda)
    st = stream_handle(cuda)
    dv = [t.to(cuda).contiguous() for t in (mvx, real, hard, soft, eps)]
    check(LIB.vg_critic_input(ptr(dv[0]), n, F, ptr(dv[1]), ptr(dv[2]), ptr(dv[3]), ptr(dv[4]), K, 3, ptr(X), st),
          "vg_critic_input")
    mix = eps * real + (1 - eps) * soft  # the reference's rounding (trainer.py:298-301)
    exp = torch.cat([torch.cat([mvx, real], 1), torch.cat([mvx, hard], 1), torch.cat([mvx, mix], 1)])
    assert torch.equal(X.cpu(), exp)
    gg = torch.randn(n, K, generator=g, dtype=torch.float64)
    gg[3] = 0.0
    sc = torch.randn(3 * n, dtype=torch.float64)
    u0, out = torch.empty(n, K, device=cuda), torch.empty(2, device=cuda)
    ggd, scd = gg.float().to(cuda), sc.float().to(cuda)
    gws = torch.empty(int(LIB.vg_gp_head_ws_floats(n)), device=cuda)
    cnt = torch.zeros(1, dtype=torch.int32, device=cuda)
    check(LIB.vg_gp_head(ptr(ggd), n, K, ptr(scd), 10.0, ptr(u0), K, ptr(out), ptr(gws), ptr(cnt), st),
          "vg_gp_head")
    leaf = gg.clone().requires_grad_(True)
    gp = ((leaf.norm(dim=1) - 1) ** 2).mean() * 10.0
    (gref,) = torch.autograd.grad(gp, leaf)
    loss = sc[n:2 * n].mean() - sc[:n].mean() + gp
    assert abs(out[1].item() - gp.item()) <= 1e-5 * abs(gp.item())
    assert abs(out[0].item() - loss.item()) <= 1e-5 * max(1.0, abs(loss.item()))
    gref[3] = 0.0  # torch's norm backward at 0 is 0 as well (subgradient)
    assert _close(u0, gref)[0]
    assert int(cnt.item()) == 0  # counter left at 0


# --------------------------------------------------------------- engine
class _RecRNG:
    """Seeded CPU draws in the engine's (= the reference's) order, recorded."""
    mode = "fixed"

    def __init__(self, seed):
        self.g = torch.Generator().manual_seed(seed)
        self.draws = []

    def keep_mask(self, shape, p, device):
        t = torch.empty(*shape).bernoulli_(1 - p, generator=self.g).div_(1 - p)
        self.draws.append(t)
        return t.to(device)

    def uniform(self, shape, device):
        t = torch.rand(*shape, generator=self.g)
        self.draws.append(t)
        return t.to(device)


def _engine_setup(cuda, numbers=(1, 2, 3, 4), seed=11):
    from vgan import data as vdata
    from vgan.critic import CriticEngine
    from vgan.models import VoxelGNNDiscriminator

    cfg = Configuration()
    cfg.DEVICE = cuda
    torch.manual_seed(seed)
    D = VoxelGNNDiscriminator(cfg, 17, 12)
    from vgan.flat import FlatParams
    flat = FlatParams(D)
    loc, vox = _graph(numbers)
    loc, vox = loc.to(cuda), vox.to(cuda)
    prep = vdata.prepared(loc, vox, cfg.NUM_CLASSES)
    n = vox.num_nodes
    g = torch.Generator().manual_seed(seed + 1)
    logits = torch.randn(n, 7, generator=g) * 2
    soft = torch.softmax(logits, 1)
    hard = torch.nn.functional.one_hot(soft.argmax(1), 7).float()
    return cfg, D, flat, loc, vox, prep, hard, soft, CriticEngine(D, cfg)


def test_engine_matches_f64_references(cuda):
    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda)
    n = vox.num_nodes
    rng = _RecRNG(3)
    flat.zero_grad()
    loss = eng.loss_and_grad(loc, vox, hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0), rng)
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().double() for k, p in D.named_parameters()}
    nb = len(eng.blocks)
    real_k, fake_k, eps, mix_k = rng.draws[:nb], rng.draws[nb:2 * nb], rng.draws[2 * nb], rng.draws[2 * nb + 1:]
    d = torch.float64
    ei = vox.edge_index.cpu()
    P = {k: v.detach().cpu().double() for k, v in D.state_dict().items()}
    units = {c: CR.d_units(nb, len(eng.dec), ei, n, [k.double() for k in ks])
             for c, ks in (("real", real_k), ("fake", fake_k), ("mix", mix_k))}
    mvx = prep.matched_voxel_x.cpu().double()
    real = prep.onehot_f.cpu().double()
    e = eps.double()
    mix = e * real + (1 - e) * soft.double()
    x0s = {"real": torch.cat([mvx, real], 1), "fake": torch.cat([mvx, hard.double()], 1),
           "mix": torch.cat([mvx, mix], 1)}
    lab = slice(mvx.shape[1], mvx.shape[1] + 7)
    l1, gp1, g1 = CR.run(units, x0s, lab, float(cfg.LAMBDA_GP), P)
    l2, gp2, g2 = CR.autograd_loss(units, x0s, lab, float(cfg.LAMBDA_GP), P)
    assert abs(l1.item() - l2.item()) <= 1e-10 * max(1.0, abs(l2.item()))
    assert abs(loss.item() - l2.item()) <= 1e-5 * max(1.0, abs(l2.item())), (loss.item(), l2.item())
    assert abs(eng.last_gp.item() - gp2.item()) <= 1e-5 * max(1.0, abs(gp2.item()))
    ok, worst, total = grads_close(grads, g2, rtol=1e-3)
    assert ok, (worst, total)


def test_engine_matches_autograd_path_on_gpu(cuda):
    """Same host RNG stream: the engine consumes it exactly like
    Trainer._compute_discriminator_loss (reference order)."""
    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6), seed=4)
    from vgan.rng import RNG
    from vgan.trainer import Trainer
    from vgan.models import VoxelGNNGenerator

    cfg.runtime["rng"] = "host"
    G = VoxelGNNGenerator(cfg, 17, 12)
    tr = Trainer(G, D, None, torch.optim.Adam(G.parameters()), torch.optim.Adam(D.parameters()), None, cfg)
    rng = RNG("host")
    hd, sd = hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0)
    torch.manual_seed(123)
    tr.flat_d.zero_grad()
    l_eng = eng.loss_and_grad(loc, vox, hd, sd, rng)
    g_eng = {k: p.grad.detach().clone() for k, p in D.named_parameters()}
    after = torch.get_rng_state()
    torch.manual_seed(123)
    tr.flat_d.zero_grad()
    l_ag = tr._compute_discriminator_loss(loc, vox, hd, sd)
    l_ag.backward()
    assert torch.equal(torch.get_rng_state(), after)
    g_ag = {k: p.grad.detach().clone() for k, p in D.named_parameters()}
    assert abs(l_eng.item() - l_ag.item()) <= 1e-5 * max(1.0, abs(l_ag.item()))
    ok, worst, total = grads_close(g_eng, g_ag, rtol=1e-3)
    assert ok, (worst, total)


@pytest.mark.parametrize("precision", ["f32", "bf16"])
def test_grouped_weight_gradients_bit_identical(cuda, precision, monkeypatch):
    """The weight-gradient products of a backward run as ONE vg_gemm_tn_group
    launch at its end (FoldCollector.tn) instead of one launch per layer.  The
    grouped plan splits each product over fewer row chunks (64 instead of
    768 workgroups per output tile), so the f32 sums differ only in order: the critic loss is
    identical and the D and G gradients agree to 1e-6 relative."""
    from vgan import _lib, ops
    from vgan._lib import gemm_precision_scope
    from vgan.models import VoxelGNNGenerator

    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6), seed=4)
    torch.manual_seed(9)
    G = VoxelGNNGenerator(cfg, 17, 12).to(cuda).eval()
    from vgan.flat import FlatParams
    flat_g = FlatParams(G)
    z = torch.randn(1, vox.num_nodes, cfg.Z_DIM, device=cuda)
    noise = torch.empty(vox.num_nodes, 7, device=cuda).exponential_()
    w = torch.randn(vox.num_nodes, 7, device=cuda)
    hd, sd = hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0)
    out = {}
    for grouped in (True, False):
        monkeypatch.setattr(_lib, "_TN_GROUP", grouped)
        with gemm_precision_scope(precision):
            flat.zero_grad()
            loss = eng.loss_and_grad(loc, vox, hd, sd, _RecRNG(3))
            flat_g.zero_grad()
            logits, _, soft_g = G(loc, vox, z, noise=noise)
            with ops.direct_param_grads(), ops.deferred_param_folds(cuda):
                ((logits * w).sum() + (soft_g * w).sum()).backward()
        torch.cuda.synchronize()
        out[grouped] = (loss.item(), flat.grad.clone(), flat_g.grad.clone())
    assert out[True][0] == out[False][0]
    assert rel_err(out[True][1], out[False][1]) < 1e-6
    assert rel_err(out[True][2], out[False][2]) < 1e-6


@pytest.mark.parametrize("training", [True, False])
def test_gemm_fused_graphnorm_backward_partials(cuda, training, monkeypatch):
    """The critic engine's GraphNorm backward with its column partials formed
    in the epilogue of the GEMM that produces g_y (vg_gemm_gn_bwd + the tile
    fold) against the separate partial pass: the same sums in another order,
    so loss and D gradient agree to f32 rounding."""
    from vgan import critic as vcritic

    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6, 7), seed=8)
    D.train(training)
    hd, sd = hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0)
    out = {}
    for fuse in (True, False):
        monkeypatch.setattr(vcritic, "_GN_FUSE", fuse)
        flat.zero_grad()
        loss = eng.loss_and_grad(loc, vox, hd, sd, _RecRNG(21))
        torch.cuda.synchronize()
        out[fuse] = (loss.item(), flat.grad.clone())
    assert vox.num_nodes >= 64
    assert abs(out[True][0] - out[False][0]) <= 1e-6 * max(1.0, abs(out[False][0]))
    assert rel_err(out[True][1], out[False][1]) < 1e-5


def test_grouped_jvp_source_passes_bit_identical(cuda, monkeypatch):
    """The tangent sweep's source passes (dQ/dh injections, att_src partials)
    run as one vg_gat_jvp_src_group launch before pass D instead of one
    launch per block: the same block bodies and partial rows, so the loss and
    the D gradient are bit-identical."""
    from vgan import _lib

    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6), seed=12)
    hd, sd = hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0)
    out = {}
    for grouped in (True, False):
        monkeypatch.setattr(_lib, "_JVP_GROUP", grouped)
        flat.zero_grad()
        loss = eng.loss_and_grad(loc, vox, hd, sd, _RecRNG(5))
        torch.cuda.synchronize()
        out[grouped] = (loss.item(), flat.grad.clone())
    assert out[True][0] == out[False][0]
    assert torch.equal(out[True][1], out[False][1])


@pytest.mark.parametrize("training,fuse", [(True, True), (False, True), (True, False)])
def test_gat_backward_forms_graphnorm_backward(cuda, training, fuse, monkeypatch):
    """The GraphNorm backward's elementwise pass formed in the GAT backward's
    destination-row pass (vg_gat_bwd_gn, gnbwd.h) against its own launch: one
    formula over the same column sums, so the loss and the D gradient are the
    same up to f32 contraction (dropout masks, the pass-D injection, both
    sum folds: GEMM tiles and the separate partial pass)."""
    from vgan import critic as vcritic

    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6, 7), seed=31)
    D.train(training)
    monkeypatch.setattr(vcritic, "_GN_FUSE", fuse)
    hd, sd = hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0)
    out = {}
    for rows in (True, False):
        monkeypatch.setattr(vcritic, "_GN_ROWS", rows)
        flat.zero_grad()
        loss = eng.loss_and_grad(loc, vox, hd, sd, _RecRNG(22))
        torch.cuda.synchronize()
        out[rows] = (loss.item(), flat.grad.clone())
    assert out[True][0] == out[False][0]
    assert rel_err(out[True][1], out[False][1]) < 1e-6


@pytest.mark.parametrize("precision", ["f32", "bf16"])
def test_autograd_graphnorm_partials_from_next_gemm(cuda, precision, monkeypatch):
    """Autograd path (the generator iteration): a GraphNorm whose output feeds
    a linear layer takes its backward's column partials from that layer's dX
    GEMM epilogue (ops.gemm_gn_bwd + vg_graphnorm_bwd_seg_tiles) instead of a
    partial pass; the encoder's last GraphNorm (its output also goes to the
    decoder concat) keeps the separate pass.  Gradients agree to f32 rounding."""
    from vgan import ops
    from vgan._lib import gemm_precision_scope
    from vgan.flat import FlatParams
    from vgan.models import VoxelGNNGenerator
    from vgan.rng import RNG

    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6, 7), seed=6)
    torch.manual_seed(13)
    G = VoxelGNNGenerator(cfg, 17, 12).to(cuda).train()
    flat_g = FlatParams(G)
    z = torch.randn(1, vox.num_nodes, cfg.Z_DIM, device=cuda)
    noise = torch.empty(vox.num_nodes, 7, device=cuda).exponential_()
    w = torch.randn(vox.num_nodes, 7, device=cuda)
    calls = []
    orig = ops.gemm_gn_bwd
    monkeypatch.setattr(ops, "gemm_gn_bwd", lambda *a: calls.append(1) or orig(*a))
    out = {}
    ops._GN_HINTS.clear()  # hints of earlier tests' forwards whose backward never ran
    for epi in (True, False):
        monkeypatch.setattr(ops, "_GN_EPI", epi)
        G.rng = RNG("fixed", seed=3)
        flat_g.zero_grad()
        with gemm_precision_scope(precision):
            logits, _, soft_g = G(loc, vox, z, noise=noise)
            with ops.direct_param_grads(), ops.deferred_param_folds(cuda):
                ((logits * w).sum() + (soft_g * w).sum()).backward()
        torch.cuda.synchronize()
        out[epi] = flat_g.grad.clone()
        assert not ops._GN_HINTS
    assert vox.num_nodes >= 64 and len(calls) >= 10
    # bf16: the f32 sums differ in order only (~1e-7), but a downstream operand
    # rounded to bf16 turns such a difference into a bf16 ulp (2^-8)
    assert rel_err(out[True], out[False]) < (1e-5 if precision == "f32" else 2e-2)
