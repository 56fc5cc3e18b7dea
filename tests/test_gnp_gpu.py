"""GraphNorm column statistics from the GAT aggregation's epilogue
(vg_gat_aggregate_fwd_gnp + vg_graphnorm_fwd_gnp, ops.gnp_buffer) against
the separate statistics pass (vg_graphnorm_fwd_seg / _drop) and a torch fp32
GraphNorm (torch_geometric GraphNorm, batch=None: models.py:73-75,193-195).

The aggregation's out / alpha must stay bit-identical to vg_gat_aggregate_fwd;
the statistics are the same Welford sums grouped by workgroup instead of by
row chunk, so they agree with the chunked fold to f32 rounding (tolerances
below), and dropout masks drawn in-kernel are bit-identical."""
from __future__ import annotations

import pytest
import torch

from parity_util import rel_err
from test_critic_gpu import _RecRNG, _engine_setup
from test_ops_gpu import _aggregate_ref_kernel, _graph, _star_graph
from vgan import ops
from vgan._lib import LIB, check, ptr

pytestmark = pytest.mark.gpu

EPS = 1e-5


def _csr(cuda, graph: str, copies: int):
    if graph == "star":
        ei, n = _star_graph(600)
    else:
        _, vox = _graph(stress=(graph == "stress"))
        ei, n = vox.edge_index, vox.num_nodes
    csr = ops.CSR(ei.to(cuda), n)
    csr.ell()
    if graph == "big":  # >= 100k rows: the 64-channel slice path of the aggregation
        copies = -(-100_000 // n)
    return csr.stacked(copies) if copies > 1 else csr


def _gn_torch(x, S, w, b, ms, keep=None):
    """fp32 GraphNorm + ReLU (+ dropout multipliers) per segment."""
    ys, stats = [], []
    for xs in x.chunk(S):
        mu = xs.mean(0)
        c = xs - mu * ms
        d = (c.pow(2).mean(0) + EPS).sqrt()  # PyG 2.6.1 GraphNorm(batch=None): stats = [mu | d]
        ys.append(torch.relu(w * c / d + b))
        stats.append(torch.cat([mu, d]))
    y = torch.cat(ys)
    return (y * keep if keep is not None else y), torch.cat(stats)


@pytest.mark.parametrize("graph,copies,C", [(g, k, c) for g, k in (("lattice", 1), ("lattice", 3), ("stress", 1),
                                                                     ("stress", 5), ("star", 1), ("star", 3))
                                             for c in (1, 3, 8, 12, 32, 64, 128)]
                         + [("big", 0, 128)])  # the 64-channel slice path needs C > 64
def test_aggregate_gnp_matches_statistics_pass(cuda, graph, copies, C):
    torch.manual_seed(C + 7 * copies)
    csr = _csr(cuda, graph, copies)
    n, seg = csr.num_nodes, csr.seg_rows
    S = n // seg
    gnp, g = ops.gnp_buffer(csr, C, cuda)
    assert gnp is not None and g in (8, 16, 32) and seg >= g
    h = torch.randn(n, C, device=cuda)
    a_s, a_d = 0.5 * torch.randn(n, device=cuda), 0.5 * torch.randn(n, device=cuda)
    b = torch.randn(C, device=cuda)
    out, alpha = torch.empty_like(h), torch.empty(csr.num_edges, device=cuda)
    gnp.fill_(float("nan"))  # every partial the fold reads must be written
    ops.aggregate_fwd_raw(csr, C, ptr(h), ptr(a_s), ptr(a_d), ptr(b), 0.2, ptr(out), ptr(alpha), csr.stream(), gnp)
    ref_out, ref_alpha = _aggregate_ref_kernel(csr, h, a_s, a_d, b)
    assert torch.equal(out, ref_out) and torch.equal(alpha, ref_alpha)

    w = 1 + 0.2 * torch.randn(C, device=cuda)
    bb = 0.2 * torch.randn(C, device=cuda)
    ms = 1 + 0.2 * torch.randn(C, device=cuda)
    st = ops.stream_handle(cuda)
    y1, st1 = torch.empty_like(out), torch.empty(S * 2 * C, device=cuda)
    check(LIB.vg_graphnorm_fwd_gnp(ptr(out), S, seg, C, ptr(w), ptr(bb), ptr(ms), None, 0.0, 0, None, 0, EPS,
                                   ptr(y1), None, ptr(st1), ptr(gnp), g, st), "vg_graphnorm_fwd_gnp")
    y2, st2 = torch.empty_like(out), torch.empty(S * 2 * C, device=cuda)
    ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(S, seg, C)), device=cuda)
    check(LIB.vg_graphnorm_fwd_seg(ptr(out), S, seg, C, ptr(w), ptr(bb), ptr(ms), None, EPS, ptr(y2), ptr(st2),
                                   ptr(ws), None, st), "vg_graphnorm_fwd_seg")
    y_ref, st_ref = _gn_torch(out.double(), S, w.double(), bb.double(), ms.double())
    torch.cuda.synchronize()
    assert torch.isfinite(st1).all()
    # column statistics: f32 Welford in another grouping, 1e-5 of the f64 values
    assert (st1.double() - st_ref).abs().max().item() <= 1e-5 * max(1.0, st_ref.abs().max().item())
    assert (st1 - st2).abs().max().item() <= 1e-5 * max(1.0, st2.abs().max().item())
    assert rel_err(y1.double(), y_ref) < 1e-5
    assert rel_err(y1, y2) < 1e-5


@pytest.mark.parametrize("C", [4, 64])
def test_gnp_dropout_mask_bit_identical(cuda, C):
    """In-kernel dropout through the partials path draws the same multipliers
    (counter-based Philox on the element index) as vg_graphnorm_fwd_drop."""
    torch.manual_seed(C)
    csr = _csr(cuda, "lattice", 3)
    n, seg = csr.num_nodes, csr.seg_rows
    gnp, g = ops.gnp_buffer(csr, C, cuda)
    h = torch.randn(n, C, device=cuda)
    a_s, a_d = 0.5 * torch.randn(n, device=cuda), 0.5 * torch.randn(n, device=cuda)
    b = torch.randn(C, device=cuda)
    out, alpha = torch.empty_like(h), torch.empty(csr.num_edges, device=cuda)
    ops.aggregate_fwd_raw(csr, C, ptr(h), ptr(a_s), ptr(a_d), ptr(b), 0.2, ptr(out), ptr(alpha), csr.stream(), gnp)
    w, bb, ms = torch.ones(C, device=cuda), torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    it = torch.tensor([5], dtype=torch.int64, device=cuda)
    st = ops.stream_handle(cuda)
    y1, k1, s1 = torch.empty_like(out), torch.empty_like(out), torch.empty(6 * C, device=cuda)
    check(LIB.vg_graphnorm_fwd_gnp(ptr(out), 3, seg, C, ptr(w), ptr(bb), ptr(ms), None, 0.2, 1234, ptr(it), 77, EPS,
                                   ptr(y1), ptr(k1), ptr(s1), ptr(gnp), g, st), "vg_graphnorm_fwd_gnp")
    y2, k2, s2 = torch.empty_like(out), torch.empty_like(out), torch.empty(6 * C, device=cuda)
    ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(3, seg, C)), device=cuda)
    check(LIB.vg_graphnorm_fwd_drop(ptr(out), 3, seg, C, ptr(w), ptr(bb), ptr(ms), 0.2, 1234, ptr(it), 77, EPS,
                                    ptr(y2), ptr(k2), ptr(s2), ptr(ws), None, st), "vg_graphnorm_fwd_drop")
    torch.cuda.synchronize()
    assert torch.equal(k1, k2)
    assert 0.1 < (k1 == 0).float().mean().item() < 0.3
    assert rel_err(y1, y2) < 1e-5


def test_gnp_abi_rejects_bad_segments(cuda):
    """Segments shorter than a workgroup's rows, or not dividing N: VG_EINVAL."""
    csr = _csr(cuda, "lattice", 1)
    n, C = csr.num_nodes, 64
    g = int(LIB.vg_gat_gnp_rows(n, C))
    assert g == 16 and int(LIB.vg_gat_gnp_rows(n, 8)) == 32
    assert int(LIB.vg_gat_gnp_floats(n, C)) == 2 * -(-n // g) * 2 * C * 3  # room for segment-aligned blocks
    h = torch.zeros(n, C, device=cuda)
    v = torch.zeros(n, device=cuda)
    out, alpha = torch.empty_like(h), torch.empty(csr.num_edges, device=cuda)
    gnp = torch.empty(int(LIB.vg_gat_gnp_floats(n, C)), device=cuda)
    for seg in (g - 1, n - 1):
        rc = LIB.vg_gat_aggregate_fwd_gnp(ptr(csr.row_ptr), ptr(csr.col), None, 0, n, C, ptr(h), ptr(v), ptr(v),
                                          ptr(v[:C]), 0.2, ptr(out), ptr(alpha), seg, ptr(gnp), csr.stream())
        assert rc != 0


@pytest.mark.parametrize("training", [True, False])
def test_critic_engine_and_generator_with_gnp(cuda, training, monkeypatch):
    """The critic engine and the generator's autograd path with the GraphNorm
    statistics from the aggregation against the separate statistics pass:
    the same loss and gradients to f32 rounding, and the fused path runs for
    every GraphNorm of both networks."""
    from vgan import _lib
    from vgan.flat import FlatParams
    from vgan.models import VoxelGNNGenerator
    from vgan.rng import RNG

    monkeypatch.setattr(_lib, "_GN_APPLY_GEMM", False)  # every GraphNorm applies itself (counted below)
    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6, 7), seed=17)
    D.train(training)
    torch.manual_seed(19)
    G = VoxelGNNGenerator(cfg, 17, 12).to(cuda).train(training)
    flat_g = FlatParams(G)
    z = torch.randn(1, vox.num_nodes, cfg.Z_DIM, device=cuda)
    noise = torch.empty(vox.num_nodes, 7, device=cuda).exponential_()
    wgt = torch.randn(vox.num_nodes, 7, device=cuda)
    hd, sd = hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0)
    calls = []
    orig = LIB.vg_graphnorm_fwd_gnp

    def counted(*a):
        calls.append(1)
        return orig(*a)

    out = {}
    for fuse in (True, False):
        monkeypatch.setattr(ops, "_GN_FWD_FUSE", fuse)
        monkeypatch.setattr(LIB, "vg_graphnorm_fwd_gnp", counted)
        calls.clear()
        flat.zero_grad()
        loss = eng.loss_and_grad(loc, vox, hd, sd, _RecRNG(4))
        G.rng = RNG("fixed", seed=3)
        flat_g.zero_grad()
        logits, _, soft_g = G(loc, vox, z, noise=noise)
        with ops.direct_param_grads(), ops.deferred_param_folds(cuda):
            ((logits * wgt).sum() + (soft_g * wgt).sum()).backward()
        torch.cuda.synchronize()
        out[fuse] = (loss.item(), flat.grad.clone(), logits.detach().clone(), flat_g.grad.clone(), len(calls))
    n_gn = len(eng.blocks) + G.encoder.num_blocks
    assert out[True][4] == n_gn and out[False][4] == 0
    assert abs(out[True][0] - out[False][0]) <= 1e-5 * max(1.0, abs(out[False][0]))
    assert rel_err(out[True][1], out[False][1]) < 1e-4
    assert rel_err(out[True][2], out[False][2]) < 1e-5
    # the G gradient: the two statistics orders differ by f32 rounding, which
    # the generator gradient amplifies (tools/gnp_g_probe.py: each path is
    # 1.7e-5 / 3.2e-5 from the f64 oracle where the oracle's own f32 is 6.9e-6
    # off; these draws measured 3.5e-4 between the paths)
    assert rel_err(out[True][3], out[False][3]) < 1e-3


def _lin_att_gn_case(cuda, S, n, cin, cout, mode, seed=0):
    """vg_gat_lin_att_gn against vg_graphnorm_fwd_gnp + vg_gat_lin_att on the
    same GraphNorm input / statistics (keep: none, multipliers, drawn)."""
    import ctypes

    from vgan._lib import VgGnApply

    g = torch.Generator(device=cuda).manual_seed(seed)
    R = S * n
    x = torch.randn(R, cin, device=cuda, generator=g) * 1.5 + 0.3
    w = 1 + 0.2 * torch.randn(cin, device=cuda, generator=g)
    b = 0.2 * torch.randn(cin, device=cuda, generator=g)
    ms = 1 + 0.2 * torch.randn(cin, device=cuda, generator=g)
    W = torch.randn(cout, cin, device=cuda, generator=g) / cin ** 0.5
    att_s, att_d = torch.randn(cout, device=cuda, generator=g), torch.randn(cout, device=cuda, generator=g)
    stats = torch.empty(S * 2 * cin, device=cuda)
    ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(S, n, cin)), device=cuda)
    st = ops.stream_handle(cuda)
    keep_in = (torch.rand(R, cin, device=cuda, generator=g) > 0.2).float() / 0.8 if mode == "keep" else None
    it = torch.tensor([3], dtype=torch.int64, device=cuda)
    # reference: GraphNorm (statistics + apply), then the projection
    y_ref, k_ref = torch.empty_like(x), torch.empty_like(x)
    if mode == "drop":
        check(LIB.vg_graphnorm_fwd_drop(ptr(x), S, n, cin, ptr(w), ptr(b), ptr(ms), 0.2, 99, ptr(it), 5, EPS,
                                        ptr(y_ref), ptr(k_ref), ptr(stats), ptr(ws), None, st), "fwd_drop")
    else:
        check(LIB.vg_graphnorm_fwd_seg(ptr(x), S, n, cin, ptr(w), ptr(b), ptr(ms), ptr(keep_in), EPS, ptr(y_ref),
                                       ptr(stats), ptr(ws), None, st), "fwd_seg")
    H0, s0, d0 = torch.empty(R, cout, device=cuda), torch.empty(R, device=cuda), torch.empty(R, device=cuda)
    check(LIB.vg_gat_lin_att(ptr(y_ref), cin, ptr(W), R, cin, cout, ptr(att_s), ptr(att_d), ptr(H0), ptr(s0),
                             ptr(d0), st), "lin_att")
    # fused: the same statistics, the GraphNorm applied in the operand load
    y, kp = torch.full_like(x, float("nan")), torch.full_like(x, float("nan"))
    H1, s1, d1 = torch.empty(R, cout, device=cuda), torch.empty(R, device=cuda), torch.empty(R, device=cuda)
    desc = VgGnApply(stats=stats.data_ptr(), weight=w.data_ptr(), bias=b.data_ptr(), mean_scale=ms.data_ptr(),
                     keep=keep_in.data_ptr() if keep_in is not None else None, eps=EPS,
                     p_drop=0.2 if mode == "drop" else 0.0, seg_rows=n, salt=5 if mode == "drop" else 0,
                     seed=99 if mode == "drop" else 0, iter=it.data_ptr() if mode == "drop" else None,
                     y=y.data_ptr(), keep_out=kp.data_ptr() if mode == "drop" else None)
    check(LIB.vg_gat_lin_att_gn(ptr(x), ptr(W), R, cin, cout, ptr(att_s), ptr(att_d), ptr(H1), ptr(s1), ptr(d1),
                                ctypes.byref(desc), st), "lin_att_gn")
    torch.cuda.synchronize()
    return (y_ref, k_ref, H0, s0, d0), (y, kp, H1, s1, d1)


@pytest.mark.parametrize("mode", ["none", "keep", "drop"])
@pytest.mark.parametrize("S,n", [(1, 700), (3, 1001), (5, 130)])
@pytest.mark.parametrize("cin,cout", [(64, 32), (32, 16), (8, 16), (16, 64), (128, 64)])
def test_lin_att_gn_matches_separate_apply(cuda, mode, S, n, cin, cout):
    """The GraphNorm output y, the drawn dropout multipliers and the projection
    (H, a_src, a_dst) equal the separate GraphNorm apply + projection; the
    tiles that straddle a segment boundary use the next segment's statistics."""
    ref, got = _lin_att_gn_case(cuda, S, n, cin, cout, mode, seed=cin + cout + S)
    y_ref, k_ref, H0, s0, d0 = ref
    y, kp, H1, s1, d1 = got
    if mode == "drop":
        assert torch.equal(kp, k_ref)
    # same formula and operation order as k_gn_apply4: equal up to FMA contraction
    assert (y - y_ref).abs().max().item() <= 1e-6 * max(1.0, y_ref.abs().max().item())
    assert rel_err(H1, H0) < 1e-6 and rel_err(s1, s0) < 1e-6 and rel_err(d1, d0) < 1e-6


def test_lin_att_gn_rejects_unsupported(cuda):
    """C > 64 (several column tiles), Cin > 128 or segments shorter than a
    64-row tile: VG_EINVAL (the caller applies the GraphNorm itself)."""
    import ctypes

    from vgan._lib import VgGnApply

    z = torch.zeros(256 * 256, device=cuda)
    desc = VgGnApply(stats=z.data_ptr(), weight=z.data_ptr(), bias=z.data_ptr(), mean_scale=z.data_ptr(), eps=EPS,
                     seg_rows=128, y=None)
    st = ops.stream_handle(cuda)
    for N, cin, c, seg in ((256, 32, 128, 128), (256, 256, 32, 128), (256, 32, 32, 32)):
        desc.seg_rows = seg
        rc = LIB.vg_gat_lin_att_gn(ptr(z), ptr(z), N, cin, c, ptr(z), ptr(z), ptr(z), ptr(z), ptr(z),
                                   ctypes.byref(desc), st)
        assert rc != 0


@pytest.mark.parametrize("training", [True, False])
def test_critic_engine_gn_apply_in_gemm(cuda, training, monkeypatch):
    """The critic engine with each block's GraphNorm applied in the next
    block's projection GEMM (vg_gat_lin_att_gn) against the separate apply:
    the same loss and D gradient to f32 rounding, and the fused GEMM runs for
    every block whose successor projects to <= 64 channels."""
    from vgan import _lib

    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6, 7), seed=23)
    D.train(training)
    hd, sd = hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0)
    calls = []
    orig = LIB.vg_gat_lin_att_gn

    def counted(*a):
        calls.append(1)
        return orig(*a)

    monkeypatch.setattr(LIB, "vg_gat_lin_att_gn", counted)
    out = {}
    for fuse in (True, False):
        monkeypatch.setattr(_lib, "_GN_APPLY_GEMM", fuse)
        calls.clear()
        flat.zero_grad()
        loss = eng.loss_and_grad(loc, vox, hd, sd, _RecRNG(8))
        torch.cuda.synchronize()
        out[fuse] = (loss.item(), flat.grad.clone(), len(calls))
    widths = [conv.out_channels for conv, _ in eng.blocks]
    assert out[True][2] == sum(1 for c in widths[1:] if c <= 64) and out[False][2] == 0
    assert abs(out[True][0] - out[False][0]) <= 1e-6 * max(1.0, abs(out[False][0]))
    assert rel_err(out[True][1], out[False][1]) < 1e-5


@pytest.mark.parametrize("training", [True, False])
def test_critic_tangent_graphnorm_sums_from_gat_pass(cuda, training, monkeypatch):
    """Pass C with each GraphNorm's tangent sums (sum u, sum xt u, sum p,
    sum p u, sum p xt) formed in the GAT tangent pass that produces u
    (vg_gat_jvp2_gn_deferred + vg_graphnorm_jvp2_part) against the separate
    sums pass (vg_graphnorm_jvp2): pass C feeds only the gradient, so the loss
    is identical and the D gradient agrees to f32 rounding (sums in another
    order); the fused path runs for every block."""
    from vgan import _lib

    cfg, D, flat, loc, vox, prep, hard, soft, eng = _engine_setup(cuda, numbers=(5, 6, 7), seed=41)
    D.train(training)
    hd, sd = hard.to(cuda).unsqueeze(0), soft.to(cuda).unsqueeze(0)
    calls = []
    orig = LIB.vg_gat_jvp2_gn_deferred

    def counted(*a):
        calls.append(1)
        return orig(*a)

    monkeypatch.setattr(LIB, "vg_gat_jvp2_gn_deferred", counted)
    out = {}
    for fuse in (True, False):
        monkeypatch.setattr(_lib, "_GN_JVP_FUSE", fuse)
        calls.clear()
        flat.zero_grad()
        loss = eng.loss_and_grad(loc, vox, hd, sd, _RecRNG(12))
        torch.cuda.synchronize()
        out[fuse] = (loss.item(), flat.grad.clone(), len(calls))
    assert out[True][2] == len(eng.blocks) and out[False][2] == 0
    assert out[True][0] == out[False][0]
    assert rel_err(out[True][1], out[False][1]) < 1e-5


@pytest.mark.parametrize("C", [1, 8, 32, 64, 128])
def test_stacked_statistics_bitwise_equal_separate(cuda, C):
    """Segment-aligned partial blocks: the column statistics of a stacked
    3-copy aggregation (the critic engine's real / fake / mix forward) are bit
    for bit those of three separate aggregations over the copies -- the
    grouping autograd's three separate discriminator passes use."""
    csr = _csr(cuda, "lattice", 1)
    n = csr.num_nodes
    st3 = csr.stacked(3)
    torch.manual_seed(C)
    hs = [torch.randn(n, C, device=cuda) for _ in range(3)]
    ass = [0.5 * torch.randn(n, device=cuda) for _ in range(3)]
    ads = [0.5 * torch.randn(n, device=cuda) for _ in range(3)]
    b = torch.randn(C, device=cuda)
    ms = torch.rand(C, device=cuda) + 0.2
    st = ops.stream_handle(cuda)

    def run(graph, h, a_s, a_d, segs):
        gnp, g = ops.gnp_buffer(graph, C, cuda)
        out, alpha = torch.empty_like(h), torch.empty(graph.num_edges, device=cuda)
        ops.aggregate_fwd_raw(graph, C, ptr(h), ptr(a_s), ptr(a_d), ptr(b), 0.2, ptr(out), ptr(alpha), st, gnp)
        stats = torch.empty(segs * 2 * C, device=cuda)
        check(LIB.vg_graphnorm_stats_gnp(segs, n, C, ptr(gnp), g, ptr(ms), 1e-5, ptr(stats), st),
              "vg_graphnorm_stats_gnp")
        return out, stats

    out3, s3 = run(st3, torch.cat(hs).contiguous(), torch.cat(ass), torch.cat(ads), 3)
    for k in range(3):
        o1, s1 = run(csr, hs[k], ass[k], ads[k], 1)
        assert torch.equal(out3[k * n:(k + 1) * n], o1)
        assert torch.equal(s3[k * 2 * C:(k + 1) * 2 * C], s1), k


@pytest.mark.parametrize("graph,copies", [("lattice", 1), ("lattice", 3), ("lattice", 5), ("stress", 1),
                                          ("stress", 3), ("star", 3)])
@pytest.mark.parametrize("C", [4, 8, 12, 16, 24])
@pytest.mark.parametrize("drop", [False, True])
def test_fused_fold_apply_bitwise_equal_two_launches(cuda, graph, copies, C, drop):
    """vg_graphnorm_fwd_gnp as ONE launch on the narrow layers (k_gn_apply4_gnp:
    every workgroup folds its segment's partials, then applies): the statistics
    it stores are bit for bit vg_graphnorm_stats_gnp's (k_stats_final_gnp's fold
    order), every segment's are written (buffer pre-filled with NaN; small
    segments put several in one workgroup's range), y matches an fp32 apply of
    those statistics and the dropout multipliers are vg_graphnorm_fwd_drop's."""
    torch.manual_seed(C + 11 * copies)
    csr = _csr(cuda, graph, copies)
    n, seg = csr.num_nodes, csr.seg_rows
    S = n // seg
    gnp, g = ops.gnp_buffer(csr, C, cuda)
    fused = int(LIB.vg_graphnorm_fwd_gnp_fused(seg, C, g))
    if graph != "stress":
        assert fused == 1, (seg, C, g)
    h = torch.randn(n, C, device=cuda)
    a_s, a_d = 0.5 * torch.randn(n, device=cuda), 0.5 * torch.randn(n, device=cuda)
    b = torch.randn(C, device=cuda)
    out, alpha = torch.empty_like(h), torch.empty(csr.num_edges, device=cuda)
    st = ops.stream_handle(cuda)
    ops.aggregate_fwd_raw(csr, C, ptr(h), ptr(a_s), ptr(a_d), ptr(b), 0.2, ptr(out), ptr(alpha), st, gnp)
    w = 1 + 0.2 * torch.randn(C, device=cuda)
    bb = 0.2 * torch.randn(C, device=cuda)
    ms = torch.rand(C, device=cuda) + 0.2
    it = torch.tensor([3], dtype=torch.int64, device=cuda)
    y1, k1 = torch.empty_like(out), torch.empty_like(out)
    s1 = torch.full((S * 2 * C,), float("nan"), device=cuda)
    check(LIB.vg_graphnorm_fwd_gnp(ptr(out), S, seg, C, ptr(w), ptr(bb), ptr(ms), None, 0.2 if drop else 0.0,
                                   99, ptr(it) if drop else None, 5, EPS, ptr(y1), ptr(k1) if drop else None,
                                   ptr(s1), ptr(gnp), g, st), "vg_graphnorm_fwd_gnp")
    s2 = torch.empty(S * 2 * C, device=cuda)
    check(LIB.vg_graphnorm_stats_gnp(S, seg, C, ptr(gnp), g, ptr(ms), EPS, ptr(s2), st), "vg_graphnorm_stats_gnp")
    torch.cuda.synchronize()
    assert torch.equal(s1, s2)
    sv = s2.view(S, 2, C)
    mu, d = sv[:, 0].repeat_interleave(seg, 0), sv[:, 1].repeat_interleave(seg, 0)
    y_ref = torch.relu((out - mu * ms) / d * w + bb)
    if drop:
        y2, k2 = torch.empty_like(out), torch.empty_like(out)
        ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(S, seg, C)), device=cuda)
        check(LIB.vg_graphnorm_fwd_drop(ptr(out), S, seg, C, ptr(w), ptr(bb), ptr(ms), 0.2, 99, ptr(it), 5, EPS,
                                        ptr(y2), ptr(k2), ptr(s2), ptr(ws), None, st), "vg_graphnorm_fwd_drop")
        torch.cuda.synchronize()
        assert torch.equal(k1, k2)
        y_ref = y_ref * k1
    assert (y1 - y_ref).abs().max().item() <= 1e-5 * max(1.0, y_ref.abs().max().item())
