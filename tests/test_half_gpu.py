"""f16 inference path (configs[4]): every f16 kernel against an f32 reference
of the same op on the same (f16-representable) inputs, the whole f16 generator
forward against the f32 one, and the graphed f16 inference sweep.

Tolerances: a kernel's f16 output may differ from the f32 reference by the
final rounding to binary16 (relative 2^-11) plus f32 accumulation-order
differences -- bounded here by 4e-3 relative to the output scale.  The whole
forward (5 + 5 + 4 + 1 GEMM layers, 14 GAT blocks through a 1-channel
bottleneck whose GraphNorm rescales every rounding error) compounds f16 storage
rounding: bounded by 2e-2 RMS relative error of the logits, 5e-2 (99th
percentile) and 0.2 (max) of their scale, and >= 97% agreement of the
predicted types (argmax of the logits)."""
import pytest
import torch

from vgan import data as vdata
from vgan import ops
from vgan._lib import LIB, check, ptr, stream_handle
from vgan.config import Configuration
from vgan.half import HalfGenerator, _r8
from vgan.infer import InferenceSweep, geometric_taus
from vgan.models import VoxelGNNGenerator
from vgan.synth import SyntheticDataset

pytestmark = pytest.mark.gpu


def _h16(rows, cols, ld, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.zeros(rows, ld, dtype=torch.float16)
    x[:, :cols] = (torch.randn(rows, cols, generator=g) * scale).half()
    return x.to(dev)


def _close(got, want, tol=4e-3):
    scale = want.abs().max().clamp_min(1e-3)
    err = (got.float() - want.float()).abs().max() / scale
    assert err < tol, float(err)


@pytest.mark.parametrize("n,m,k", [(1000, 128, 128), (333, 64, 528), (77, 7, 16), (4100, 16, 272), (50, 1, 8)])
def test_hgemm_bias_act(cuda, n, m, k):
    a = _h16(n, k, k, cuda, seed=1)
    w = _h16(m, k, k, cuda, scale=0.1, seed=2)
    b = torch.randn(m, device=cuda)
    s = stream_handle(cuda)
    ref = a.float() @ w.float().t() + b
    for act, f in ((0, lambda v: v), (1, torch.relu), (2, lambda v: torch.nn.functional.leaky_relu(v, 0.2))):
        out = torch.full((n, m), float("nan"), device=cuda)
        check(LIB.vg_hgemm(ptr(a), k, ptr(w), k, n, m, k, ptr(b), act, 0.2, ptr(out), m, 1, s), "vg_hgemm")
        _close(out, f(ref))
        ldo = _r8(m) + 8
        o16 = torch.full((n, ldo), float("nan"), dtype=torch.float16, device=cuda)
        check(LIB.vg_hgemm(ptr(a), k, ptr(w), k, n, m, k, ptr(b), act, 0.2, ptr(o16), ldo, 0, s), "vg_hgemm")
        _close(o16[:, :m], f(ref))
        assert torch.all(o16[:, m:_r8(m)] == 0)  # pad columns written as 0
        assert torch.isnan(o16[:, _r8(m):]).all()  # nothing beyond the padded width


@pytest.mark.parametrize("n,m,k", [(1000, 128, 272), (513, 64, 128), (129, 16, 32)])
def test_hgemm_ln_act(cuda, n, m, k):
    a = _h16(n, k, k, cuda, seed=3)
    w = _h16(m, k, k, cuda, scale=0.1, seed=4)
    b, g, be = torch.randn(m, device=cuda), torch.rand(m, device=cuda) + 0.5, torch.randn(m, device=cuda)
    out = torch.empty(n, m, dtype=torch.float16, device=cuda)
    check(LIB.vg_hgemm_ln_act(ptr(a), k, ptr(w), k, n, m, k, ptr(b), ptr(g), ptr(be), 1e-5, 0.2, ptr(out), m,
                              stream_handle(cuda)), "vg_hgemm_ln_act")
    ref = torch.nn.functional.leaky_relu(
        torch.nn.functional.layer_norm(a.float() @ w.float().t() + b, (m,), g, be, 1e-5), 0.2)
    _close(out, ref)


@pytest.mark.parametrize("cin,cout", [(128, 64), (8, 1), (16, 2), (64, 128)])
def test_hgat_lin_att_and_aggregate(cuda, cin, cout):
    loc, vox = SyntheticDataset(8, seed=4).batch(range(3))
    loc, vox = loc.to(cuda), vox.to(cuda)
    csr = vdata.prepared(loc, vox, 7).csr
    n = vox.num_nodes
    x = _h16(n, cin, _r8(cin), cuda, seed=5)
    w = _h16(cout, cin, _r8(cin), cuda, scale=0.2, seed=6)
    att_s, att_d = torch.randn(cout, device=cuda) * 0.3, torch.randn(cout, device=cuda) * 0.3
    bias = torch.randn(cout, device=cuda)
    s = stream_handle(cuda)
    ldh = _r8(cout)
    h = torch.empty(n, ldh, dtype=torch.float16, device=cuda)
    a_s, a_d = torch.empty(n, device=cuda), torch.empty(n, device=cuda)
    check(LIB.vg_hgat_lin_att(ptr(x), _r8(cin), ptr(w), _r8(cin), n, _r8(cin), cout, ptr(att_s), ptr(att_d), ptr(h),
                              ldh, ptr(a_s), ptr(a_d), s), "vg_hgat_lin_att")
    href = x.float()[:, :cin] @ w.float()[:, :cin].t()
    _close(h[:, :cout], href)
    assert torch.all(h[:, cout:] == 0)
    _close(a_s, href @ att_s)
    _close(a_d, href @ att_d)
    # aggregation on the f16 h vs the f32 scatter kernel on the same values
    out = torch.empty_like(h)
    check(LIB.vg_hgat_fwd(ptr(csr.row_ptr), ptr(csr.col), n, cout, ldh, ptr(h), ptr(a_s), ptr(a_d), ptr(bias), 0.2,
                          ptr(out), ldh, s), "vg_hgat_fwd")
    h32 = h[:, :cout].float().contiguous()
    ref = ops.gat_conv(csr, h32, att_s.view(1, 1, -1), att_d.view(1, 1, -1), bias, 0.2, pre=(a_s, a_d))
    _close(out[:, :cout], ref)
    assert torch.all(out[:, cout:] == 0)


@pytest.mark.parametrize("c,segs", [(128, 1), (1, 3), (32, 2)])
def test_graphnorm_fwd_h(cuda, c, segs):
    n = 3001
    ld = _r8(c)
    x = _h16(segs * n, c, ld, cuda, scale=2.0, seed=7) + 0.5
    w, b, ms = torch.rand(c, device=cuda) + 0.5, torch.randn(c, device=cuda), torch.rand(c, device=cuda)
    s = stream_handle(cuda)
    ldy = ld + 16  # y as a column slice of a wider row
    y = torch.full((segs * n, ldy), float("nan"), dtype=torch.float16, device=cuda)
    stats = torch.empty(segs * 2 * c, device=cuda)
    ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(segs, n, c)), device=cuda)
    check(LIB.vg_graphnorm_fwd_h(ptr(x), ld, segs, n, c, ptr(w), ptr(b), ptr(ms), 1e-5, ptr(y), ldy, ptr(stats),
                                 ptr(ws), s), "vg_graphnorm_fwd_h")
    xs = x[:, :c].float().view(segs, n, c)
    mu = xs.mean(1, keepdim=True)
    o = xs - mu * ms
    d = (o.pow(2).mean(1, keepdim=True) + 1e-5).sqrt()  # PyG 2.6.1 GraphNorm(batch=None)
    ref = torch.relu(w * o / d + b).reshape(segs * n, c)
    _close(y[:, :c], ref)
    assert torch.all(y[:, c:ld] == 0)
    assert torch.isnan(y[:, ld:]).all()


@pytest.mark.parametrize("copies", [1, 3, 10])
@pytest.mark.parametrize("c", [1, 4, 8, 16, 32, 64, 128])
def test_hgat_gnp_partials_and_graphnorm(cuda, c, copies):
    """vg_hgat_fwd_gnp: the same f16 output as vg_hgat_fwd bit for bit, plus the
    following GraphNorm's column partials per segment-aligned block, from which
    vg_graphnorm_fwd_h_gnp's statistics match vg_graphnorm_fwd_h's statistics
    pass over the stored halves (f32 Welford in another grouping: 1e-5) and
    an f64 GraphNorm of the f16 output; every partial the fold reads is
    written (buffer pre-filled with NaN).  Stacked copies: the sweep's
    temperatures, each normalised on its own."""
    loc, vox = SyntheticDataset(8, seed=4).batch(range(3))
    loc, vox = loc.to(cuda), vox.to(cuda)
    base = vdata.prepared(loc, vox, 7).csr
    n = vox.num_nodes
    csr = base.stacked(copies) if copies > 1 else base
    rows = csr.num_nodes
    ld = _r8(c)
    h = _h16(rows, c, ld, cuda, seed=8)
    a_s, a_d = 0.4 * torch.randn(rows, device=cuda), 0.4 * torch.randn(rows, device=cuda)
    bias = torch.randn(c, device=cuda)
    s = stream_handle(cuda)
    g = int(LIB.vg_hgat_gnp_rows(rows, ld))
    assert 0 < g <= n
    gnp = torch.full((int(LIB.vg_hgat_gnp_floats(rows, ld)),), float("nan"), device=cuda)
    o1, o2 = torch.empty(rows, ld, dtype=torch.float16, device=cuda), torch.empty(rows, ld, dtype=torch.float16,
                                                                                   device=cuda)
    check(LIB.vg_hgat_fwd_gnp(ptr(csr.row_ptr), ptr(csr.col), rows, c, ld, ptr(h), ptr(a_s), ptr(a_d), ptr(bias), 0.2,
                              ptr(o1), ld, n, ptr(gnp), s), "vg_hgat_fwd_gnp")
    check(LIB.vg_hgat_fwd(ptr(csr.row_ptr), ptr(csr.col), rows, c, ld, ptr(h), ptr(a_s), ptr(a_d), ptr(bias), 0.2,
                          ptr(o2), ld, s), "vg_hgat_fwd")
    w, b, ms = torch.rand(c, device=cuda) + 0.5, torch.randn(c, device=cuda), torch.rand(c, device=cuda)
    y1, y2 = torch.empty_like(o1), torch.empty_like(o1)
    st1 = torch.full((copies * 2 * c,), float("nan"), device=cuda)
    st2 = torch.empty(copies * 2 * c, device=cuda)
    check(LIB.vg_graphnorm_fwd_h_gnp(ptr(o1), ld, copies, n, c, ptr(w), ptr(b), ptr(ms), 1e-5, ptr(y1), ld, ptr(st1),
                                     ptr(gnp), g, s), "vg_graphnorm_fwd_h_gnp")
    ws = torch.empty(int(LIB.vg_graphnorm_seg_ws_floats(copies, n, c)), device=cuda)
    check(LIB.vg_graphnorm_fwd_h(ptr(o2), ld, copies, n, c, ptr(w), ptr(b), ptr(ms), 1e-5, ptr(y2), ld, ptr(st2),
                                 ptr(ws), s), "vg_graphnorm_fwd_h")
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert torch.isfinite(st1).all()
    assert (st1 - st2).abs().max().item() <= 1e-5 * max(1.0, st2.abs().max().item())
    xs = o1[:, :c].double().view(copies, n, c)
    mu = xs.mean(1, keepdim=True)
    d = ((xs - mu * ms.double()).pow(2).mean(1, keepdim=True) + 1e-5).sqrt()
    ref = torch.relu(w.double() * (xs - mu * ms.double()) / d + b.double()).reshape(rows, c)
    _close(y1[:, :c], ref)
    _close(y1[:, :c], y2[:, :c].float())
    assert torch.all(y1[:, c:] == 0)


@pytest.mark.parametrize("copies", [1, 4, 16])
@pytest.mark.parametrize("cprev,cout", [(64, 32), (1, 2), (4, 8), (16, 128), (128, 64)])
def test_hgat_lin_att_gn_equals_apply_then_project(cuda, cprev, cout, copies):
    """vg_hgat_lin_att_gn (the previous block's GraphNorm + ReLU applied as the
    projection loads its operand) against vg_graphnorm_fwd_h_gnp's stored f16
    output projected by vg_hgat_lin_att: h, a_src and a_dst bit for bit (the
    same f16 operand values reach the MFMA); copies up to the 16 segments the
    kernel stages; the statistics of vg_graphnorm_stats_gnp are those the
    apply folds."""
    loc, vox = SyntheticDataset(8, seed=4).batch(range(3))
    loc, vox = loc.to(cuda), vox.to(cuda)
    base = vdata.prepared(loc, vox, 7).csr
    n = vox.num_nodes
    csr = base.stacked(copies) if copies > 1 else base
    rows = csr.num_nodes
    ldp, ldh = _r8(cprev), _r8(cout)
    s = stream_handle(cuda)
    hp = _h16(rows, cprev, ldp, cuda, seed=9)
    a_s0, a_d0 = 0.4 * torch.randn(rows, device=cuda), 0.4 * torch.randn(rows, device=cuda)
    bias = torch.randn(cprev, device=cuda)
    g = int(LIB.vg_hgat_gnp_rows(rows, ldp))
    gnp = torch.empty(int(LIB.vg_hgat_gnp_floats(rows, ldp)), device=cuda)
    agg = torch.empty(rows, ldp, dtype=torch.float16, device=cuda)
    check(LIB.vg_hgat_fwd_gnp(ptr(csr.row_ptr), ptr(csr.col), rows, cprev, ldp, ptr(hp), ptr(a_s0), ptr(a_d0),
                              ptr(bias), 0.2, ptr(agg), ldp, n, ptr(gnp), s), "vg_hgat_fwd_gnp")
    gw, gb, gms = torch.rand(cprev, device=cuda) + 0.5, 0.3 * torch.randn(cprev, device=cuda), torch.rand(cprev,
                                                                                                        device=cuda)
    st1, st2 = torch.empty(copies * 2 * cprev, device=cuda), torch.empty(copies * 2 * cprev, device=cuda)
    y = torch.empty_like(agg)
    check(LIB.vg_graphnorm_fwd_h_gnp(ptr(agg), ldp, copies, n, cprev, ptr(gw), ptr(gb), ptr(gms), 1e-5, ptr(y), ldp,
                                     ptr(st1), ptr(gnp), g, s), "vg_graphnorm_fwd_h_gnp")
    check(LIB.vg_graphnorm_stats_gnp(copies, n, cprev, ptr(gnp), g, ptr(gms), 1e-5, ptr(st2), s),
          "vg_graphnorm_stats_gnp")
    w = _h16(cout, cprev, ldp, cuda, scale=0.2, seed=10)
    att_s, att_d = torch.randn(cout, device=cuda) * 0.3, torch.randn(cout, device=cuda) * 0.3
    outs = []
    for fused in (True, False):
        h = torch.full((rows, ldh), float("nan"), dtype=torch.float16, device=cuda)
        a_s, a_d = torch.empty(rows, device=cuda), torch.empty(rows, device=cuda)
        if fused:
            check(LIB.vg_hgat_lin_att_gn(ptr(agg), ldp, ptr(w), ldp, rows, ldp, cout, ptr(att_s), ptr(att_d), ptr(h),
                                         ldh, ptr(a_s), ptr(a_d), ptr(gw), ptr(gb), ptr(gms), ptr(st2), copies, n,
                                         cprev, s), "vg_hgat_lin_att_gn")
        else:
            check(LIB.vg_hgat_lin_att(ptr(y), ldp, ptr(w), ldp, rows, ldp, cout, ptr(att_s), ptr(att_d), ptr(h), ldh,
                                      ptr(a_s), ptr(a_d), s), "vg_hgat_lin_att")
        outs.append((h, a_s, a_d))
    torch.cuda.synchronize()
    assert torch.equal(st1, st2)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert torch.all(outs[0][0][:, cout:] == 0)
    bad = LIB.vg_hgat_lin_att_gn(ptr(agg), ldp, ptr(w), ldp, rows, ldp, cout, ptr(att_s), ptr(att_d), ptr(outs[0][0]),
                                 ldh, ptr(outs[0][1]), ptr(outs[0][2]), ptr(gw), ptr(gb), ptr(gms), ptr(st2), 17,
                                 rows // 17 if rows % 17 == 0 else 1, cprev, s)
    assert bad != 0  # more segments than the kernel stages, or a split that does not cover n


@pytest.fixture(scope="module")
def gen_batch(cuda):
    cfg = Configuration()
    torch.manual_seed(11)
    G = VoxelGNNGenerator(cfg, 17, 12).to(cuda).eval()
    loc, vox = SyntheticDataset(16, seed=9).batch(range(4))
    return cfg, G, loc.to(cuda), vox.to(cuda)


@pytest.mark.parametrize("k", [1, 3])
def test_half_generator_matches_f32_forward(cuda, gen_batch, k):
    cfg, G, loc, vox = gen_batch
    n = vox.num_nodes
    z = torch.randn(k, n, cfg.Z_DIM, device=cuda)
    noise = torch.empty(k * n, 7, device=cuda).exponential_()
    with torch.no_grad():
        l32, _, _ = G(loc, vox, z, noise=noise.view(k, n, 7) if k > 1 else noise)
    hg = HalfGenerator(G)
    l16, h16, s16 = hg(loc, vox, z, noise=noise)
    l32 = l32.reshape(-1, 7)
    l16 = l16.reshape(-1, 7)
    d = (l16 - l32).abs()
    rms = float(d.pow(2).mean().sqrt() / l32.pow(2).mean().sqrt())
    p99 = float(d.flatten().kthvalue(int(0.99 * d.numel())).values / l32.abs().max())
    mx = float(d.max() / l32.abs().max())
    agree = float((l16.argmax(1) == l32.argmax(1)).float().mean())
    print(f"k={k}: logits16 vs logits32: rms rel {rms:.2e}, p99 {p99:.2e}, max {mx:.2e} (of max|logits|); "
          f"argmax agreement {agree:.4f}")
    assert rms < 2e-2 and p99 < 5e-2 and mx < 0.2
    assert agree >= 0.97
    assert torch.all(h16.sum(-1) == 1)


def test_half_sweep_graphed(cuda, gen_batch):
    """The f16 sweep captures and replays; replays draw fresh z / noise."""
    cfg, G, loc, vox = gen_batch
    taus = geometric_taus(1.0, 0.1, 4)
    sw = InferenceSweep(G, taus, graphed=True, dtype="f16")
    a = sw.run_batch(loc, vox).clone()
    b = sw.run_batch(loc, vox).clone()
    assert a.shape == (len(taus), vox.num_nodes) and a.dtype == torch.int8
    assert int(a.min()) >= 0 and int(a.max()) < 7
    assert not torch.equal(a, b)
    res = InferenceSweep(G, taus, graphed=False, dtype="f16").run([(loc, vox)])
    assert res["samples"] == vox.num_graphs * len(taus)
