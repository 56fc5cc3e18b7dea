"""HIP operators vs the CPU oracle (torch-geometric 2.6.1 semantics restated).

Tolerances (fp32 kernels vs fp64/fp32 CPU oracle): forward 1e-5 relative
(order-of-summation only); gradients 1e-4 relative; double backward 1e-4.
"""
import pytest
import torch

from oracle import pyg
from oracle.reference import type_matched_mean
from parity_util import rel_err
from vgan import ops, synth

pytestmark = pytest.mark.gpu


def _graph(numbers=(1, 2), stress=False):
    items = [(synth.make_stress_building(777, n, F=3, Y=9, X=9) if stress else synth.make_building(777, n))
             for n in numbers]
    from vgan.graph import GraphBatch

    loc = GraphBatch.from_data_list([l for l, _ in items])
    vox = GraphBatch.from_data_list([v for _, v in items])
    return loc, vox


def _expected_csr(ei, n):
    """Reference edge order of GATConv: remove loops, append loops; rows by dst."""
    ei2 = pyg.add_self_loops(pyg.remove_self_loops(ei), n)
    rows = [[] for _ in range(n)]
    for k in range(ei2.shape[1]):
        rows[int(ei2[1, k])].append(int(ei2[0, k]))
    return rows


def test_csr_matches_gatconv_edge_order(cuda):
    _, vox = _graph()
    ei = vox.edge_index.clone()
    # add explicit self loops + an isolated-ish node pattern to exercise removal
    ei = torch.cat([ei, torch.tensor([[0, 5], [0, 5]])], 1)
    n = vox.num_nodes
    csr = ops.CSR(ei.to(cuda), n)
    rows = _expected_csr(ei, n)
    rp, col = csr.row_ptr.cpu().tolist(), csr.col.cpu().tolist()
    assert rp[-1] == sum(len(r) for r in rows) == csr.num_edges
    for i in range(n):
        assert col[rp[i]:rp[i + 1]] == rows[i], i
    # CSC: for each source, the CSR slots pointing at it, ascending
    cp, cs, cd = csr.csc_ptr.cpu().tolist(), csr.csc_slot.cpu().tolist(), csr.csc_dst.cpu().tolist()
    for j in range(0, n, 37):
        slots = [k for k in range(rp[-1]) if col[k] == j]
        assert cs[cp[j]:cp[j + 1]] == slots
        for k, d in zip(cs[cp[j]:cp[j + 1]], cd[cp[j]:cp[j + 1]]):
            assert rp[d] <= k < rp[d + 1]


def test_csr_rejects_out_of_range(cuda):
    with pytest.raises(ValueError):
        ops.CSR(torch.tensor([[0, 9], [1, 0]], device=cuda), 3)


@pytest.mark.parametrize("C", [1, 2, 3, 4, 8, 16, 24, 32, 64, 100, 128, 130, 256])
@pytest.mark.parametrize("stress", [False, True])
def test_gat_forward_backward(cuda, C, stress):
    torch.manual_seed(C)
    _, vox = _graph(stress=stress)
    n = vox.num_nodes
    csr = ops.CSR(vox.edge_index.to(cuda), n)
    h = torch.randn(n, C, dtype=torch.float64, requires_grad=True)
    a_s = torch.randn(n, dtype=torch.float64, requires_grad=True)
    a_d = torch.randn(n, dtype=torch.float64, requires_grad=True)
    b = torch.randn(C, dtype=torch.float64, requires_grad=True)
    ref = pyg.gat_propagate(h, a_s, a_d, vox.edge_index) + b
    g_out = torch.randn(n, C, dtype=torch.float64)
    ref_grads = torch.autograd.grad(ref, (h, a_s, a_d, b), g_out)

    hc, asc, adc, bc = (t.detach().float().to(cuda).requires_grad_(True) for t in (h, a_s, a_d, b))
    out = ops.gat_aggregate(csr, hc, asc, adc, bc)
    assert rel_err(out, ref) < 1e-5
    grads = torch.autograd.grad(out, (hc, asc, adc, bc), g_out.float().to(cuda))
    for got, want in zip(grads, ref_grads):
        assert rel_err(got, want) < 1e-4
    # the primitive re-expression (create_graph path) agrees with the fused kernel
    comp = ops.gat_aggregate_composed(csr, hc, asc, adc, bc)
    assert rel_err(comp, out) < 1e-6


@pytest.mark.parametrize("C", [1, 8, 64])
def test_gat_double_backward(cuda, C):
    torch.manual_seed(3 + C)
    _, vox = _graph((4,))
    n = vox.num_nodes
    csr = ops.CSR(vox.edge_index.to(cuda), n)
    base = [torch.randn(n, C, dtype=torch.float64), torch.randn(n, dtype=torch.float64),
            torch.randn(n, dtype=torch.float64), torch.randn(C, dtype=torch.float64)]
    w1 = torch.randn(n, C, dtype=torch.float64)
    w2 = [torch.randn_like(t) for t in base]

    def second_order(fn, tensors, w1, w2):
        out = fn(*tensors)
        g = torch.autograd.grad((out * w1).sum(), tensors, create_graph=True)
        s = sum((gi * wi).sum() for gi, wi in zip(g, w2))
        res = torch.autograd.grad(s, tensors, allow_unused=True)
        return [torch.zeros_like(t) if r is None else r for r, t in zip(res, tensors)]

    ref_t = [t.clone().requires_grad_(True) for t in base]
    ref = second_order(lambda h, a, d, b: pyg.gat_propagate(h, a, d, vox.edge_index) + b, ref_t, w1, w2)
    gpu_t = [t.float().to(cuda).requires_grad_(True) for t in base]
    got = second_order(lambda h, a, d, b: ops.gat_aggregate(csr, h, a, d, b), gpu_t, w1.float().to(cuda),
                       [w.float().to(cuda) for w in w2])
    for g, r in zip(got, ref):
        assert rel_err(g, r) < 1e-4


@pytest.mark.parametrize("C", [1, 16, 64])
def test_gat_layer_double_backward_through_projection(cuda, C):
    """a_src = h @ att_src inside the graph (as in GATConv): second-order grads
    w.r.t. x and every parameter vs the oracle GATConv in float64."""
    torch.manual_seed(11 + C)
    _, vox = _graph((4,))
    n = vox.num_nodes
    csr = ops.CSR(vox.edge_index.to(cuda), n)
    cin = 2 * C
    conv = pyg.GATConv(cin, C).double()
    with torch.no_grad():
        conv.bias.uniform_(-0.3, 0.3)
    x0 = torch.randn(n, cin, dtype=torch.float64)
    w1 = torch.randn(n, C, dtype=torch.float64)

    def run(x, W, att_s, att_d, b, fn):
        out = fn(x, W, att_s, att_d, b)
        gx, = torch.autograd.grad((out * w1.to(out.device)).sum(), x, create_graph=True)
        pen = (gx.norm(dim=1) - 1).pow(2).mean()
        return torch.autograd.grad(pen, (x, W, att_s, att_d, b), allow_unused=True)

    def oracle_fn(x, W, a_s, a_d, b):
        h = x @ W.t()
        return pyg.gat_propagate(h, h @ a_s.view(-1), h @ a_d.view(-1), vox.edge_index) + b

    def hip_fn(x, W, a_s, a_d, b):
        h = x @ W.t()
        return ops.gat_aggregate(csr, h, torch.mv(h, a_s.view(-1)), torch.mv(h, a_d.view(-1)), b)

    params = [conv.lin.weight.detach(), conv.att_src.detach(), conv.att_dst.detach(), conv.bias.detach()]
    rt = [x0.clone().requires_grad_(True)] + [p.clone().requires_grad_(True) for p in params]
    ref = run(*rt, oracle_fn)
    w1 = w1.float().to(cuda)
    gt = [t.detach().float().to(cuda).requires_grad_(True) for t in rt]
    got = run(*gt, hip_fn)
    for g, r in zip(got, ref):
        if r is None:
            continue
        assert rel_err(g, r) < 1e-3


def test_sparse_primitives_adjoint_identities(cuda):
    torch.manual_seed(0)
    _, vox = _graph((5, 6))
    n = vox.num_nodes
    csr = ops.CSR(vox.edge_index.to(cuda), n)
    E = csr.num_edges
    w = torch.randn(E, device=cuda)
    x = torch.randn(n, 16, device=cuda)
    g = torch.randn(n, 16, device=cuda)
    # <spmm(w, x), g> == <x, spmm_t(w, g)> == <w, sddmm(g, x)>
    a = (ops.spmm(csr, w, x) * g).sum()
    b = (x * ops.spmm_t(csr, w, g)).sum()
    c = (w * ops.sddmm(csr, g, x)).sum()
    assert torch.allclose(a, b, rtol=1e-4) and torch.allclose(a, c, rtol=1e-4)
    v = torch.randn(n, device=cuda)
    e = torch.randn(E, device=cuda)
    assert torch.allclose((ops.gather(csr, v, True) * e).sum(), (v * ops.scatter_src(csr, e)).sum(), rtol=1e-4)
    assert torch.allclose((ops.gather(csr, v, False) * e).sum(), (v * ops.seg_sum(csr, e)).sum(), rtol=1e-4)


@pytest.mark.parametrize("C", [1, 2, 7, 16, 64, 128])
@pytest.mark.parametrize("with_keep", [False, True])
def test_graphnorm_relu_dropout(cuda, C, with_keep):
    torch.manual_seed(C)
    n = 3000
    x = (torch.randn(n, C, dtype=torch.float64) * 2 + 0.5)
    w = torch.rand(C, dtype=torch.float64) + 0.5
    b = torch.randn(C, dtype=torch.float64) * 0.3
    ms = torch.rand(C, dtype=torch.float64)
    keep = (torch.rand(n, C) > 0.2).double() / 0.8 if with_keep else None
    if C > 1:
        x[:, 0] = 1.25  # zero-variance column
    ts = [t.clone().requires_grad_(True) for t in (x, w, b, ms)]
    gn = pyg.GraphNorm(C).double()
    with torch.no_grad():
        gn.weight.copy_(w)
        gn.bias.copy_(b)
        gn.mean_scale.copy_(ms)
    ref = ops.graphnorm_relu_dropout_torch(ts[0], ts[1], ts[2], ts[3], keep, 1e-5)
    assert torch.allclose(ref, torch.relu(gn(x)) * (keep if keep is not None else 1.0))
    gy = torch.randn(n, C, dtype=torch.float64)
    ref_g = torch.autograd.grad(ref, ts, gy)
    gt = [t.float().to(cuda).requires_grad_(True) for t in (x, w, b, ms)]
    out = ops.graphnorm_relu_dropout(gt[0], gt[1], gt[2], gt[3], keep.float().to(cuda) if with_keep else None)
    assert rel_err(out, ref) < 1e-5
    got_g = torch.autograd.grad(out, gt, gy.float().to(cuda))
    for a, r in zip(got_g, ref_g):
        assert rel_err(a, r) < 1e-4


def test_graphnorm_double_backward(cuda):
    torch.manual_seed(1)
    n, C = 500, 8
    base = [torch.randn(n, C, dtype=torch.float64), torch.rand(C, dtype=torch.float64) + 0.5,
            torch.randn(C, dtype=torch.float64), torch.rand(C, dtype=torch.float64)]
    keep = (torch.rand(n, C) > 0.2).double() / 0.8
    w1 = torch.randn(n, C, dtype=torch.float64)
    w2 = [torch.randn_like(t) for t in base]

    def second(fn, ts, w1, w2):
        g = torch.autograd.grad((fn(*ts) * w1).sum(), ts, create_graph=True)
        res = torch.autograd.grad(sum((a * b).sum() for a, b in zip(g, w2)), ts, allow_unused=True)
        return [torch.zeros_like(t) if r is None else r for r, t in zip(res, ts)]

    rt = [t.clone().requires_grad_(True) for t in base]
    ref = second(lambda *a: ops.graphnorm_relu_dropout_torch(*a, keep, 1e-5), rt, w1, w2)
    gt = [t.float().to(cuda).requires_grad_(True) for t in base]
    kc = keep.float().to(cuda)
    got = second(lambda *a: ops.graphnorm_relu_dropout(*a, kc), gt, w1.float().to(cuda),
                 [w.float().to(cuda) for w in w2])
    for a, r in zip(got, ref):
        assert rel_err(a, r) < 1e-4


def test_type_mean(cuda):
    loc, vox = _graph((8, 9, 10))
    want = type_matched_mean(loc.x, loc.type, vox.type)
    got = ops.type_mean(loc.x.to(cuda), loc.type.to(cuda), vox.type.to(cuda), 7)
    assert torch.allclose(got.cpu(), want, atol=1e-6)
    # program graph without some types -> zeros for those voxels; empty program graph -> all zeros
    keep = loc.type != 4
    got2 = ops.type_mean(loc.x[keep].to(cuda), loc.type[keep].to(cuda), vox.type.to(cuda), 7)
    want2 = type_matched_mean(loc.x[keep], loc.type[keep], vox.type)
    assert torch.allclose(got2.cpu(), want2, atol=1e-6)
    assert (got2[vox.type.to(cuda) == 4] == 0).all()


def test_gumbel_head(cuda):
    torch.manual_seed(0)
    n, k = 4000, 7
    logits = torch.randn(n, k, requires_grad=True)
    noise = torch.empty(n, k).exponential_()
    soft = ((logits - noise.log()) / 1.0).softmax(-1)
    hard = torch.zeros_like(soft).scatter_(-1, soft.argmax(1, keepdim=True), 1.0)
    hard = hard - soft.detach() + soft
    gh, gs = torch.randn(n, k), torch.randn(n, k)
    ref_g, = torch.autograd.grad((hard * gh).sum() + (soft * gs).sum(), logits)
    lc = logits.detach().to(cuda).requires_grad_(True)
    h2, s2 = ops.gumbel_head(lc, noise.to(cuda))
    assert torch.allclose(s2.cpu(), soft, atol=1e-6)
    assert torch.equal(h2.cpu().argmax(1), hard.argmax(1))
    assert torch.allclose(h2.cpu(), hard, atol=1e-6)
    got_g, = torch.autograd.grad((h2 * gh.to(cuda)).sum() + (s2 * gs.to(cuda)).sum(), lc)
    assert torch.allclose(got_g.cpu(), ref_g, atol=1e-5)


def test_far_and_confusion(cuda):
    from oracle.reference import far_pairs
    from vgan.config import Configuration

    loc, vox = _graph((11, 12, 13, 14))
    torch.manual_seed(0)
    label = torch.randn(vox.num_nodes, 7).softmax(-1)
    og, orf = far_pairs(Configuration(), _oracle_voxel(vox), label.unsqueeze(0))
    gen, ref = ops.far_per_graph(vox.x.to(cuda), label.to(cuda), vox.ptr.to(cuda), vox.site_area.to(cuda))
    assert torch.allclose(gen.cpu(), og, rtol=1e-5) and torch.allclose(ref.cpu(), orf)
    conf, conf_all = ops.confusion(vox.type.to(cuda), label.to(cuda), vox.ptr.to(cuda))
    pred = label.argmax(1)
    want = torch.zeros(7, 7, dtype=torch.int32)
    want.index_put_((vox.type, pred), torch.ones_like(pred, dtype=torch.int32), accumulate=True)
    assert torch.equal(conf_all.cpu(), want) and torch.equal(conf.sum(0).cpu(), want)


def _oracle_voxel(vox):
    from oracle import pyg as P

    return P.Batch.from_data_list([P.Data(x=vox[g].x, site_area=vox[g].site_area) for g in range(vox.num_graphs)])


def test_adam_matches_torch(cuda):
    torch.manual_seed(0)
    p = torch.randn(5000)
    ref = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=2e-4, betas=(0.5, 0.999))
    pc, m, v = p.to(cuda), torch.zeros(5000, device=cuda), torch.zeros(5000, device=cuda)
    for t in range(1, 6):
        g = torch.randn(5000)
        ref.grad = g.clone()
        opt.step()
        ops.adam_flat(pc, g.to(cuda), m, v, 2e-4, 0.5, 0.999, 1e-8, 0.0, t)
    assert torch.allclose(pc.cpu(), ref.detach(), atol=1e-7, rtol=0)
