"""configs[3] at full size: 8 x 50k-voxel stress buildings (20 floors of 50 x 50,
4-neighbour floors plus 3 x 3 blocks to the floors above and below; N = 400,000,
E' = 8,626,816 with the self loops), the scatter / LDS bandwidth stress graph the
bench times.

* every aggregation kernel -- the register gather (vg_gat_aggregate_fwd: the
  64-channel slice path at this size), the padded-column form (ELL), the
  16-row LDS tile kernel and the persistent staged kernel -- at C = 128 / 64 / 1
  where it applies, in three voxel numberings (the reference's row-major, 4 x 4
  floor tiles, 4 x 4 x 4 lattice blocks), against the f64 oracle
  (``oracle.pyg.gat_propagate``, the restated PyG 2.6.1 GATConv propagate) on
  ~5,000 sampled destination rows -- the rows' exact in-edge subgraphs, so the
  oracle sees the same softmax segments -- and bit for bit against each other;
* one GATConv block (64 -> 128 channels) forward and backward on the whole
  graph against autograd of the oracle's GATConv in f64: the upstream gradient
  lives on the sampled rows, so every gradient (x, lin.weight, att_src,
  att_dst, bias) is exactly that of the rows' subgraph.

Match: models.py:144 (GATConv in the encoder stacks), SURVEY.md 8(d) cfg #4.
"""
import pytest
import torch

from oracle import pyg
from parity_util import rel_err
from vgan import ops, synth
from vgan._lib import LIB, check, ptr
from vgan.graph import GraphBatch
from vgan.locality import blocked, tiled

pytestmark = pytest.mark.gpu

ORDERS = ("rowmajor", "tiled", "blocked")


@pytest.fixture(scope="module")
def stress_items():
    return [synth.make_stress_building(777, i)[1] for i in range(8)]


_GRAPHS = {}


def _graph(order, items, cuda):
    if order not in _GRAPHS:
        vs = items if order == "rowmajor" else [tiled(v, 4)[0] if order == "tiled" else blocked(v)[0] for v in items]
        vox = GraphBatch.from_data_list(vs)
        ei = vox.edge_index
        csr = ops.CSR(ei.to(cuda), vox.num_nodes)
        _GRAPHS.clear()  # one numbering resident at a time
        _GRAPHS[order] = (ei, vox.num_nodes, csr)
    return _GRAPHS[order]


def _sample_rows(n, seed=0, k=4096):
    g = torch.Generator().manual_seed(seed)
    edges = torch.cat([torch.arange(64), torch.arange(n - 64, n)]
                      + [torch.arange(b * 50000 - 8, b * 50000 + 8) for b in range(1, 8)])
    return torch.unique(torch.cat([torch.randint(0, n, (k,), generator=g), edges]))


def _subgraph(ei, rows):
    """The rows' in-edges (self loops removed: GATConv re-adds them), relabelled
    onto the compact node set V = rows + their sources; (V, edges, rows in V)."""
    ei = pyg.remove_self_loops(ei)
    sub = ei[:, torch.isin(ei[1], rows)]
    V = torch.unique(torch.cat([rows, sub[0]]))
    return V, torch.searchsorted(V, sub), torch.searchsorted(V, rows)


def _oracle_rows(h, a_s, a_d, bias, ei, rows):
    V, sub, rl = _subgraph(ei, rows)
    out = pyg.gat_propagate(h.cpu()[V].double(), a_s.cpu()[V].double(), a_d.cpu()[V].double(), sub)
    return (out + bias.cpu().double())[rl]


def _run(kind, csr, c, h, a_s, a_d, b):
    n = csr.num_nodes
    out = torch.empty(n, c, device=h.device)
    alpha = torch.empty(csr.num_edges, device=h.device)
    args = (c, ptr(h), ptr(a_s), ptr(a_d), ptr(b), 0.2, ptr(out), ptr(alpha))
    if kind == "register":
        check(LIB.vg_gat_aggregate_fwd(ptr(csr.row_ptr), ptr(csr.col), n, *args, csr.stream()), kind)
    elif kind == "ell":
        ell, w = csr.ell()
        assert ell is not None and w == 32  # the stress lattice's largest degree is 23
        check(LIB.vg_gat_aggregate_fwd_ell(ptr(csr.row_ptr), ptr(csr.col), ptr(ell), w, n, *args, csr.stream()), kind)
    elif kind == "lds":
        plan = csr.tile_plan()
        check(LIB.vg_gat_aggregate_fwd_lds(ptr(csr.row_ptr), ptr(csr.col), n, *args, ptr(plan), csr._tile_umax,
                                           csr.stream()), kind)
    elif kind == "staged":
        check(LIB.vg_gat_aggregate_fwd_staged(ptr(csr.row_ptr), ptr(csr.col), n, *args, ptr(csr.stage_plan()),
                                              csr.stream()), kind)
    else:  # the wave-specialised ring
        err = torch.zeros(1, dtype=torch.int32, device=h.device)
        check(LIB.vg_gat_aggregate_fwd_ring(ptr(csr.row_ptr), ptr(csr.col), n, *args, ptr(csr.ring_plan()), ptr(err),
                                            csr.stream()), kind)
        assert int(err.item()) == 0, "ring hand-over wait expired"
    return out, alpha


@pytest.mark.parametrize("order", ORDERS)
@pytest.mark.parametrize("C", [128, 64, 1])
def test_stress_aggregations_against_oracle(cuda, stress_items, order, C):
    ei, n, csr = _graph(order, stress_items, cuda)
    assert n == 400000 and csr.num_edges == 8626816
    torch.manual_seed(C)
    h = torch.randn(n, C, device=cuda)
    a_s, a_d = 0.5 * torch.randn(n, device=cuda), 0.5 * torch.randn(n, device=cuda)
    b = torch.randn(C, device=cuda)
    kinds = ["register", "ell"] + (["lds"] if C % 64 == 0 else []) + (["staged", "ring"] if C in (64, 128) else [])
    outs = {k: _run(k, csr, C, h, a_s, a_d, b) for k in kinds}
    torch.cuda.synchronize()
    ref_out, ref_alpha = outs["register"]
    for k in kinds[1:]:  # the same 16-lane softmax grouping and gather order: bit for bit
        assert torch.equal(outs[k][0], ref_out), k
        assert torch.equal(outs[k][1], ref_alpha), k
    rows = _sample_rows(n, seed=C)
    want = _oracle_rows(h, a_s, a_d, b, ei, rows)
    err = rel_err(ref_out.cpu()[rows], want)
    print(f"{order} C={C}: {len(rows)} rows, rel err vs f64 oracle {err:.2e}")
    assert err < 1e-5
    if "staged" in kinds:
        ucount = csr.stage_plan()[:csr.stage_tiles()].cpu()
        print(f"{order}: {int((ucount > 0).sum())} staged tiles, {int((ucount < 0).sum())} from global memory")
        if order == "blocked":
            assert (ucount > 0).all()  # every 4 x 4 x 4 block fits the 288-row image


def test_stress_gat_block_forward_backward_against_oracle(cuda, stress_items):
    from vgan.models import GATConv

    ei, n, csr = _graph("blocked", stress_items, cuda)
    torch.manual_seed(5)
    conv = GATConv(64, 128).to(cuda)
    with torch.no_grad():
        conv.bias.normal_()
    ref = pyg.GATConv(64, 128).double()
    ref.load_state_dict({k: v.detach().cpu().double() for k, v in conv.state_dict().items()})
    x = torch.randn(n, 64, device=cuda, requires_grad=True)
    y = conv(x, csr)
    rows = _sample_rows(n, seed=7, k=2048)
    g = torch.zeros(n, 128, device=cuda)
    g[rows.to(cuda)] = torch.randn(len(rows), 128, device=cuda)
    y.backward(g)
    torch.cuda.synchronize()
    V, sub, rl = _subgraph(ei, rows)
    xr = x.detach().cpu()[V].double().requires_grad_(True)
    yr = ref(xr, sub)
    (yr[rl] * g.cpu()[rows].double()).sum().backward()
    assert rel_err(y.detach().cpu()[rows], yr.detach()[rl]) < 1e-5
    gx = x.grad.cpu()
    outside = torch.ones(n, dtype=torch.bool)
    outside[V] = False
    assert torch.count_nonzero(gx[outside]) == 0  # no gradient outside the rows' subgraph
    errs = {"x": rel_err(gx[V], xr.grad)}
    for name, p in conv.named_parameters():
        errs[name] = rel_err(p.grad.cpu().reshape(-1), dict(ref.named_parameters())[name].grad.reshape(-1))
    print({k: f"{v:.2e}" for k, v in errs.items()})
    for k, v in errs.items():
        assert v < 1e-4, k


@pytest.mark.parametrize("C", [64, 128])
def test_ring_aggregation_ragged_graph_bitwise(cuda, C):
    """The wave-specialised ring kernel on a graph that exercises its other
    paths: a ragged last tile (N % 64 != 0), rows with no in-edges, hub rows
    longer than 64 edges (their tiles aggregated from global memory) and tiles
    with more distinct sources than the ring's 288-row image -- bit-identical to the
    register kernel, with the hand-over flag untouched."""
    from vgan import ops

    g = torch.Generator().manual_seed(C)
    n = 5000 + 37
    e_loc = torch.randint(0, 40, (2, 30000), generator=g)  # mostly local edges
    e_loc[1] = (e_loc[0] + torch.randint(0, 40, (30000,), generator=g)) % n
    e_loc[0] = (e_loc[0] * 97 + torch.randint(0, n, (30000,), generator=g) // 50) % n
    hubs = torch.stack([torch.randint(0, n, (600,), generator=g), torch.full((600,), 123)])  # deg 600 row
    wide = torch.stack([torch.randint(0, n, (900,), generator=g), torch.randint(640, 704, (900,), generator=g)])
    ei = torch.cat([e_loc, hubs, wide], 1)
    ei = ei[:, ei[1] != 4000]  # row 4000: only its self loop
    csr = ops.CSR(ei.to(cuda), n)
    torch.manual_seed(C)
    h = torch.randn(n, C, device=cuda)
    a_s, a_d = 0.5 * torch.randn(n, device=cuda), 0.5 * torch.randn(n, device=cuda)
    b = torch.randn(C, device=cuda)
    ref_out, ref_alpha = _run("register", csr, C, h, a_s, a_d, b)
    out, alpha = _run("ring", csr, C, h, a_s, a_d, b)
    torch.cuda.synchronize()
    ucount = csr.ring_plan()[:-(-n // LIB.vg_gat_ring_tile_rows())].cpu()  # the plan's per-tile counts
    assert (ucount < 0).any() and (ucount > 0).any()  # both tile kinds ran
    assert torch.equal(out, ref_out) and torch.equal(alpha, ref_alpha)


def _ragged_graph(n, seed):
    g = torch.Generator().manual_seed(seed)
    e_loc = torch.randint(0, 40, (2, 6 * n), generator=g)
    e_loc[1] = (e_loc[0] + torch.randint(0, 40, (6 * n,), generator=g)) % n
    e_loc[0] = (e_loc[0] * 97 + torch.randint(0, n, (6 * n,), generator=g) // 50) % n
    hubs = torch.stack([torch.randint(0, n, (300,), generator=g), torch.full((300,), 7)])  # a 300-edge row
    return torch.cat([e_loc, hubs], 1)


def _tile_partials_f64(out, rt, seg_rows):
    """(n, mean, M2) of every rt-row block of every segment, per column, f64."""
    x = out.double().cpu()
    rows, c = x.shape
    res = []
    for s0 in range(0, rows, seg_rows):
        for r0 in range(s0, s0 + seg_rows, rt):
            blk = x[r0:min(r0 + rt, s0 + seg_rows)]
            mu = blk.mean(0)
            res.append((blk.shape[0], mu, ((blk - mu) ** 2).sum(0)))
    return res


@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("shape", ["ragged", "stacked3"])
def test_ring_gnp_partials_and_statistics(cuda, C, shape):
    """vg_gat_aggregate_fwd_ring_gnp: output and alpha bit-identical to the
    register kernel; every 64-row tile's (count, mean, M2) per column against
    f64 of the output; the GraphNorm statistics folded from them
    (vg_graphnorm_stats_gnp with gnp_rows = 64) against f64 column statistics
    of each segment -- one ragged segment (N % 64 != 0, a 300-edge hub row left
    to global memory) and three stacked copies of a 64-row-aligned graph.
    Match: models.py:73-75 (GraphNorm after each GATConv)."""
    rt = int(LIB.vg_gat_ring_tile_rows())
    if shape == "ragged":
        n = 5000 + 37
        csr = ops.CSR(_ragged_graph(n, C).to(cuda), n)
    else:
        n1 = 64 * 79
        csr = ops.CSR(_ragged_graph(n1, C + 1).to(cuda), n1).stacked(3)
    n, seg = csr.num_nodes, csr.seg_rows
    S = n // seg
    torch.manual_seed(C)
    h = torch.randn(n, C, device=cuda) * 2 + 0.5
    a_s, a_d = 0.5 * torch.randn(n, device=cuda), 0.5 * torch.randn(n, device=cuda)
    b = torch.randn(C, device=cuda)
    ref_out, ref_alpha = _run("register", csr, C, h, a_s, a_d, b)
    out, alpha = torch.empty_like(ref_out), torch.empty_like(ref_alpha)
    gnp = torch.full((int(LIB.vg_gat_ring_gnp_floats(n, C)),), float("nan"), device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    check(LIB.vg_gat_aggregate_fwd_ring_gnp(ptr(csr.row_ptr), ptr(csr.col), n, C, ptr(h), ptr(a_s), ptr(a_d), ptr(b),
                                            0.2, ptr(out), ptr(alpha), ptr(csr.ring_plan()), seg, ptr(gnp), ptr(err),
                                            csr.stream()), "vg_gat_aggregate_fwd_ring_gnp")
    ms = torch.rand(C, device=cuda) + 0.2
    stats = torch.empty(S * 2 * C, device=cuda)
    check(LIB.vg_graphnorm_stats_gnp(S, seg, C, ptr(gnp), rt, ptr(ms), 1e-5, ptr(stats), csr.stream()),
          "vg_graphnorm_stats_gnp")
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert torch.equal(out, ref_out) and torch.equal(alpha, ref_alpha)
    tiles = -(-n // rt)
    assert (csr.ring_plan()[:tiles] < 0).any() and (csr.ring_plan()[:tiles] > 0).any()
    part = gnp[:tiles * 2 * C * 3].view(tiles, 2, C, 3)[:, 0].double().cpu()
    want = _tile_partials_f64(out, rt, seg)
    assert len(want) == tiles
    wn = torch.tensor([w[0] for w in want], dtype=torch.float64)
    wmu = torch.stack([w[1] for w in want])
    wm2 = torch.stack([w[2] for w in want])
    assert torch.equal(part[:, 0, 0], wn)
    assert rel_err(part[:, :, 1], wmu) < 1e-6
    assert rel_err(part[:, :, 2], wm2) < 1e-5
    x = out.double().cpu().view(S, seg, C)
    mu = x.mean(1)
    o = x - ms.double().cpu() * mu.unsqueeze(1)
    d = (o.pow(2).mean(1) + 1e-5).sqrt()
    st = stats.double().cpu().view(S, 2, C)
    print(f"{shape} C={C}: stats rel err mean {rel_err(st[:, 0], mu):.2e}, denom {rel_err(st[:, 1], d):.2e}")
    assert rel_err(st[:, 0], mu) < 1e-6 and rel_err(st[:, 1], d) < 1e-6
