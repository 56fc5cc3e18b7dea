"""Voxel renumbering for gather locality (vgan.locality): a permutation inside
the building that keeps every edge in place, so every destination row sees its
sources in the reference's order -- the GATConv output is the permuted output
(CPU: the oracle's restated GATConv in f64; GPU: the HIP aggregation bit for
bit)."""
import pytest
import torch

from oracle import pyg
from vgan.graph import GraphData
from vgan.locality import block_order, blocked, renumber, tile_order, tiled
from vgan.synth import make_stress_building, make_building


def _destination_sources(ei, n):
    rows = [[] for _ in range(n)]
    for s, d in ei.t().tolist():
        rows[d].append(s)
    return rows


@pytest.mark.parametrize("maker", [make_building, make_stress_building])
def test_tiled_order_is_a_permutation_keeping_row_source_order(maker):
    _, v = maker(777, 3) if maker is make_building else maker(777, 0, F=3, Y=13, X=11)
    v2, perm = tiled(v, 4)
    n = v.num_nodes
    assert sorted(perm.tolist()) == list(range(n))
    assert torch.equal(v2.x, v.x[perm]) and torch.equal(v2.type, v.type[perm])
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(n)
    assert torch.equal(v2.edge_index, inv[v.edge_index])  # edges relabelled in place
    old, new = _destination_sources(v.edge_index, n), _destination_sources(v2.edge_index, n)
    for r in range(n):  # row r of the new numbering = old row perm[r], sources in the same order
        assert new[r] == [int(inv[s]) for s in old[int(perm[r])]]
    # a 16-row group of the new numbering is a 4 x 4 patch of one floor
    loc = v2.location[:16]
    assert len(set(loc[:, 0].tolist())) == 1 and (loc[:, 1].max() - loc[:, 1].min()) == 3


def test_gatconv_is_equivariant_under_renumbering():
    _, v = make_stress_building(777, 1, F=3, Y=9, X=10)
    v2, perm = tiled(v, 4)
    torch.manual_seed(0)
    conv = pyg.GATConv(16, 8).double()
    x = torch.randn(v.num_nodes, 16, dtype=torch.float64)
    y = conv(x, v.edge_index)
    y2 = conv(x[perm], v2.edge_index)
    assert torch.allclose(y2, y[perm], atol=1e-12, rtol=0)


def test_tile_order_keys():
    loc = torch.tensor([[0, 0, 5], [0, 0, 0], [1, 0, 0], [0, 4, 0], [0, 1, 1]])
    perm = tile_order(loc, 4)
    # floor 0 tile (0,0): (0,0,0), (0,1,1); floor 0 tile (0,1): (0,0,5); tile (1,0): (0,4,0); floor 1
    assert perm.tolist() == [1, 4, 0, 3, 2]


def test_block_order_is_a_3d_block_permutation():
    _, v = make_stress_building(777, 0, F=8, Y=12, X=12)
    v2, perm = blocked(v, (4, 4, 4))
    n = v.num_nodes
    assert sorted(perm.tolist()) == list(range(n))
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(n)
    assert torch.equal(v2.edge_index, inv[v.edge_index])
    # every 64-row group is one 4 x 4 x 4 block of the lattice
    for g in range(n // 64):
        loc = v2.location[64 * g:64 * g + 64]
        for c in range(3):
            assert int(loc[:, c].max() - loc[:, c].min()) == 3 and int(loc[:, c].min()) % 4 == 0
    # fewer distinct sources per 64-row tile than the floor tiles give
    def distinct(ei):
        dst, src = ei[1], ei[0]
        return sum(len(set(src[(dst >= lo) & (dst < lo + 64)].tolist())) for lo in range(0, n, 64)) / (n // 64)
    assert distinct(v2.edge_index) < 0.8 * distinct(tiled(v, 4)[0].edge_index)


def test_morton_block_order_keeps_blocks_and_groups_neighbours():
    """blocks="morton": still a permutation whose 64-row groups are whole 4 x 4 x
    4 blocks, the blocks in Z-order -- so every aligned run of 8 tiles is a 2 x 2
    x 2 region of blocks (row-major blocks: a strip along x)."""
    _, v = make_stress_building(777, 0, F=8, Y=16, X=16)
    v2, perm = blocked(v, (4, 4, 4), blocks="morton")
    n = v.num_nodes
    assert sorted(perm.tolist()) == list(range(n))
    bl = []
    for g in range(n // 64):
        loc = v2.location[64 * g:64 * g + 64]
        for c in range(3):
            assert int(loc[:, c].max() - loc[:, c].min()) == 3 and int(loc[:, c].min()) % 4 == 0
        bl.append(tuple(int(t) // 4 for t in loc.min(0).values))
    for r in range(0, len(bl), 8):
        run = bl[r:r + 8]
        for c in range(3):
            assert max(b[c] for b in run) - min(b[c] for b in run) == 1
    with pytest.raises(ValueError):
        block_order(v.location, (4, 4, 4), blocks="hilbert")


def test_block_order_ragged_edges():
    loc = torch.tensor([[0, 0, 5], [0, 0, 0], [5, 0, 0], [0, 4, 0], [1, 1, 1]])
    # blocks (f//4, y//4, x//4): (0,0,1) (0,0,0) (1,0,0) (0,1,0) (0,0,0); ny = 2, nx = 2
    assert block_order(loc, (4, 4, 4)).tolist() == [1, 4, 0, 3, 2]


def test_renumber_refuses_unknown_attributes():
    _, v = make_building(777, 3)
    n = v.num_nodes
    perm = torch.randperm(n)
    attrs = {k: getattr(v, k) for k in v.keys()}
    # an edge-level attribute whose length happens to equal the node count
    bad = GraphData(**attrs, edge_weight=torch.zeros(n))
    with pytest.raises(ValueError, match="edge_weight"):
        renumber(bad, perm)
    v2 = renumber(v, perm)
    assert v2.data_number == [v.data_number[int(i)] for i in perm]


def test_renumber_converted_building_permutes_node_ratio():
    """A building converted from the reference's JSON (vgan.convert, pinned by
    tests/golden/convert_small.pt): every per-node attribute -- node_ratio
    [N, 1] included -- follows the permutation."""
    import json
    import os

    from vgan import convert
    from vgan.config import Configuration

    fx = torch.load(os.path.join(os.path.dirname(__file__), "golden", "convert_small.pt"), weights_only=True)
    b = fx["buildings"][0]
    lo, vo = convert.process_building(json.loads(b["global_json"]), json.loads(b["local_json"]),
                                      json.loads(b["voxel_json"]), Configuration(), b["data_number"])
    _, v = convert.to_graph_pair(lo, vo)  # every attribute the store keeps
    n = v.num_nodes
    assert v.node_ratio.shape == (n, 1) and v.node_ratio.unique().numel() > 1
    v2, perm = tiled(v, 4)
    assert torch.equal(v2.node_ratio, v.node_ratio[perm])
    assert torch.equal(v2.type, v.type[perm]) and torch.equal(v2.location, v.location[perm])
    v3, perm3 = blocked(v, (4, 4, 4))
    assert torch.equal(v3.node_ratio, v.node_ratio[perm3])


@pytest.mark.gpu
def test_aggregation_on_renumbered_graph_is_permuted_bitwise(cuda):
    from vgan import ops
    from vgan._lib import ptr

    _, v = make_stress_building(777, 2, F=4, Y=20, X=20)
    v2, perm = tiled(v, 4)
    torch.manual_seed(1)
    n, C = v.num_nodes, 64
    h = torch.randn(n, C, device=cuda)
    a_s, a_d = 0.5 * torch.randn(n, device=cuda), 0.5 * torch.randn(n, device=cuda)
    b = torch.randn(C, device=cuda)
    outs = []
    for ei, p in ((v.edge_index, None), (v2.edge_index, perm.to(cuda))):
        csr = ops.CSR(ei.to(cuda), n)
        hh, ss, dd = (h, a_s, a_d) if p is None else (h[p].contiguous(), a_s[p].contiguous(), a_d[p].contiguous())
        out, alpha = torch.empty_like(h), torch.empty(csr.num_edges, device=cuda)
        ops.aggregate_fwd_raw(csr, C, ptr(hh), ptr(ss), ptr(dd), ptr(b), 0.2, ptr(out), ptr(alpha), csr.stream())
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[1], outs[0][perm.to(cuda)])
