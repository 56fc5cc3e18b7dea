"""Synthetic buildings reproduce the reference's processed-tensor layout and the
dataset invariants the reference checks (analyze.py:76-79,85; data.py:253-254)."""
import numpy as np
import pytest
import torch

from vgan import synth
from vgan.graph import GraphBatch


@pytest.mark.parametrize("number", [0, 1, 7, 4001])
def test_building_layout_and_far_invariant(number):
    local, voxel = synth.make_building(777, number)
    n = voxel.num_nodes
    assert voxel.x.shape == (n, 12) and voxel.x.dtype == torch.float32
    assert local.x.shape[1] == 17
    assert voxel.types_onehot.dtype == torch.int64 and voxel.type.dtype == torch.int64
    assert torch.equal(voxel.types_onehot.argmax(1), voxel.type)
    assert 180 <= n <= 810
    # FAR invariant: far == sum_{non-void} dim_y * dim_x / site_area (analyze.py:76-79)
    dims = voxel.dimension.double()
    nonvoid = voxel.type != 6
    gfa = (dims[nonvoid, 1] * dims[nonvoid, 2]).sum().item()
    assert np.isclose(voxel.x[0, 9].item(), gfa / voxel.site_area[0].item(), rtol=1e-6)
    assert 324 <= voxel.site_area[0].item() <= 1600
    # normalised features (data.py:298-304): coord/42, dim/11, loc/11, floor/10, site/1600
    assert torch.allclose(voxel.x[:, 3:6] * 11, voxel.dimension, atol=1e-4)
    assert torch.allclose(voxel.x[:, 10] * 10, voxel.voxel_level.float(), atol=1e-5)
    # program nodes only carry types 0..5; their one-hot block + ratio block
    assert int(local.type.max()) <= 5
    assert torch.equal(local.x[:, :7].argmax(1), local.type)


def test_edge_index_is_sorted_symmetric_loop_free():
    _, voxel = synth.make_building(777, 3)
    ei = voxel.edge_index.numpy()
    key = ei[0] * voxel.num_nodes + ei[1]
    assert (np.diff(key) > 0).all()  # adjacency.nonzero() order, no duplicates
    assert (ei[0] != ei[1]).all()
    fwd = set(map(tuple, ei.T))
    assert all((b, a) in fwd for a, b in fwd)
    deg = np.bincount(ei[1], minlength=voxel.num_nodes)
    assert deg.max() <= 6 and deg.min() >= 3


def test_type_distribution_close_to_dataset():
    counts = np.zeros(7)
    for i in range(40):
        _, v = synth.make_building(777, i)
        counts += np.bincount(v.type.numpy(), minlength=7)
    ratio = counts / counts.sum()
    assert np.allclose(ratio, synth.TYPE_RATIOS, atol=0.02)


def test_collate_offsets_and_slicing():
    items = [synth.make_building(777, i) for i in range(3)]
    loc, vox = GraphBatch.from_data_list([l for l, _ in items]), GraphBatch.from_data_list([v for _, v in items])
    sizes = [v.num_nodes for _, v in items]
    assert vox.num_graphs == 3 and vox.num_nodes == sum(sizes)
    assert vox.ptr.tolist() == [0, sizes[0], sizes[0] + sizes[1], sum(sizes)]
    g1 = vox[1]
    assert torch.equal(g1.x, items[1][1].x)
    assert torch.equal(g1.edge_index, items[1][1].edge_index)
    assert vox.data_number[2][0] == "2"


def test_stress_building_degree():
    _, v = synth.make_stress_building(777, 0, F=4, Y=10, X=10)
    deg = np.bincount(v.edge_index[1].numpy(), minlength=v.num_nodes)
    assert deg.max() == 22  # 4 in-floor + 9 up + 9 down
