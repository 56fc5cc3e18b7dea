"""Voxel numbering for gather locality (configs[3], the scatter kernel's stress graph).

The aggregation gathers every edge's source row.  The reference numbers a
building's voxels floor-major, then row-major (y, x) inside a floor
(``data.py:300-335``, ``adjacency.nonzero()``), so the 16 destination rows one
workgroup aggregates are a 16-voxel strip of one lattice row: on the stress
lattice (4-neighbour floors plus 3x3 blocks to the floors above and below)
such a strip gathers ~150 distinct source rows for ~345 edges.  Numbering each
floor in T x T tiles of (y, x) makes the 16 rows a 4 x 4 patch, whose sources
are the patch, its 4-neighbour ring and the 6 x 6 blocks above and below:
~104 distinct rows for the same edges, more reuse per workgroup out of L1/L2.

Renumbering is a permutation of the nodes inside each building: node-level
tensors are gathered, ``edge_index`` is relabelled IN PLACE of every edge (the
edge order, hence every destination row's source order and its softmax /
gather-sum order, is the reference's), per-building blocks stay contiguous
(``ptr``, ``batch``), and every per-node result maps back with the inverse
permutation.  The model is permutation-equivariant up to the f32 summation
order of GraphNorm's column statistics.
"""
from __future__ import annotations

from typing import Tuple

import torch

from .graph import GraphData


def tile_order(location: torch.Tensor, tile: int = 4) -> torch.Tensor:
    """perm [n] (new row r = old row perm[r]) numbering voxels floor by floor in
    ``tile`` x ``tile`` (y, x) tiles, row-major inside a tile; ``location`` is
    the voxels' integer (floor, y, x) [n, 3] (the reference's voxel
    ``location``, ``data.py:62``)."""
    loc = location.to(torch.int64)
    f, y, x = loc[:, 0], loc[:, 1], loc[:, 2]
    span = int(max(int(y.max()), int(x.max())) + 1) if loc.numel() else 1
    tiles = (span + tile - 1) // tile
    key = (((f * tiles + y // tile) * tiles + x // tile) * tile + y % tile) * tile + x % tile
    return torch.argsort(key, stable=True)


# node-level attributes of a voxel building (VoxelGraphData, data.py:48-77 and
# the keys vgan.synth / vgan.convert add): gathered by the permutation.
# node_ratio is per node on a voxel graph ([N, 1]: the building's ratio of
# each voxel's type, data.py:76-77,144; vgan/convert.py:165,184).
NODE_KEYS = ("x", "type", "types_onehot", "voxel_level", "coordinate", "dimension", "location", "site_area",
             "data_number", "node_ratio")
# per-building attributes: carried unchanged (none on a voxel graph today)
GRAPH_KEYS: tuple = ()


def renumber(voxel: GraphData, perm: torch.Tensor) -> GraphData:
    """The building with node ``perm[r]`` as node r: the node-level attributes
    (``NODE_KEYS``) gathered, edges relabelled in place (same order).  Any
    other key is refused rather than guessed from its shape (an edge-level
    attribute whose length happens to equal the node count would otherwise be
    permuted as if it were per node)."""
    n = voxel.num_nodes
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(n, dtype=perm.dtype)
    out = {}
    for key in voxel.keys():
        v = getattr(voxel, key)
        if key == "edge_index":
            out[key] = inv[v]
        elif key in NODE_KEYS:
            if len(v) != n:
                raise ValueError(f"node attribute {key!r} has {len(v)} rows for {n} nodes")
            out[key] = v[perm] if torch.is_tensor(v) else [v[int(i)] for i in perm]
        elif key in GRAPH_KEYS:
            out[key] = v
        else:
            raise ValueError(f"renumber: unknown voxel attribute {key!r} (add it to NODE_KEYS or GRAPH_KEYS)")
    return GraphData(**out)


def _morton3(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, bits: int) -> torch.Tensor:
    """Interleaved bits (a, b, c), a's the most significant of each triple."""
    key = torch.zeros_like(a)
    for i in range(bits - 1, -1, -1):
        key = (key << 3) | (((a >> i) & 1) << 2) | (((b >> i) & 1) << 1) | ((c >> i) & 1)
    return key


def block_order(location: torch.Tensor, block=(4, 4, 4), blocks: str = "rowmajor") -> torch.Tensor:
    """perm [n] numbering voxels in (floor, y, x) blocks of ``block`` = (bf, by,
    bx), row-major inside a block.  A 64-row aggregation tile is then a 4 x 4 x 4
    block of the lattice: on the stress lattice its sources are the block grown
    by one voxel in y and x on each of its floors and on the floors just above
    and below -- about 6 x 6 x 6 = 216 distinct rows for ~1,400 edges (6.4
    edges per distinct source row, against 3.1 for the 4 x 4 floor tiles of
    ``tile_order``).

    ``blocks`` orders the blocks themselves: "rowmajor" (floor, y, x), or
    "morton" (Z-order of the block coordinates), under which any run of
    consecutive tiles -- what one XCD's workgroups aggregate at a time -- is a
    compact 3-D region, so a tile's halo rows on the floors above and below
    are those its neighbours in the run stage too (row-major blocks put the
    vertical neighbour a whole block layer, ~170 tiles, later)."""
    loc = location.to(torch.int64)
    bf, by, bx = (int(b) for b in block)
    f, y, x = loc[:, 0], loc[:, 1], loc[:, 2]
    ny = int(y.max()) // by + 1 if loc.numel() else 1
    nx = int(x.max()) // bx + 1 if loc.numel() else 1
    inner = ((f % bf) * by + y % by) * bx + x % bx
    if blocks == "morton":
        nf = int(f.max()) // bf + 1 if loc.numel() else 1
        bits = max(1, max(nf, ny, nx) - 1).bit_length()
        outer = _morton3(f // bf, y // by, x // bx, bits)
    elif blocks == "rowmajor":
        outer = ((f // bf) * ny + y // by) * nx + x // bx
    else:
        raise ValueError(f"block_order: blocks must be 'rowmajor' or 'morton', not {blocks!r}")
    return torch.argsort(outer * (bf * by * bx) + inner, stable=True)


def tiled(voxel: GraphData, tile: int = 4) -> Tuple[GraphData, torch.Tensor]:
    """(renumbered building, perm) in ``tile_order`` of its ``location``."""
    perm = tile_order(voxel.location, tile)
    return renumber(voxel, perm), perm


def blocked(voxel: GraphData, block=(4, 4, 4), blocks: str = "rowmajor") -> Tuple[GraphData, torch.Tensor]:
    """(renumbered building, perm) in ``block_order`` of its ``location``."""
    perm = block_order(voxel.location, block, blocks)
    return renumber(voxel, perm), perm
