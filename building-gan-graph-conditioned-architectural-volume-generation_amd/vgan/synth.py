"""Seeded synthetic buildings in the reference's processed-tensor layout.

The reference dataset (``building_gan/data/6types-raw_data-10000.zip``) is a
Git-LFS stub, so every workload here is generated.  Each building reproduces
the tensors ``DataCreatorHelper.process_data`` (``data.py:215-391``) and
``GraphDataset.__init__`` (``data.py:113-148``) would have produced:

voxel graph (``VoxelGraphData``, ``data.py:48-77``)
    x [n, 12] f32 = coordinate/42 (3) | dimension/11 (3) | location/11 (3) |
    far | floor/10 | site_area/1600;  type [n] i64 (0..6, VOID = 6);
    types_onehot [n, 7] i64;  edge_index [2, E] i64, lexicographically sorted
    like ``adjacency.nonzero().t()`` (``data.py:335``);  site_area [n] f32
    (raw area repeated per node, ``data.py:146``);  data_number (list).
local / program graph (``LocalGraphData``, ``data.py:16-45``)
    x [m, 17] f32 = onehot(type) (7) | onehot * type_ratio (7) | far |
    floor/10 | site_area/1600;  type [m] i64 (0..5);  edge_index [2, M] i64.

Sizes follow the survey calibration: floors U{4..10}, a
U{6..9} x U{6..9} footprint grid (mean ~394 voxels, dataset mean ~399 from
``analyze.py:100``), 6-neighbour voxel adjacency in both directions, voxel
types drawn from the ``analyze.py:100`` ratios, and a FAR that satisfies the
``analyze.py:76-79`` invariant ``far == sum_{non-void} dim_y*dim_x / site``.

``make_stress_building`` is the config-#4 graph: a 20 x 50 x 50 lattice with
4-neighbour floors plus 3x3 blocks to the floors above and below (degree ~20.6).
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import numpy as np
import torch

from .graph import GraphBatch, GraphData

NUM_CLASSES = 7
VOID = 6
# analyze.py:100 -- VOID(-1 -> 6) 0.3365, then types 0..5
TYPE_RATIOS = np.array([0.13101, 0.06349, 0.02747, 0.04949, 0.38088, 0.01116, 0.3365])
TYPE_RATIOS = TYPE_RATIOS / TYPE_RATIOS.sum()

_NORM_COORD, _NORM_DIM, _NORM_LOC, _NORM_FLOOR, _NORM_SITE = 42.0, 11.0, 11.0, 10.0, 1600.0

_SIX = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]
_STRESS = [(0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)] + [
    (df, dj, di) for df in (-1, 1) for dj in (-1, 0, 1) for di in (-1, 0, 1)
]


def lattice_edges(F: int, Y: int, X: int, offsets: Sequence[Tuple[int, int, int]]) -> np.ndarray:
    """Directed lattice adjacency, sorted by (src, dst) like ``adjacency.nonzero()``."""
    f, j, i = np.meshgrid(np.arange(F), np.arange(Y), np.arange(X), indexing="ij")
    f, j, i = f.ravel(), j.ravel(), i.ravel()
    src_all, dst_all = [], []
    for df, dj, di in offsets:
        nf, nj, ni = f + df, j + dj, i + di
        ok = (nf >= 0) & (nf < F) & (nj >= 0) & (nj < Y) & (ni >= 0) & (ni < X)
        src_all.append(((f * Y + j) * X + i)[ok])
        dst_all.append(((nf * Y + nj) * X + ni)[ok])
    src = np.concatenate(src_all)
    dst = np.concatenate(dst_all)
    order = np.lexsort((dst, src))
    return np.stack([src[order], dst[order]]).astype(np.int64)


def _building(rng: np.random.Generator, number: int, F: int, Y: int, X: int,
              offsets, dim_lo: float, dim_hi: float) -> Tuple[GraphData, GraphData]:
    n = F * Y * X
    zdim = rng.uniform(3.0, 4.5, size=F)
    ydim = rng.uniform(dim_lo, dim_hi, size=Y)
    xdim = rng.uniform(dim_lo, dim_hi, size=X)
    zc = np.concatenate([[0.0], np.cumsum(zdim)[:-1]])
    yc = np.concatenate([[0.0], np.cumsum(ydim)[:-1]])
    xc = np.concatenate([[0.0], np.cumsum(xdim)[:-1]])
    f, j, i = np.meshgrid(np.arange(F), np.arange(Y), np.arange(X), indexing="ij")
    f, j, i = f.ravel(), j.ravel(), i.ravel()
    coord = np.stack([zc[f], yc[j], xc[i]], 1)
    dims = np.stack([zdim[f], ydim[j], xdim[i]], 1)
    loc = np.stack([f, j, i], 1).astype(np.float64)
    vtype = rng.choice(NUM_CLASSES, size=n, p=TYPE_RATIOS).astype(np.int64)

    footprint = float(ydim.sum() * xdim.sum())
    site_area = float(np.clip(round(footprint * rng.uniform(1.05, 1.6)), 324, 1600))
    nonvoid = vtype != VOID
    gfa = float((dims[nonvoid, 1] * dims[nonvoid, 2]).sum())
    far = gfa / site_area

    ratio = np.bincount(vtype, minlength=NUM_CLASSES) / n
    vx = np.concatenate(
        [
            coord / _NORM_COORD,
            dims / _NORM_DIM,
            loc / _NORM_LOC,
            np.full((n, 1), far),
            f[:, None] / _NORM_FLOOR,
            np.full((n, 1), site_area / _NORM_SITE),
        ],
        1,
    )
    onehot = np.eye(NUM_CLASSES, dtype=np.int64)[vtype]
    vei = lattice_edges(F, Y, X, offsets)
    tag = str(number)
    voxel = GraphData(
        x=torch.tensor(vx, dtype=torch.float32),
        edge_index=torch.from_numpy(vei),
        type=torch.from_numpy(vtype),
        types_onehot=torch.from_numpy(onehot),
        voxel_level=torch.from_numpy(f.astype(np.int64)),
        coordinate=torch.tensor(coord, dtype=torch.float32),
        dimension=torch.tensor(dims, dtype=torch.float32),
        location=torch.from_numpy(loc.astype(np.int64)),
        site_area=torch.full((n,), site_area, dtype=torch.float32),
        data_number=[tag] * n,
    )

    # program graph: per floor, nodes for the non-void types present on it
    l_floor: List[int] = []
    l_type: List[int] = []
    l_id: List[int] = []
    for fl in range(F):
        on_floor = vtype[f == fl]
        present = [t for t in range(NUM_CLASSES - 1) if (on_floor == t).any()]
        budget = int(rng.integers(2, 15))
        counts = {t: 1 for t in present}
        extra = max(0, budget - len(present))
        for _ in range(extra):
            if not present:
                break
            counts[present[int(rng.integers(len(present)))]] += 1
        if not present:  # keep every floor represented
            counts = {4: 1}
        for t, c in sorted(counts.items()):
            for k in range(c):
                l_floor.append(fl)
                l_type.append(t)
                l_id.append(k)
    m = len(l_type)
    lt = np.array(l_type, dtype=np.int64)
    lf = np.array(l_floor, dtype=np.int64)
    lonehot = np.eye(NUM_CLASSES, dtype=np.float64)[lt]
    lx = np.concatenate(
        [
            lonehot,
            lonehot * ratio[None, :],
            np.full((m, 1), far),
            lf[:, None] / _NORM_FLOOR,
            np.full((m, 1), site_area / _NORM_SITE),
        ],
        1,
    )
    # same-floor chain + same-type link to the next floor; pairs (a, b) in
    # lexicographic order (the nonzeros of the m x m relation, row-major)
    ida = np.array(l_id, dtype=np.int64)
    idx = np.arange(m)
    chain = (lf[:, None] == lf[None, :]) & (np.abs(idx[:, None] - idx[None, :]) == 1)
    link = (np.abs(lf[:, None] - lf[None, :]) == 1) & (lt[:, None] == lt[None, :]) & (ida[:, None] == ida[None, :])
    rel = (chain | link) & (idx[:, None] != idx[None, :])
    lei = np.stack(np.nonzero(rel)).astype(np.int64).reshape(2, -1)
    local = GraphData(
        x=torch.tensor(lx, dtype=torch.float32),
        edge_index=torch.from_numpy(np.ascontiguousarray(lei)),
        type=torch.from_numpy(lt),
        type_id=torch.tensor(l_id, dtype=torch.int64),
        floor=torch.from_numpy(lf),
        types_onehot=torch.from_numpy(lonehot.astype(np.int64)),
        site_area=torch.full((m,), site_area, dtype=torch.float32),
        data_number=[tag] * m,
    )
    return local, voxel


def make_building(seed: int, number: int) -> Tuple[GraphData, GraphData]:
    """One dataset-like building; deterministic in (seed, number)."""
    rng = np.random.default_rng([seed, number])
    F = int(rng.integers(4, 11))
    Y = int(rng.integers(6, 10))
    X = int(rng.integers(6, 10))
    return _building(rng, number, F, Y, X, _SIX, 3.0, 4.6)


def make_stress_building(seed: int, number: int, F: int = 20, Y: int = 50, X: int = 50):
    """Config #4: ~50k voxels, 4-neighbour floors + 3x3 inter-floor blocks."""
    rng = np.random.default_rng([seed, number, 4])
    return _building(rng, number, F, Y, X, _STRESS, 3.0, 4.6)


class SyntheticDataset:
    """Indexable dataset of synthetic buildings (drop-in for ``GraphDataset``).

    ``dataset[i] -> (local GraphData, voxel GraphData)`` and
    ``SyntheticDataset.collate_fn`` mirror ``data.py:150-163``.
    """

    def __init__(self, size: int, seed: int = 777, stress: bool = False):
        self.size = int(size)
        self.seed = int(seed)
        self.stress = stress
        self._cache = {}

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, i: int):
        i = int(i)
        if i not in self._cache:
            maker = make_stress_building if self.stress else make_building
            self._cache[i] = maker(self.seed, i)
        return self._cache[i]

    @staticmethod
    def collate_fn(items):
        locals_, voxels = zip(*items)
        return GraphBatch.from_data_list(locals_), GraphBatch.from_data_list(voxels)

    def batch(self, indices: Sequence[int]):
        return self.collate_fn([self[i] for i in indices])


def write_synthetic_store(path: str, size: int, seed: int = 777) -> None:
    """A GraphStore of ``size`` synthetic buildings (vgan.store.write_store over
    SyntheticDataset(size, seed)); the bench runs it in a child process while
    the GPU legs run: one intra-op thread at a lowered priority, so that it
    takes no more than a core from the host-bound legs it runs beside."""
    from .store import write_store

    torch.set_num_threads(1)
    try:
        os.nice(10)
    except OSError:
        pass
    write_store(path, SyntheticDataset(size, seed=seed))
