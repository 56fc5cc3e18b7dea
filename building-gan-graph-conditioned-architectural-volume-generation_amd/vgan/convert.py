"""Raw-JSON building converter -> GraphStore (the reference's ``DataCreator``).

The reference turns three JSON files per building (global / local / voxel
graph, ``data.py:423-461``) into two pickled objects (``DataCreatorHelper.
process_data``, ``data.py:216-407``; ``LocalGraphData`` / ``VoxelGraphData``,
``data.py:16-77``) and later wraps them into PyG ``Data`` (``data.py:117-147``).
This module produces the same tensors and writes them into a tensor-only
``GraphStore`` instead of pickles:

* ``process_building`` returns the attribute dictionaries of ``LocalGraphData``
  / ``VoxelGraphData`` (same names, values, dtypes and shapes; pinned against
  the reference itself by ``tests/golden/convert_small.pt``);
* ``to_graph_pair`` applies the ``Data(...)`` field mapping of
  ``data.py:117-147``;
* ``convert_directories`` walks the three JSON directories in the reference's
  order and writes the store.

Arithmetic mirrors the reference's dtype flow: per-voxel features are divided
in Python double precision and then stored as float32 (``torch.tensor`` of a
float list), integer tensors divided by an ``int`` normalisation factor become
float32 quotients, and JSON ints stay int64.
"""
from __future__ import annotations

import json
import os
import re
from typing import Dict, Iterator, List, Sequence, Tuple

import torch

from .graph import GraphData
from .store import GraphStore


def _adjacency_edges(num: int, pairs: Sequence[Tuple[int, int]]) -> torch.Tensor:
    """[2, E] int64 of the distinct (row, col) pairs in row-major order: the
    result of ``adjacency.nonzero().t()`` on a dense 0/1 matrix (data.py:266-273,355-364)."""
    flat = sorted({u * num + v for u, v in pairs})
    if not flat:
        return torch.zeros(2, 0, dtype=torch.int64)
    t = torch.tensor(flat, dtype=torch.int64)
    return torch.stack([t // num, t % num])


def process_building(global_graph: dict, local_graph: dict, voxel_graph: dict, cfg,
                     data_number: str) -> Tuple[Dict[str, object], Dict[str, object]]:
    """Attribute dicts of ``LocalGraphData`` / ``VoxelGraphData`` for one building."""
    k = cfg.NUM_CLASSES
    # ---- program (local) graph: nodes keyed by (floor, type, type_id)
    nodes = local_graph["node"]
    key_of = {}
    for i, node in enumerate(nodes):
        key_of[(node["floor"], node["type"], node["type_id"])] = i
    floors = torch.tensor([node["floor"] for node in nodes])
    types = torch.tensor([node["type"] for node in nodes])
    onehot = torch.nn.functional.one_hot(types.clone(), num_classes=k)
    local_pairs = [(key_of[(n["floor"], n["type"], n["type_id"])], key_of[tuple(nb)])
                   for n in nodes for nb in n["neighbors"]]
    local_edges = _adjacency_edges(len(nodes), local_pairs)

    far = torch.tensor([global_graph["far"]])
    site_area = torch.tensor([global_graph["site_area"]])
    site_area_normalized = site_area / cfg.NORMALIZATION_FACTOR_SITE
    ratio = [0] * k
    for gnode in global_graph["global_node"]:
        ratio[gnode["type"]] = gnode["proportion"]
    type_ratio = torch.tensor(ratio)

    # ---- voxel graph: nodes keyed by location (floor, y, x)
    vnodes = voxel_graph["voxel_node"]
    vkey = {}
    feats: List[List[float]] = []
    vtypes: List[int] = []
    counts = [0] * k
    for i, vn in enumerate(vnodes):
        vkey[tuple(vn["location"])] = i
        feats.append([c / cfg.NORMALIZATION_FACTOR_COORDINATE for c in vn["coordinate"]]
                     + [d / cfg.NORMALIZATION_FACTOR_DIMENSION for d in vn["dimension"]]
                     + [l / cfg.NORMALIZATION_FACTOR_LOCATION for l in vn["location"]])
        t = cfg.VOID if vn["type"] == cfg.VOID_OLD else vn["type"]
        counts[t] += 1
        vtypes.append(t)
    voxel_pairs = [(vkey[tuple(vn["location"])], vkey[tuple(nb)]) for vn in vnodes for nb in vn["neighbors"]]
    vfloors = torch.tensor([vn["location"][0] for vn in vnodes])
    vtypes_t = torch.tensor(vtypes)

    local_rec = {
        "far": far,
        "site_area": site_area,
        "site_area_normalized": site_area_normalized,
        "type_ratio": type_ratio,
        "local_graph_node_cluster": types.clone(),
        "local_graph_types_onehot": onehot,
        "local_graph_floor_levels": floors,
        "local_graph_floor_levels_normalized": floors / cfg.NORMALIZATION_FACTOR_FLOOR_LEVEL,
        "local_graph_edge_indices": local_edges,
        "local_graph_center": torch.tensor([node["center"] for node in nodes]),
        "local_graph_types": types.clone(),
        "local_graph_type_ids": torch.tensor([node["type_id"] for node in nodes]),
        "data_number": data_number,
    }
    voxel_rec = {
        "far": far,
        "site_area": site_area,
        "site_area_normalized": site_area_normalized,
        "voxel_graph_types": vtypes_t,
        "voxel_graph_types_onehot": torch.nn.functional.one_hot(vtypes_t.clone(), num_classes=k),
        "voxel_graph_floor_levels": vfloors,
        "voxel_graph_floor_levels_normalized": vfloors / cfg.NORMALIZATION_FACTOR_FLOOR_LEVEL,
        "voxel_graph_features": torch.tensor(feats),
        "voxel_graph_edge_indices": _adjacency_edges(len(vnodes), voxel_pairs),
        "voxel_graph_node_coordinate": torch.tensor([vn["coordinate"] for vn in vnodes]),
        "voxel_graph_node_dimension": torch.tensor([vn["dimension"] for vn in vnodes]),
        "voxel_graph_location": torch.tensor([vn["location"] for vn in vnodes]),
        "voxel_graph_node_ratio": torch.tensor(counts) / len(vnodes),
        "data_number": data_number,
    }
    return _local_object(local_rec), _voxel_object(voxel_rec)


def _local_object(rec: Dict[str, object]) -> Dict[str, object]:
    """LocalGraphData.__init__ (data.py:16-45): the model-facing attributes."""
    onehot = rec["local_graph_types_onehot"]
    m = onehot.shape[0]
    ratio_per_node = onehot * rec["type_ratio"]
    x = torch.cat([onehot, ratio_per_node, torch.zeros(m, 1) + rec["far"],
                   rec["local_graph_floor_levels_normalized"].reshape(m, 1),
                   rec["site_area_normalized"].repeat(m).reshape(m, 1)], dim=1)
    return {
        "x": x,
        "data_number": rec["data_number"],
        "site_area": rec["site_area"],
        "site_area_normalized": rec["site_area_normalized"],
        "local_graph_types_onehot": onehot,
        "edge_index": rec["local_graph_edge_indices"],
        "local_graph_floor_levels": rec["local_graph_floor_levels"],
        "local_graph_type_ratio_per_node": ratio_per_node,
        "local_graph_node_cluster": rec["local_graph_node_cluster"],
        "local_graph_center": rec["local_graph_center"],
        "local_graph_types": rec["local_graph_types"],
        "local_graph_type_ids": rec["local_graph_type_ids"],
    }


def _voxel_object(rec: Dict[str, object]) -> Dict[str, object]:
    """VoxelGraphData.__init__ (data.py:48-77)."""
    onehot = rec["voxel_graph_types_onehot"]
    n = onehot.shape[0]
    x = torch.cat([rec["voxel_graph_features"], torch.zeros(n, 1) + rec["far"],
                   rec["voxel_graph_floor_levels_normalized"].reshape(n, 1),
                   rec["site_area_normalized"].repeat(n).reshape(n, 1)], dim=1)
    return {
        "x": x,
        "data_number": rec["data_number"],
        "site_area": rec["site_area"],
        "site_area_normalized": rec["site_area_normalized"],
        "voxel_graph_types": rec["voxel_graph_types"],
        "voxel_graph_types_onehot": onehot,
        "edge_index": rec["voxel_graph_edge_indices"],
        "voxel_graph_floor_levels": rec["voxel_graph_floor_levels"],
        "voxel_graph_node_coordinate": rec["voxel_graph_node_coordinate"],
        "voxel_graph_node_dimension": rec["voxel_graph_node_dimension"],
        "voxel_graph_location": rec["voxel_graph_location"],
        "voxel_graph_node_ratio": (onehot * rec["voxel_graph_node_ratio"]).max(dim=1)[0].unsqueeze(1),
    }


def to_graph_pair(local: Dict[str, object], voxel: Dict[str, object]) -> Tuple[GraphData, GraphData]:
    """The ``Data(...)`` wrapping of GraphDataset.__init__ (data.py:117-147)."""
    m = local["x"].shape[0]
    n = voxel["x"].shape[0]
    lg = GraphData(
        x=local["x"], edge_index=local["edge_index"], node_cluster=local["local_graph_node_cluster"],
        node_ratio=local["local_graph_type_ratio_per_node"], types_onehot=local["local_graph_types_onehot"],
        center=local["local_graph_center"], type=local["local_graph_types"], type_id=local["local_graph_type_ids"],
        floor=local["local_graph_floor_levels"], data_number=[local["data_number"]] * m,
        site_area=local["site_area"].repeat(m),
    )
    vg = GraphData(
        x=voxel["x"], edge_index=voxel["edge_index"], voxel_level=voxel["voxel_graph_floor_levels"],
        type=voxel["voxel_graph_types"], types_onehot=voxel["voxel_graph_types_onehot"],
        coordinate=voxel["voxel_graph_node_coordinate"], dimension=voxel["voxel_graph_node_dimension"],
        location=voxel["voxel_graph_location"], node_ratio=voxel["voxel_graph_node_ratio"],
        data_number=[voxel["data_number"]] * n, site_area=voxel["site_area"].repeat(n),
    )
    return lg, vg


def _numbered(directory: str) -> List[str]:
    files = [os.path.join(directory, d) for d in os.listdir(directory)]
    return sorted(files, key=lambda p: int(os.path.basename(p).replace(".json", "").split("_")[-1]))


def iter_json_buildings(global_dir: str, local_dir: str, voxel_dir: str, cfg) -> Iterator[Tuple[GraphData, GraphData]]:
    """DataCreator.create's walk (data.py:414-453): the three directories sorted
    by the trailing number of each file name, matched by that number."""
    for gp, lp, vp in zip(_numbered(global_dir), _numbered(local_dir), _numbered(voxel_dir)):
        nums = [os.path.basename(p).replace(".json", "").split("_")[-1] for p in (gp, lp, vp)]
        if len(set(nums)) != 1:
            raise ValueError(f"unmatched building files {gp}, {lp}, {vp}")
        with open(gp) as f:
            g = json.load(f)
        with open(lp) as f:
            loc = json.load(f)
        with open(vp) as f:
            vox = json.load(f)
        data_number = "".join(re.findall(r"\d", os.path.basename(gp)))
        yield to_graph_pair(*process_building(g, loc, vox, cfg, data_number))


def convert_directories(global_dir: str, local_dir: str, voxel_dir: str, out_path: str, cfg) -> GraphStore:
    """Convert a raw-JSON dataset into a GraphStore at ``out_path``."""
    return GraphStore.write(out_path, iter_json_buildings(global_dir, local_dir, voxel_dir, cfg))
