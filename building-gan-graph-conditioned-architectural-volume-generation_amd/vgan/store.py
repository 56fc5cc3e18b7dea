"""Tensor-only building store + native batch collate (the path's data loader).

Replaces the reference's data path up to the model inputs:

* ``GraphDataset`` (``data.py:80-150``): one pickled ``LocalGraphData`` /
  ``VoxelGraphData`` object per building, ``torch.load``-ed and wrapped into
  PyG ``Data`` (``data.py:116-147``).  Those pickles need the reference's
  classes and ``weights_only=False`` (refused by torch >= 2.6 defaults), so the
  store keeps plain arrays instead: every node-level attribute of all buildings
  concatenated into one ``.npy`` per key (memory-mapped, ``allow_pickle=False``),
  edges as building-local int32 ``esrc`` / ``edst``, and ``node_ptr`` /
  ``edge_ptr`` offsets per building (the layout of PyG's InMemoryDataset slices).
* ``GraphDataset.collate_fn`` (``data.py:156-163``, two
  ``Batch.from_data_list``): ``GraphStore.collate`` gathers the selected
  buildings with the host C++ library (``csrc/collate.cpp``, ``libvgan_host.so``,
  ``include/vgan_host.h``) into (optionally pinned) buffers and also emits the
  voxel graph's int32 CSR + self loops and CSC, which ``vgan.data`` uploads
  instead of rebuilding them on the device (no host sync per batch).

The collated batch is identical, key for key and bit for bit, to
``GraphBatch.from_data_list`` over ``store[i]`` (tests/test_store_cpu.py).
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .graph import GraphBatch, GraphData

HOST_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvgan_host.so")
FORMAT = "vgan-graphstore"
VERSION = 1
KINDS = ("local", "voxel")
CSR_KINDS = ("voxel",)  # graphs whose GATConv index structures the collate emits

_p, _i32, _i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64

# name -> (restype, argtypes); every function listed here is declared in include/vgan_host.h
HOST_SIGNATURES = {
    "vgh_collate_sizes": (ctypes.c_int, [_p, _p, _p, _p, _i64, _p, _i32, _p]),
    "vgh_collate_rows": (ctypes.c_int, [_p, _i64, _p, _i64, _p, _i32, _p, _i32]),
    "vgh_collate_graph": (ctypes.c_int, [_p, _p, _p, _p, _i64, _p, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p]),
}
_HOST_ERRORS = {1: "invalid argument", 2: "building index out of range", 3: "edge endpoint outside its building",
                4: "batch too large for int32 ids"}

_HOST = None


def host_lib() -> ctypes.CDLL:
    """libvgan_host.so (built by ``make -C .../csrc``); raises if it is missing."""
    global _HOST
    if _HOST is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise RuntimeError(f"{HOST_LIB_PATH} is not built (run __graft_entry__.build())")
        lib = ctypes.CDLL(HOST_LIB_PATH)
        for name, (res, args) in HOST_SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _HOST = lib
    return _HOST


def _host_check(rc: int, name: str) -> None:
    if rc != 0:
        raise ValueError(f"{name}: {_HOST_ERRORS.get(rc, f'error {rc}')}")


def _np_ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def _t_ptr(t: Optional[torch.Tensor]) -> Optional[ctypes.c_void_p]:
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_NP_TO_TORCH = {np.dtype(k): v for k, v in ((np.float32, torch.float32), (np.float64, torch.float64),
                                            (np.int64, torch.int64), (np.int32, torch.int32),
                                            (np.uint8, torch.uint8), (np.bool_, torch.bool))}


class GraphStore:
    """A directory of per-key arrays for ``len(store)`` buildings.

    ``store[i]`` returns the building as a ``(local, voxel)`` ``GraphData``
    pair (the reference's ``GraphDataset.__getitem__``, ``data.py:150-151``);
    ``store.collate(indices)`` builds the mini-batch pair natively.
    """

    def __init__(self, path: str, mmap: bool = True):
        self.path = path
        with open(os.path.join(path, "meta.json")) as f:
            meta = json.load(f)
        if meta.get("format") != FORMAT or meta.get("version") != VERSION:
            raise ValueError(f"{path} is not a {FORMAT} v{VERSION} store")
        self.meta = meta
        self.num_buildings = int(meta["num_buildings"])
        mode = "r" if mmap else None
        self._arr: Dict[str, Dict[str, np.ndarray]] = {}
        for kind in KINDS:
            g = meta["graphs"][kind]
            arrs = {name: np.load(os.path.join(path, f"{kind}.{name}.npy"), mmap_mode=mode, allow_pickle=False)
                    for name in ("node_ptr", "edge_ptr", "esrc", "edst")}
            for key in g["node_keys"]:
                arrs[key] = np.load(os.path.join(path, f"{kind}.{key}.npy"), mmap_mode=mode, allow_pickle=False)
            for name in ("node_ptr", "edge_ptr"):
                if arrs[name].shape != (self.num_buildings + 1,):
                    raise ValueError(f"{kind}.{name} has shape {arrs[name].shape}")
            self._arr[kind] = arrs

    # ------------------------------------------------------------------ write
    @staticmethod
    def write(path: str, items: Iterable[Tuple[GraphData, GraphData]]) -> "GraphStore":
        """Write (local, voxel) building pairs as a store.  Node-level tensor
        attributes keep their dtype and trailing shape; ``edge_index`` becomes
        building-local int32 endpoints; list attributes (``data_number``) must
        hold one value per building, as ``data.py:145,160`` builds them."""
        os.makedirs(path, exist_ok=True)
        cols: Dict[str, Dict[str, List[np.ndarray]]] = {k: {} for k in KINDS}
        lists: Dict[str, Dict[str, List]] = {k: {} for k in KINDS}
        order: Dict[str, List[str]] = {}
        counts: Dict[str, List[Tuple[int, int]]] = {k: [] for k in KINDS}
        n_items = 0
        for pair in items:
            for kind, g in zip(KINDS, pair):
                keys = g.keys()
                if kind not in order:
                    order[kind] = list(keys)
                elif list(keys) != order[kind]:
                    raise ValueError(f"building {n_items}: {kind} keys {keys} differ from {order[kind]}")
                n = g.num_nodes
                for key in keys:
                    v = getattr(g, key)
                    if key == "edge_index":
                        ei = v.detach().cpu().numpy()
                        if ei.ndim != 2 or ei.shape[0] != 2:
                            raise ValueError("edge_index must be [2, E]")
                        if ei.size and (ei.min() < 0 or ei.max() >= n):
                            raise ValueError(f"building {n_items}: {kind} edge_index outside [0, {n})")
                        cols[kind].setdefault("esrc", []).append(ei[0].astype(np.int32))
                        cols[kind].setdefault("edst", []).append(ei[1].astype(np.int32))
                    elif torch.is_tensor(v):
                        if v.dim() == 0 or v.shape[0] != n:
                            raise ValueError(f"{kind}.{key}: only node-level tensors are stored")
                        cols[kind].setdefault(key, []).append(np.ascontiguousarray(v.detach().cpu().numpy()))
                    else:
                        vals = list(v)
                        if len(vals) != n or any(x != vals[0] for x in vals):
                            raise ValueError(f"{kind}.{key}: list attributes must repeat one value per building")
                        lists[kind].setdefault(key, []).append(vals[0])
                counts[kind].append((n, int(getattr(g, "edge_index").shape[1])))
            n_items += 1
        if n_items == 0:
            raise ValueError("no buildings to write")
        meta = {"format": FORMAT, "version": VERSION, "num_buildings": n_items, "graphs": {}}
        for kind in KINDS:
            nn_ = np.array([c[0] for c in counts[kind]], dtype=np.int64)
            ne_ = np.array([c[1] for c in counts[kind]], dtype=np.int64)
            np.save(os.path.join(path, f"{kind}.node_ptr.npy"), np.concatenate([[0], np.cumsum(nn_)]).astype(np.int64))
            np.save(os.path.join(path, f"{kind}.edge_ptr.npy"), np.concatenate([[0], np.cumsum(ne_)]).astype(np.int64))
            node_keys = []
            for key, parts in cols[kind].items():
                # one dtype per key: torch's promotion over all buildings (a JSON
                # int site_area next to float ones -> float32, as torch.cat does)
                dt = _NP_TO_TORCH[parts[0].dtype]
                for q in parts[1:]:
                    dt = torch.promote_types(dt, _NP_TO_TORCH[q.dtype])
                np_dt = next(k for k, v in _NP_TO_TORCH.items() if v == dt)
                arr = np.concatenate([q.astype(np_dt, copy=False) for q in parts], axis=0)
                np.save(os.path.join(path, f"{kind}.{key}.npy"), arr, allow_pickle=False)
                if key not in ("esrc", "edst"):
                    node_keys.append(key)
            meta["graphs"][kind] = {"keys": order[kind], "node_keys": node_keys, "lists": lists[kind]}
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(meta, f)
        return GraphStore(path)

    # ------------------------------------------------------------------- read
    def __len__(self) -> int:
        return self.num_buildings

    def num_nodes(self, kind: str, i: int) -> int:
        p = self._arr[kind]["node_ptr"]
        return int(p[i + 1] - p[i])

    def _graph(self, kind: str, i: int) -> GraphData:
        a = self._arr[kind]
        g = self.meta["graphs"][kind]
        n0, n1 = int(a["node_ptr"][i]), int(a["node_ptr"][i + 1])
        e0, e1 = int(a["edge_ptr"][i]), int(a["edge_ptr"][i + 1])
        out = {}
        for key in g["keys"]:
            if key == "edge_index":
                out[key] = torch.from_numpy(np.stack([a["esrc"][e0:e1], a["edst"][e0:e1]]).astype(np.int64))
            elif key in g["lists"]:
                out[key] = [g["lists"][key][i]] * (n1 - n0)
            else:
                out[key] = torch.from_numpy(np.array(a[key][n0:n1]))
        return GraphData(**out)

    def __getitem__(self, i: int) -> Tuple[GraphData, GraphData]:
        i = int(i)
        if not 0 <= i < self.num_buildings:
            raise IndexError(i)
        return self._graph("local", i), self._graph("voxel", i)

    # ---------------------------------------------------------------- collate
    def _collate_kind(self, kind: str, index: np.ndarray, pin: bool, threads: int) -> GraphBatch:
        lib = host_lib()
        a = self._arr[kind]
        g = self.meta["graphs"][kind]
        count = int(index.size)
        common = (_np_ptr(a["node_ptr"]), _np_ptr(a["edge_ptr"]), _np_ptr(a["esrc"]), _np_ptr(a["edst"]),
                  self.num_buildings, _np_ptr(index), count)
        sizes = np.zeros(3, dtype=np.int64)
        _host_check(lib.vgh_collate_sizes(*common, _np_ptr(sizes)), "vgh_collate_sizes")
        n, e, ep = (int(v) for v in sizes)

        def empty(shape, dtype):
            return torch.empty(shape, dtype=dtype, pin_memory=pin)

        out = {}
        ptr = empty((count + 1,), torch.int64)
        batch = empty((n,), torch.int64)
        edge_index = empty((2, e), torch.int64)
        csr = None
        if kind in CSR_KINDS:
            csr = (empty((n + 1,), torch.int32), empty((ep,), torch.int32), empty((n + 1,), torch.int32),
                   empty((ep,), torch.int32), empty((ep,), torch.int32))
        _host_check(lib.vgh_collate_graph(*common, threads, _t_ptr(ptr), _t_ptr(batch), _t_ptr(edge_index),
                                          *(_t_ptr(t) for t in (csr or (None,) * 5))), "vgh_collate_graph")
        for key in g["keys"]:
            if key == "edge_index":
                out[key] = edge_index
            elif key in g["lists"]:
                vals = g["lists"][key]
                out[key] = [[vals[int(b)]] * self.num_nodes(kind, int(b)) for b in index]
            else:
                src = a[key]
                dst = empty((n,) + tuple(src.shape[1:]), _NP_TO_TORCH[src.dtype])
                row_bytes = int(src.strides[0]) if src.ndim > 1 else src.dtype.itemsize
                if not src.flags.c_contiguous:
                    raise ValueError(f"{kind}.{key} is not C-contiguous")
                _host_check(lib.vgh_collate_rows(_np_ptr(src), row_bytes, _np_ptr(a["node_ptr"]), self.num_buildings,
                                                 _np_ptr(index), count, _t_ptr(dst), threads), "vgh_collate_rows")
                out[key] = dst
        out["batch"] = batch
        out["ptr"] = ptr
        gb = GraphBatch(**out)
        gb.set_derived("ptr_host", [int(v) for v in ptr.tolist()])
        if csr is not None:
            gb.set_derived("csr_arrays", csr)
            # the largest in-degree (self loop included) from the host row_ptr:
            # the device side sizes its padded column array (CSR.ell) without a sync
            rp = csr[0].numpy()
            gb.set_derived("csr_max_degree", int(np.diff(rp).max()) if rp.size > 1 else 0)
        return gb

    def collate(self, indices: Sequence[int], pin: bool = False, threads: int = 4) -> Tuple[GraphBatch, GraphBatch]:
        """(local, voxel) GraphBatch of the buildings ``indices`` (in order);
        ``pin`` allocates page-locked buffers for an asynchronous upload."""
        index = np.ascontiguousarray(np.asarray(list(indices), dtype=np.int64))
        if index.size == 0:
            raise ValueError("collate needs at least one building")
        return tuple(self._collate_kind(kind, index, pin, threads) for kind in KINDS)  # type: ignore[return-value]


def write_store(path: str, dataset, indices: Optional[Sequence[int]] = None) -> GraphStore:
    """Write ``dataset[i]`` (a ``(local, voxel)`` pair per index) as a store."""
    idx = range(len(dataset)) if indices is None else indices
    return GraphStore.write(path, (dataset[i] for i in idx))
