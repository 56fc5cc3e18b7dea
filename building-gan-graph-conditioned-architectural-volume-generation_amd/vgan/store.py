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
import math
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
    "vgh_collate_max_in_degree": (ctypes.c_int, [_p, _p, _p, _p, _i64, _p, _i32, _p]),
    "vgh_pool_pid": (_i64, []),
    "vgh_csr_ell": (ctypes.c_int, [_p, _p, _i32, _i32, _p]),
    "vgh_csr_stacked": (ctypes.c_int, [_p, _p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p]),
    "vgh_type_mean": (ctypes.c_int, [_p, _p, _i32, _i32, _p, _i32, _i32, _p, _i32, _i32]),
}
ELL_WIDTHS = (8, 16, 32)  # vgan.ops.ELL_WIDTHS
CRITIC_COPIES = 3  # the critic engine's stacked real / fake / mix graph (vgan.critic)


def _prepare_spec(prepare):
    """``prepare``: the number of classes (training batches: the critic's 3
    block-diagonal copies are built too), or (classes, stacked copy counts)
    -- e.g. (7, ()) for inference batches, which build their stacked graph
    on the device."""
    if isinstance(prepare, (tuple, list)):
        k, copies = int(prepare[0]), tuple(sorted({int(c) for c in prepare[1] if int(c) > 1}))
    else:
        k, copies = int(prepare), (CRITIC_COPIES,)
    return k, copies
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
    # Every tensor of a collated (local, voxel) pair -- and, with ``prepare``,
    # the per-batch structures vgan.data would otherwise build on the device
    # -- is carved out of ONE host buffer (page-locked for the loader), so a
    # new batch reaches the GPU as one host-to-device copy (``upload_pair``).

    def _layout(self, index: np.ndarray, prepare):
        """(sizes per kind, [(name, shape, torch dtype)]) of a pair's buffer."""
        lib = host_lib()
        count = int(index.size)
        items, sizes = [], {}
        for kind in KINDS:
            a = self._arr[kind]
            common = (_np_ptr(a["node_ptr"]), _np_ptr(a["edge_ptr"]), _np_ptr(a["esrc"]), _np_ptr(a["edst"]),
                      self.num_buildings, _np_ptr(index), count)
            sz = np.zeros(3, dtype=np.int64)
            _host_check(lib.vgh_collate_sizes(*common, _np_ptr(sz)), "vgh_collate_sizes")
            n, e, ep = (int(v) for v in sz)
            sizes[kind] = (n, e, ep, common)
            items += [(f"{kind}.ptr", (count + 1,), torch.int64), (f"{kind}.batch", (n,), torch.int64),
                      (f"{kind}.edge_index", (2, e), torch.int64)]
            if kind in CSR_KINDS:
                items += [(f"{kind}.csr.{k}", (n + 1,) if k.endswith("ptr") else (ep,), torch.int32)
                          for k in ("row_ptr", "col", "csc_ptr", "csc_slot", "csc_dst")]
            g = self.meta["graphs"][kind]
            for key in g["keys"]:
                if key != "edge_index" and key not in g["lists"]:
                    src = a[key]
                    items.append((f"{kind}.{key}", (n,) + tuple(src.shape[1:]), _NP_TO_TORCH[src.dtype]))
        extras = None
        if prepare is not None:
            n, _, ep, common = sizes["voxel"]
            md = np.zeros(1, dtype=np.int32)
            _host_check(host_lib().vgh_collate_max_in_degree(*common, _np_ptr(md)), "vgh_collate_max_in_degree")
            w = next((x for x in ELL_WIDTHS if int(md[0]) <= x), 0)
            fl = int(self._arr["local"]["x"].shape[1])
            fv = int(self._arr["voxel"]["x"].shape[1])
            k, copies = _prepare_spec(prepare)
            extras = {"max_degree": int(md[0]), "ell_width": w, "n_classes": k, "fl": fl, "copies": copies}
            items += [("prep.matched_voxel_x", (n, fl + fv), torch.float32), ("prep.matched_x", (n, fl), torch.float32),
                      ("prep.onehot_f", (n, k), torch.float32), ("prep.critic_seeds4", (4 * n, 1), torch.float32)]
            for c in copies:
                items += [(f"prep.stacked{c}.{kk}", (c * n + 1,) if kk.endswith("ptr") else (c * ep,), torch.int32)
                          for kk in ("row_ptr", "col", "csc_ptr", "csc_slot", "csc_dst")]
                if w:
                    items.append((f"prep.stacked{c}_ell", (c * n * w,), torch.int32))
            if w:
                items.append(("prep.ell", (n * w,), torch.int32))
        return sizes, items, extras

    def collate_pair(self, indices: Sequence[int], pin: bool = False, threads: int = 4,
                     prepare=None) -> Tuple[GraphBatch, GraphBatch]:
        """(local, voxel) GraphBatch of the buildings ``indices`` (in order), all
        tensors views of one host buffer (page-locked with ``pin``).
        ``prepare`` = the number of classes (or (classes, extra stacked copy
        counts), ``_prepare_spec``): also the voxel batch's per-batch
        structures (vgan.data.prepared: padded columns, the critic's stacked
        graph and its padded columns, the type-matched mean | voxel.x, the float
        one-hot, the critic's adjoint seeds), bit for bit what the device
        would build."""
        index = np.ascontiguousarray(np.asarray(list(indices), dtype=np.int64))
        if index.size == 0:
            raise ValueError("collate needs at least one building")
        lib = host_lib()
        sizes, items, extras = self._layout(index, prepare)
        layout, off = {}, 0
        for name, shape, dt in items:
            nbytes = _nbytes(shape, dt)
            layout[name] = (off, tuple(shape), dt)
            off += (nbytes + 255) // 256 * 256
        blob = torch.empty(max(off, 256), dtype=torch.uint8, pin_memory=pin)
        v = _host_views(blob, layout)
        out = []
        for kind in KINDS:
            n, e, ep, common = sizes[kind]
            csr = tuple(v[f"{kind}.csr.{k}"] for k in ("row_ptr", "col", "csc_ptr", "csc_slot", "csc_dst")) \
                if kind in CSR_KINDS else (None,) * 5
            _host_check(lib.vgh_collate_graph(*common, threads, _t_ptr(v[f"{kind}.ptr"]), _t_ptr(v[f"{kind}.batch"]),
                                              _t_ptr(v[f"{kind}.edge_index"]), *(_t_ptr(t) for t in csr)),
                        "vgh_collate_graph")
            a = self._arr[kind]
            g = self.meta["graphs"][kind]
            attrs = {}
            for key in g["keys"]:
                if key == "edge_index":
                    attrs[key] = v[f"{kind}.edge_index"]
                elif key in g["lists"]:
                    vals = g["lists"][key]
                    attrs[key] = [[vals[int(b)]] * self.num_nodes(kind, int(b)) for b in index]
                else:
                    src, dst = a[key], v[f"{kind}.{key}"]
                    if not src.flags.c_contiguous:
                        raise ValueError(f"{kind}.{key} is not C-contiguous")
                    row_bytes = int(src.strides[0]) if src.ndim > 1 else src.dtype.itemsize
                    _host_check(lib.vgh_collate_rows(_np_ptr(src), row_bytes, _np_ptr(a["node_ptr"]),
                                                     self.num_buildings, _np_ptr(index), int(index.size),
                                                     _t_ptr(dst), threads), "vgh_collate_rows")
                    attrs[key] = dst
            attrs["batch"] = v[f"{kind}.batch"]
            attrs["ptr"] = v[f"{kind}.ptr"]
            gb = GraphBatch(**attrs)
            gb.set_derived("ptr_host", attrs["ptr"].tolist())
            if kind in CSR_KINDS:
                gb.set_derived("csr_arrays", csr)
                # the largest in-degree (self loop included) from the host row_ptr:
                # the device side sizes its padded column array without a sync
                rp = csr[0].numpy()
                gb.set_derived("csr_max_degree", int(np.diff(rp).max()) if rp.size > 1 else 0)
            out.append(gb)
        local, voxel = out
        if extras is not None:
            self._prepare(local, voxel, v, extras)
        for gb in out:
            gb.set_derived("blob", (blob, layout))
        return local, voxel

    @staticmethod
    def _prepare(local: GraphBatch, voxel: GraphBatch, v: Dict[str, torch.Tensor], extras: dict) -> None:
        lib = host_lib()
        n = voxel.num_nodes
        rp, col, cp, cs, cd = voxel.derived("csr_arrays")
        ep = col.numel()
        k, fl, w = extras["n_classes"], extras["fl"], extras["ell_width"]
        lx = local.x
        if lx.dtype != torch.float32 or not lx.is_contiguous() or local.type.dtype != torch.int64 \
                or voxel.type.dtype != torch.int64 or voxel.x.dtype != torch.float32:
            raise ValueError("prepare: local.x / voxel.x must be float32 and the types int64")
        mv = v["prep.matched_voxel_x"]
        _host_check(lib.vgh_type_mean(_t_ptr(lx), _t_ptr(local.type), lx.shape[0], fl, _t_ptr(voxel.type), n, k,
                                      _t_ptr(mv), mv.shape[1], 0), "vgh_type_mean")
        # numpy, not torch, for the host copies: torch's CPU copy between two
        # views of one storage took 30-40 ms here (its intra-op thread pool,
        # on the loader's thread), numpy's 0.1 ms
        mvn = mv.numpy()
        np.copyto(mvn[:, fl:], voxel.x.numpy())
        np.copyto(v["prep.matched_x"].numpy(), mvn[:, :fl])
        np.copyto(v["prep.onehot_f"].numpy(), voxel.types_onehot.numpy(), casting="unsafe")
        seeds = v["prep.critic_seeds4"].numpy()  # vgan.critic.CriticEngine.prepare_batch
        seeds[:n] = np.float32(-1.0 / n)
        seeds[n:2 * n] = np.float32(1.0 / n)
        seeds[2 * n:3 * n] = 0.0
        seeds[3 * n:] = 1.0
        names = ["matched_voxel_x", "matched_x", "onehot_f", "critic_seeds4"]
        if w:
            _host_check(lib.vgh_csr_ell(_t_ptr(rp), _t_ptr(col), n, w, _t_ptr(v["prep.ell"])), "vgh_csr_ell")
            names.append("ell")
        for c in extras["copies"]:
            st = tuple(v[f"prep.stacked{c}.{kk}"] for kk in ("row_ptr", "col", "csc_ptr", "csc_slot", "csc_dst"))
            _host_check(lib.vgh_csr_stacked(*(_t_ptr(t) for t in (rp, col, cp, cs, cd)), n, ep, c,
                                            *(_t_ptr(t) for t in st)), "vgh_csr_stacked")
            names += [f"stacked{c}.{kk}" for kk in ("row_ptr", "col", "csc_ptr", "csc_slot", "csc_dst")]
            if w:
                _host_check(lib.vgh_csr_ell(_t_ptr(st[0]), _t_ptr(st[1]), c * n, w, _t_ptr(v[f"prep.stacked{c}_ell"])),
                            "vgh_csr_ell")
                names.append(f"stacked{c}_ell")
        voxel.set_derived("prepared_arrays", {
            "names": names, "views": {nm: v[f"prep.{nm}"] for nm in names}, "ell_width": w,
            "max_degree": extras["max_degree"], "n_classes": k, "copies": extras["copies"],
            # the program batch these were built from (vgan.data checks the pairing)
            "local": (local.x.data_ptr(), local.type.data_ptr())})
        _stamp_versions(local, voxel)

    def collate(self, indices: Sequence[int], pin: bool = False, threads: int = 4,
                prepare=None) -> Tuple[GraphBatch, GraphBatch]:
        """(local, voxel) GraphBatch of the buildings ``indices`` (in order);
        ``pin`` allocates the page-locked buffer of an asynchronous upload."""
        return self.collate_pair(indices, pin=pin, threads=threads, prepare=prepare)


_ELEM_SIZE = {dt: torch.empty((), dtype=dt).element_size() for dt in (torch.int32, torch.int64, torch.float32,
                                                                        torch.float64, torch.int8, torch.uint8,
                                                                        torch.int16, torch.float16, torch.bool)}


def _nbytes(shape, dtype) -> int:
    return math.prod(shape) * _ELEM_SIZE[dtype]


_TORCH_TO_NP = {v: k for k, v in _NP_TO_TORCH.items()}
_TORCH_TO_NP.update({torch.int8: np.dtype(np.int8), torch.int16: np.dtype(np.int16),
                     torch.float16: np.dtype(np.float16)})


def _view(blob: torch.Tensor, off: int, shape, dtype) -> torch.Tensor:
    return blob[off:off + _nbytes(shape, dtype)].view(dtype).view(shape)


# Views of a collated buffer, ~60 per pair: torch's slice + two views cost
# ~8 us of interpreter time each (a third of the loader's time per batch);
# a numpy view wrapped by from_numpy (host) or an empty tensor re-pointed at
# the device buffer's storage (device) ~1.5-2.5 us.
def _host_views(blob: torch.Tensor, layout) -> Dict[str, torch.Tensor]:
    raw = blob.numpy()
    out = {}
    for name, (off, shape, dt) in layout.items():
        a = raw[off:off + _nbytes(shape, dt)].view(_TORCH_TO_NP[dt]).reshape(shape)
        out[name] = torch.from_numpy(a)
    return out


def _contig_strides(shape) -> Tuple[int, ...]:
    st, acc = [], 1
    for d in reversed(shape):
        st.append(acc)
        acc *= int(d)
    return tuple(reversed(st))


def _device_views(dev_blob: torch.Tensor, layout) -> Dict[str, torch.Tensor]:
    storage = dev_blob.untyped_storage()
    base = dev_blob.storage_offset()
    proto = {}
    out = {}
    for name, (off, shape, dt) in layout.items():
        p = proto.get(dt)
        if p is None:
            p = proto[dt] = torch.empty(0, dtype=dt, device=dev_blob.device)
        size = _ELEM_SIZE[dt]
        out[name] = p.new_empty(0).set_(storage, (base + off) // size, tuple(shape), _contig_strides(shape))
    return out


def upload_pair(local: GraphBatch, voxel: GraphBatch, device, non_blocking: bool = True
                ) -> Tuple[GraphBatch, GraphBatch]:
    """A collated pair on ``device``: its host buffer copied in ONE
    host-to-device copy, every tensor (node attributes, the CSR / CSC, the
    prepared structures) a view of the device copy.  Pairs without a shared
    buffer fall back to per-tensor ``.to``."""
    b1, b2 = local.derived("blob"), voxel.derived("blob")
    if b1 is None or b2 is None or b1[0] is not b2[0]:
        return local.to(device, non_blocking=non_blocking), voxel.to(device, non_blocking=non_blocking)
    blob, layout = b1
    dev_blob = blob.to(device, non_blocking=non_blocking)
    host0 = blob.data_ptr()
    dv = _device_views(dev_blob, layout)
    by_ptr = {(host0 + off, tuple(shape), dt): dv[name] for name, (off, shape, dt) in layout.items()}

    def move(t):
        if not torch.is_tensor(t):
            return t
        hit = by_ptr.get((t.data_ptr(), tuple(t.shape), t.dtype))
        return hit if hit is not None else t.to(device, non_blocking=non_blocking)

    out = []
    for gb in (local, voxel):
        moved = GraphBatch(**{k: move(getattr(gb, k)) for k in gb.keys()})
        for key in ("ptr_host", "csr_max_degree"):
            if gb.derived(key) is not None:
                moved.set_derived(key, gb.derived(key))
        if gb.derived("csr_arrays") is not None:
            moved.set_derived("csr_arrays", tuple(move(t) for t in gb.derived("csr_arrays")))
        pa = gb.derived("prepared_arrays")
        if pa is not None:
            moved.set_derived("prepared_arrays", dict(pa, views={k: move(t) for k, t in pa["views"].items()}))
        moved.set_derived("device_blob", dev_blob)
        out.append(moved)
    lo, vo = out
    pa = vo.derived("prepared_arrays")
    if pa is not None:  # the pairing key, now of the device tensors
        vo.set_derived("prepared_arrays", dict(pa, local=(lo.x.data_ptr(), lo.type.data_ptr())))
        _stamp_versions(lo, vo)
    return lo, vo


def _stamp_versions(local: GraphBatch, voxel: GraphBatch) -> None:
    """The identity of every input when the prepared structures were built --
    address, shape and autograd version of each tensor (``vgan.data._inputs_key``):
    an in-place edit, or an attribute REPLACED by a new tensor (whose version
    is 0 again), afterwards invalidates them."""
    from .data import _inputs_key

    pa = voxel.derived("prepared_arrays")
    pa["inputs_key"] = _inputs_key(local, voxel)


def write_store(path: str, dataset, indices: Optional[Sequence[int]] = None) -> GraphStore:
    """Write ``dataset[i]`` (a ``(local, voxel)`` pair per index) as a store."""
    idx = range(len(dataset)) if indices is None else indices
    return GraphStore.write(path, (dataset[i] for i in idx))
