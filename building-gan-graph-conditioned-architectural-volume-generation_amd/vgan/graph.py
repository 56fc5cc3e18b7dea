"""Graph containers: one building (``GraphData``) and a collated mini-batch (``GraphBatch``).

These replace the two PyG containers the reference path touches:

* ``torch_geometric.data.Data`` built per building at ``data.py:117-147``;
* ``torch_geometric.data.Batch.from_data_list`` called by the collate at
  ``data.py:156-163``.

Only the behaviour the path relies on is provided: node-level tensors are
concatenated along dim 0, ``edge_index`` is shifted by the running node count,
list attributes (``data_number``) become a list of lists, ``batch``/``ptr``
describe the graph membership, ``batch[gi]`` slices one building back out
(``trainer.py:364,421``) and ``.to(device)`` moves every tensor.

On top of that the batch owns the per-batch derived structures of the HIP
path (destination-sorted CSR with self loops, its source-sorted transpose) so
that they are built once per batch instead of once per GATConv call.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional

import torch

_INCREMENT_KEYS = ("edge_index",)


class GraphData:
    """One building: a bag of named tensors/lists with PyG ``Data`` access style."""

    def __init__(self, **attrs: Any):
        object.__setattr__(self, "_store", {})
        for key, value in attrs.items():
            self._store[key] = value

    def __getattr__(self, key: str) -> Any:
        store = object.__getattribute__(self, "_store")
        if key in store:
            return store[key]
        raise AttributeError(key)

    def __setattr__(self, key: str, value: Any) -> None:
        self._store[key] = value

    def keys(self) -> List[str]:
        return list(self._store.keys())

    @property
    def num_nodes(self) -> int:
        return int(self._store["x"].shape[0])

    def to(self, device, non_blocking: bool = False) -> "GraphData":
        moved = {
            k: (v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v)
            for k, v in self._store.items()
        }
        return GraphData(**moved)


class GraphBatch(GraphData):
    """A collated set of buildings (PyG ``Batch`` semantics for the used subset)."""

    def __init__(self, **attrs: Any):
        super().__init__(**attrs)
        object.__setattr__(self, "_derived", {})

    # ------------------------------------------------------------------ collate
    @classmethod
    def from_data_list(cls, items: Iterable[GraphData]) -> "GraphBatch":
        items = list(items)
        if not items:
            raise ValueError("from_data_list needs at least one graph")
        keys = items[0].keys()
        counts = [it.num_nodes for it in items]
        offsets = [0]
        for c in counts:
            offsets.append(offsets[-1] + c)
        out: Dict[str, Any] = {}
        for key in keys:
            vals = [getattr(it, key) for it in items]
            if torch.is_tensor(vals[0]):
                if key in _INCREMENT_KEYS:
                    out[key] = torch.cat([v + offsets[i] for i, v in enumerate(vals)], dim=1)
                else:
                    out[key] = torch.cat(vals, dim=0)
            else:
                out[key] = list(vals)
        device = items[0].x.device
        out["batch"] = torch.repeat_interleave(
            torch.arange(len(items), device=device), torch.tensor(counts, device=device)
        )
        out["ptr"] = torch.tensor(offsets, dtype=torch.long, device=device)
        return cls(**out)

    # --------------------------------------------------------------- accessors
    @property
    def num_graphs(self) -> int:
        return int(self._store["ptr"].numel() - 1)

    def _ptr_host(self) -> List[int]:
        cached = self._derived.get("ptr_host")
        if cached is None:
            cached = [int(v) for v in self._store["ptr"].cpu().tolist()]
            self._derived["ptr_host"] = cached
        return cached

    def __getitem__(self, gi: int) -> GraphData:
        ptr = self._ptr_host()
        lo, hi = ptr[gi], ptr[gi + 1]
        out: Dict[str, Any] = {}
        for key, value in self._store.items():
            if key in ("batch", "ptr"):
                continue
            if torch.is_tensor(value):
                if key in _INCREMENT_KEYS:
                    mask = (value[0] >= lo) & (value[0] < hi)
                    out[key] = value[:, mask] - lo
                else:
                    out[key] = value[lo:hi]
            else:
                out[key] = value[gi]
        return GraphData(**out)

    def to(self, device, non_blocking: bool = False) -> "GraphBatch":
        device = torch.device(device)
        tensors = [v for v in self._store.values() if torch.is_tensor(v)]
        if tensors and all(_same_device(v.device, device) for v in tensors):
            return self  # already there: keep the derived structures built on it
        moved = {
            k: (v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v)
            for k, v in self._store.items()
        }
        out = GraphBatch(**moved)
        if "ptr_host" in self._derived:
            out._derived["ptr_host"] = self._derived["ptr_host"]
        if "csr_arrays" in self._derived:  # host-built CSR/CSC (vgan.store) travels with the batch
            out._derived["csr_arrays"] = tuple(t.to(device, non_blocking=non_blocking)
                                               for t in self._derived["csr_arrays"])
            if "csr_max_degree" in self._derived:
                out._derived["csr_max_degree"] = self._derived["csr_max_degree"]
        pa = self._derived.get("prepared_arrays")
        if pa is not None and "x" in self._store:  # host-built per-batch structures (vgan.store)
            out._derived["prepared_arrays"] = dict(pa, views={k: t.to(device, non_blocking=non_blocking)
                                                              for k, t in pa["views"].items()}, local=None)
        return out

    # ------------------------------------------------------- derived, per batch
    def derived(self, key: str) -> Optional[Any]:
        return self._derived.get(key)

    def set_derived(self, key: str, value: Any) -> None:
        self._derived[key] = value

    def clear_derived(self, keep: Iterable[str] = ()) -> None:
        """Drop every derived structure except ``keep``."""
        keep = set(keep)
        for key in [k for k in self._derived if k not in keep]:
            del self._derived[key]


def _same_device(a: torch.device, b: torch.device) -> bool:
    if a.type != b.type:
        return False
    if a.type == "cpu":
        return True
    return b.index is None or a.index == b.index
