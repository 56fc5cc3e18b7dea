"""torch-geometric 2.6.1 operator semantics, restated in plain torch (CPU oracle).

The reference pins ``torch-geometric==2.6.1`` (``requirements.txt:11``) and calls
it at ``models.py:22-31,72-73,82-83,90,144,166-175,192-193,202-203,210,242``.
The package is not vendored and not installable here, so each operator below
restates the published 2.6.1 source it names; ``oracle.dense`` derives the same
quantities a second, independent way.

Restated files (package-relative paths inside torch_geometric 2.6.1):

* ``nn/conv/gat_conv.py``  GATConv(in, out) with the defaults the reference uses:
  heads=1, concat=True, negative_slope=0.2, dropout=0.0, add_self_loops=True,
  edge_dim=None, fill_value='mean', bias=True, residual=False.
* ``utils/_softmax.py``     softmax(src, index) -- the ``index`` (scatter) branch.
* ``utils/loop.py``         remove_self_loops / add_self_loops (loops appended).
* ``nn/norm/graph_norm.py`` GraphNorm(C) called with ``batch=None``.
* ``nn/sequential.py``      Sequential("x, edge_index", [...]) children named
  ``module_{i}``.
* ``nn/inits.py``           glorot / zeros; ``nn/dense/linear.py`` Linear.
* ``data/batch.py``         Batch.from_data_list for the attributes the path reads.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

NEG_SLOPE = 0.2
SOFTMAX_EPS = 1e-16
GRAPHNORM_EPS = 1e-5


# ----------------------------------------------------------------- inits.py
def glorot(t: torch.Tensor) -> None:
    bound = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-bound, bound)


class Linear(nn.Module):
    """dense/linear.py Linear with weight_initializer='glorot'."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        glorot(self.weight)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return F.linear(x, self.weight, self.bias)


# ------------------------------------------------------------------ loop.py
def remove_self_loops(edge_index: torch.Tensor) -> torch.Tensor:
    keep = edge_index[0] != edge_index[1]
    return edge_index[:, keep]


def add_self_loops(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    loops = torch.arange(num_nodes, dtype=edge_index.dtype, device=edge_index.device)
    return torch.cat([edge_index, torch.stack([loops, loops])], dim=1)


# -------------------------------------------------------------- _softmax.py
def segment_softmax(src: torch.Tensor, index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """utils.softmax(src, index, num_nodes=N) -- scatter branch.

    max is taken on ``src.detach()``; the denominator carries ``+ 1e-16``.
    """
    shape = (num_nodes,) + tuple(src.shape[1:])
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    seg_max = torch.full(shape, float("-inf"), dtype=src.dtype, device=src.device)
    seg_max = seg_max.scatter_reduce(0, idx, src.detach(), reduce="amax", include_self=True)
    out = (src - seg_max.index_select(0, index)).exp()
    seg_sum = torch.zeros(shape, dtype=src.dtype, device=src.device).scatter_add(0, idx, out)
    seg_sum = seg_sum + SOFTMAX_EPS
    return out / seg_sum.index_select(0, index)


# -------------------------------------------------------------- gat_conv.py
class GATConv(nn.Module):
    """GATConv(in, out), heads = 1; parameters ``lin.weight``, ``att_src``,
    ``att_dst`` ([1, 1, out]) and ``bias`` ([out])."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, 1
        self.lin = Linear(in_channels, out_channels, bias=False)
        self.att_src = nn.Parameter(torch.empty(1, 1, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, 1, out_channels))
        self.bias = nn.Parameter(torch.empty(out_channels))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        self.lin.reset_parameters()
        glorot(self.att_src)
        glorot(self.att_dst)
        with torch.no_grad():
            self.bias.zero_()

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        c = self.out_channels
        h = self.lin(x).view(-1, 1, c)
        a_src = (h * self.att_src).sum(-1)  # [N, 1]
        a_dst = (h * self.att_dst).sum(-1)
        out = gat_propagate(h.view(-1, c), a_src.view(-1), a_dst.view(-1), edge_index,
                            training=self.training)
        return out + self.bias


def gat_propagate(h: torch.Tensor, a_src: torch.Tensor, a_dst: torch.Tensor, edge_index: torch.Tensor,
                  slope: float = NEG_SLOPE, training: bool = False) -> torch.Tensor:
    """GATConv after the projection: self loops, edge_update (leaky_relu +
    softmax + dropout p=0) and propagate ('add' aggregation), heads = 1."""
    n, c = h.shape
    ei = add_self_loops(remove_self_loops(edge_index), n)
    src, dst = ei[0], ei[1]
    logit = F.leaky_relu(a_src.view(-1, 1).index_select(0, src) + a_dst.view(-1, 1).index_select(0, dst), slope)
    alpha = segment_softmax(logit, dst, n)
    alpha = F.dropout(alpha, p=0.0, training=training)
    msg = alpha.unsqueeze(-1) * h.view(-1, 1, c).index_select(0, src)  # [E', 1, C]
    out = torch.zeros(n, 1, c, dtype=msg.dtype, device=msg.device).index_add_(0, dst, msg)
    return out.view(-1, c)


# ------------------------------------------------------------ graph_norm.py
class GraphNorm(nn.Module):
    """GraphNorm(C); the reference only ever calls it as ``norm(x)`` (batch=None).

    nn/norm/graph_norm.py (2.6.1) ``forward``, batch=None branch:
    ``out = x - mean(x) * mean_scale``; ``var = mean(out ** 2)``;
    ``std = sqrt(var + eps)``; ``weight * out / std + bias``."""

    def __init__(self, in_channels: int, eps: float = GRAPHNORM_EPS):
        super().__init__()
        self.in_channels, self.eps = in_channels, eps
        self.weight = nn.Parameter(torch.ones(in_channels))
        self.bias = nn.Parameter(torch.zeros(in_channels))
        self.mean_scale = nn.Parameter(torch.ones(in_channels))

    def forward(self, x: torch.Tensor, batch: Optional[torch.Tensor] = None,
                batch_size: Optional[int] = None) -> torch.Tensor:
        if batch is not None:
            raise NotImplementedError("the reference path never passes a batch vector")
        out = x - x.mean(dim=0, keepdim=True) * self.mean_scale
        var = out.pow(2).mean(dim=0, keepdim=True)
        std = (var + self.eps).sqrt()
        return self.weight * out / std + self.bias


# ------------------------------------------------------------ sequential.py
class Sequential(nn.Module):
    """Sequential(input_args, modules): (module, "x, edge_index -> x") entries get
    the named inputs; bare modules get the previous output."""

    def __init__(self, input_args: str, modules: List[Any]):
        super().__init__()
        self.input_args = [a.strip() for a in input_args.split(",")]
        self._specs: List[Optional[List[str]]] = []
        for i, entry in enumerate(modules):
            if isinstance(entry, (tuple, list)):
                module, desc = entry
                lhs = desc.split("->")[0]
                self._specs.append([a.strip() for a in lhs.split(",")])
            else:
                module = entry
                self._specs.append(None)
            self.add_module(f"module_{i}", module)

    def forward(self, *args, **kwargs):
        env: Dict[str, Any] = dict(zip(self.input_args, args))
        env.update(kwargs)
        x = env[self.input_args[0]]
        for i, spec in enumerate(self._specs):
            module = getattr(self, f"module_{i}")
            if spec is None:
                x = module(x)
            else:
                x = module(*[env[a] if a != self.input_args[0] else x for a in spec])
            env[self.input_args[0]] = x
        return x


# ------------------------------------------------------------------ batch.py
class Data:
    """Minimal ``torch_geometric.data.Data`` (attribute bag)."""

    def __init__(self, **kwargs):
        self.__dict__["_d"] = dict(kwargs)

    def __getattr__(self, key):
        d = self.__dict__["_d"]
        if key in d:
            return d[key]
        raise AttributeError(key)

    def __setattr__(self, key, value):
        self.__dict__["_d"][key] = value

    def keys(self):
        return list(self._d.keys())

    @property
    def num_nodes(self) -> int:
        return int(self._d["x"].shape[0])

    def to(self, device, *args, **kwargs):
        return type(self)(**{k: (v.to(device) if torch.is_tensor(v) else v) for k, v in self._d.items()})


class Batch(Data):
    """``Batch.from_data_list`` for node tensors, ``edge_index`` and list attrs."""

    @classmethod
    def from_data_list(cls, data_list):
        data_list = list(data_list)
        sizes = [d.num_nodes for d in data_list]
        starts = [sum(sizes[:k]) for k in range(len(sizes) + 1)]
        out = {}
        for key in data_list[0].keys():
            vals = [getattr(d, key) for d in data_list]
            if torch.is_tensor(vals[0]):
                if key == "edge_index":
                    out[key] = torch.cat([v + starts[k] for k, v in enumerate(vals)], 1)
                else:
                    out[key] = torch.cat(vals, 0)
            else:
                out[key] = vals
        out["batch"] = torch.cat([torch.full((s,), k, dtype=torch.long) for k, s in enumerate(sizes)])
        out["ptr"] = torch.tensor(starts, dtype=torch.long)
        return cls(**out)

    @property
    def num_graphs(self) -> int:
        return int(self._d["ptr"].numel() - 1)

    def __getitem__(self, gi: int) -> Data:
        lo, hi = int(self._d["ptr"][gi]), int(self._d["ptr"][gi + 1])
        out = {}
        for key, val in self._d.items():
            if key in ("batch", "ptr"):
                continue
            if torch.is_tensor(val):
                if key == "edge_index":
                    keep = (val[0] >= lo) & (val[0] < hi)
                    out[key] = val[:, keep] - lo
                else:
                    out[key] = val[lo:hi]
            else:
                out[key] = val[gi]
        return Data(**out)


class Dataset:
    """Placeholder base for ``torch_geometric.data.Dataset`` subclassing."""

    def __init__(self, *args, **kwargs):
        pass


# ------------------------------------------------- message order (index view)
def gat_csr(edge_index: torch.Tensor, num_nodes: int):
    """(row_ptr, col, csc_ptr, csc_slot, csc_dst) of the edge list GATConv
    propagates over -- add_self_loops(remove_self_loops(edge_index)) -- grouped
    by destination in the order the scatter visits the edges (original edge
    order, the appended self loop last), and its transpose grouped by source in
    slot order.  Pure-Python loops: small graphs only (test checker for
    csr.hip and the host collate)."""
    ei = add_self_loops(remove_self_loops(edge_index), num_nodes).tolist()
    rows = [[] for _ in range(num_nodes)]
    for s, d in zip(ei[0], ei[1]):
        rows[d].append(s)
    row_ptr, col = [0], []
    for r in rows:
        col.extend(r)
        row_ptr.append(len(col))
    buckets = [[] for _ in range(num_nodes)]
    for i in range(num_nodes):
        for k in range(row_ptr[i], row_ptr[i + 1]):
            buckets[col[k]].append((k, i))
    csc_ptr, csc_slot, csc_dst = [0], [], []
    for b in buckets:
        csc_slot.extend(k for k, _ in b)
        csc_dst.extend(i for _, i in b)
        csc_ptr.append(len(csc_slot))
    as_i32 = lambda v: torch.tensor(v, dtype=torch.int32)  # noqa: E731
    return as_i32(row_ptr), as_i32(col), as_i32(csc_ptr), as_i32(csc_slot), as_i32(csc_dst)
