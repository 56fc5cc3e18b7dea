"""Independent dense-adjacency derivation of the GATConv / GraphNorm arithmetic.

Used only to cross-check ``oracle.pyg`` (two formulations of the same
published semantics must agree to ~1e-12 in float64).  The sparse oracle works
edge by edge with scatter/gather; this one builds the N x N incoming-edge mask
(self loops on the diagonal, original self loops dropped first -- GATConv's
remove/add pair) and takes a masked row softmax.
"""
from __future__ import annotations

import torch


def incoming_mask(edge_index: torch.Tensor, n: int) -> torch.Tensor:
    """M[i, j] = 1 iff there is an edge j -> i (dst i, src j), diagonal forced on."""
    m = torch.zeros(n, n, dtype=torch.bool)
    m[edge_index[1], edge_index[0]] = True
    m.fill_diagonal_(True)
    return m


def gat_dense(x, weight, att_src, att_dst, bias, edge_index, slope: float = 0.2):
    h = x @ weight.t()  # [N, C]
    a_s = h @ att_src.reshape(-1)
    a_d = h @ att_dst.reshape(-1)
    n = x.shape[0]
    mask = incoming_mask(edge_index, n)
    raw = a_d[:, None] + a_s[None, :]
    logits = torch.where(raw > 0, raw, slope * raw)
    logits = logits.masked_fill(~mask, float("-inf"))
    p = torch.softmax(logits, dim=1)
    return p @ h + bias, p


def graphnorm_dense(x, weight, bias, mean_scale, eps: float = 1e-5):
    """Column sums written out: mu = 1'x / n, o = x - s*mu, and the second
    moment of o expanded as var(x) + ((1 - s) mu)^2 (o's mean is (1 - s) mu),
    rather than oracle.pyg's mean(o^2) directly."""
    n = x.shape[0]
    mu = x.sum(0) / n
    var_x = (x * x).sum(0) / n - mu * mu
    var_o = var_x + ((1 - mean_scale) * mu) ** 2
    return weight * (x - mean_scale * mu) / torch.sqrt(var_o + eps) + bias
