"""Reference (test-only) for the explicit WGAN-GP critic engine.

The HIP critic (``vgan/critic.py``) replaces autograd's double backward of
``trainer.py:291-332`` with four explicit passes over the discriminator's op
chain x_k = f_k(x_{k-1}; theta_k):

  A  forward of the real / fake / mix copies;
  B  input VJP of the mix copy with seed 1:  d_{k-1} = J_k^T d_k  (g = d_0);
  C  tangent sweep u_k = J_k u_{k-1} from u_0 = dGP/dg, with the second-order
     terms of Q_k = <d_k, J_k u_{k-1}>:  theta_bar_k += dQ_k/dtheta_k and an
     injection xinj_{k-1} = dQ_k/dx_{k-1};
  D  VJP of every copy (seeds -1/N real, +1/N fake, 0 mix) with xinj added
     to the mix copy's adjoints; its parameter gradients add to pass C's.

Here every unit's VJP and second-order terms come from torch autograd on the
oracle's own ops (``oracle.pyg``), in float64, so the pass structure can be
checked against plain double backward on the CPU, and each HIP unit kernel
against these units on the GPU.
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import torch
import torch.nn.functional as F

from oracle import pyg


class Unit:
    def __init__(self, name: str, fn: Callable, params: Sequence[str]):
        self.name, self.fn, self.params = name, fn, list(params)

    def fwd(self, x, P):
        return self.fn(x, *[P[k] for k in self.params])

    def _leaves(self, x, P):
        x = x.detach().requires_grad_(True)
        ps = [P[k].detach().requires_grad_(True) for k in self.params]
        return x, ps

    def vjp(self, x, dy, P):
        x, ps = self._leaves(x, P)
        y = self.fn(x, *ps)
        gs = torch.autograd.grad(y, [x] + ps, dy, allow_unused=True)
        gs = [torch.zeros_like(t) if g is None else g for g, t in zip(gs, [x] + ps)]
        return gs[0], dict(zip(self.params, gs[1:]))

    def jvp2(self, x, u, dy, P):
        """(J u, dQ/dx, {theta: dQ/dtheta}) for Q = <dy, J(x) u> = <J^T dy, u>."""
        x, ps = self._leaves(x, P)
        y = self.fn(x, *ps)
        (vj,) = torch.autograd.grad(y, x, dy, create_graph=True)
        q = (vj * u).sum()
        if q.requires_grad:
            gs = torch.autograd.grad(q, [x] + ps, allow_unused=True, retain_graph=True)
        else:
            gs = [None] * (1 + len(ps))
        gs = [torch.zeros_like(t) if g is None else g.detach() for g, t in zip(gs, [x] + ps)]
        w = torch.zeros_like(y, requires_grad=True)
        (vw,) = torch.autograd.grad(y, x, w, create_graph=True)
        (ju,) = torch.autograd.grad((vw * u).sum(), w)
        return ju.detach(), gs[0], dict(zip(self.params, gs[1:]))


def _lin(x, w, b=None):
    return F.linear(x, w, b)


def gat_fn(edge_index, n):
    def f(h, att_s, att_d, bias):
        a_s = (h * att_s.view(1, -1)).sum(-1)
        a_d = (h * att_d.view(1, -1)).sum(-1)
        return pyg.gat_propagate(h, a_s, a_d, edge_index) + bias
    return f


def gnrd_fn(keep, eps=1e-5):
    def f(o, w, b, s):
        c = o - o.mean(dim=0, keepdim=True) * s
        y = w * c / (c.pow(2).mean(dim=0, keepdim=True) + eps).sqrt() + b
        y = torch.relu(y)
        return y * keep if keep is not None else y
    return f


def d_units(n_blocks: int, n_dec: int, edge_index, n: int, keeps) -> List[Unit]:
    """The discriminator's op chain (models.py:177-245) for one copy with fixed
    dropout multipliers ``keeps`` (one per encoder block)."""
    U = [Unit("mlp0", _lin, ["mlp_encoder.0.weight", "mlp_encoder.0.bias"]), Unit("relu", torch.relu, []),
         Unit("mlp2", _lin, ["mlp_encoder.2.weight", "mlp_encoder.2.bias"]), Unit("relu", torch.relu, [])]
    for b in range(n_blocks):
        m = f"encoder.module_{4 * b}"
        g = f"encoder.module_{4 * b + 1}"
        U.append(Unit(f"lin{b}", _lin, [f"{m}.lin.weight"]))
        U.append(Unit(f"gat{b}", gat_fn(edge_index, n), [f"{m}.att_src", f"{m}.att_dst", f"{m}.bias"]))
        U.append(Unit(f"gn{b}", gnrd_fn(keeps[b]), [f"{g}.weight", f"{g}.bias", f"{g}.mean_scale"]))
    for i in range(n_dec):
        U.append(Unit(f"dec{2 * i}", _lin, [f"decoder.{2 * i}.weight", f"decoder.{2 * i}.bias"]))
        if i < n_dec - 1:
            U.append(Unit("relu", torch.relu, []))
    return U


def run(units_by_copy, x0s, label_cols: slice, lam: float, P):
    """Passes A-D.  ``units_by_copy``/``x0s``: dicts over 'real', 'fake', 'mix'.
    Returns (loss, gp, grads dict)."""
    xs = {}
    for c, x0 in x0s.items():
        acts = [x0]
        for u in units_by_copy[c]:
            acts.append(u.fwd(acts[-1], P).detach())
        xs[c] = acts
    n = x0s["mix"].shape[0]
    K = len(units_by_copy["mix"])
    # B
    d = [None] * (K + 1)
    d[K] = torch.ones_like(xs["mix"][K])
    for k in range(K, 0, -1):
        d[k - 1], _ = units_by_copy["mix"][k - 1].vjp(xs["mix"][k - 1], d[k], P)
    g = d[0][:, label_cols]
    gn = g.norm(dim=1)
    gp = ((gn - 1) ** 2).mean() * lam
    eps0 = (lam * 2.0 / n) * ((gn - 1) / gn).unsqueeze(1) * g
    u = torch.zeros_like(x0s["mix"])
    u[:, label_cols] = eps0
    grads = {k: torch.zeros_like(v) for k, v in P.items()}
    # C
    inj = [None] * (K + 1)
    for k in range(1, K + 1):
        u, inj[k - 1], pg = units_by_copy["mix"][k - 1].jvp2(xs["mix"][k - 1], u, d[k], P)
        for name, t in pg.items():
            grads[name] += t
    # D
    for c, seed in (("real", -1.0 / n), ("fake", 1.0 / n), ("mix", 0.0)):
        xb = torch.full_like(xs[c][K], seed)
        for k in range(K, 0, -1):
            dx, pg = units_by_copy[c][k - 1].vjp(xs[c][k - 1], xb, P)
            for name, t in pg.items():
                grads[name] += t
            xb = dx + inj[k - 1] if c == "mix" else dx
    loss = xs["fake"][K].mean() - xs["real"][K].mean() + gp
    return loss, gp, grads


def autograd_loss(units_by_copy, x0s, label_cols: slice, lam: float, P):
    """Plain double backward of the same chain (trainer.py:291-332 structure)."""
    leaves = {k: v.detach().requires_grad_(True) for k, v in P.items()}

    def D(c, x):
        for u in units_by_copy[c]:
            x = u.fwd(x, leaves)
        return x

    d_real = D("real", x0s["real"])
    d_fake = D("fake", x0s["fake"])
    lab = x0s["mix"][:, label_cols].detach().requires_grad_(True)
    xm = torch.cat([x0s["mix"][:, :label_cols.start], lab], dim=1)
    s = D("mix", xm)
    (g,) = torch.autograd.grad(s, lab, torch.ones_like(s), create_graph=True)
    gp = ((g.norm(dim=1) - 1) ** 2).mean() * lam
    loss = d_fake.mean() - d_real.mean() + gp
    names = list(leaves)
    gs = torch.autograd.grad(loss, [leaves[k] for k in names], allow_unused=True)
    return loss.detach(), gp.detach(), {k: (torch.zeros_like(leaves[k]) if v is None else v)
                                        for k, v in zip(names, gs)}
