"""CPU restatement of the reference models and trainer step (oracle; test-only).

Follows, module for module and in the same RNG-consumption order:

* ``VoxelGNNGenerator``   ``models.py:14-155``  (ctor ``:15-117``, forward ``:119-155``)
* ``VoxelGNNDiscriminator`` ``models.py:158-245`` (ctor ``:159-227``, forward ``:229-245``)
* gradient penalty        ``trainer.py:291-316``
* discriminator loss      ``trainer.py:318-332``
* generator loss          ``trainer.py:334-385``
* metrics                 ``trainer.py:387-443`` (sklearn, host)
* one full G+D step       ``trainer.py:459-502``

Parameter names match the reference state_dict (``matched_features_encoder.{i}``,
``mlp_encoder.{i}``, ``encoder.module_{i}.*``, ``decoder.{i}``) so state dicts
move freely between this oracle, the reference (via ``oracle.shim``) and the
HIP implementation.

Optional *injected* randomness (``noise=``) lets eval-mode parity tests feed the
same Gumbel noise to the oracle and to the GPU path; when it is omitted the
draws come from the CPU default generator exactly where the reference draws.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import pyg


def type_matched_mean(local_x, local_type, voxel_type) -> torch.Tensor:
    """models.py:122-129 -- for every voxel type present, the mean program-node
    feature of that type over the whole mini-batch (zeros if no program node)."""
    out = torch.zeros(voxel_type.shape[0], local_x.shape[1], dtype=local_x.dtype, device=local_x.device)
    for t in torch.unique(voxel_type):
        sel = local_type == t
        if sel.sum() > 0:
            out[voxel_type == t] = local_x[sel].mean(dim=0)
    return out


def _mlp_block(widths: List[int], norm: bool, act) -> nn.Sequential:
    layers: List[nn.Module] = []
    for a, b in zip(widths[:-1], widths[1:]):
        layers.append(nn.Linear(a, b))
        if norm:
            layers.append(nn.LayerNorm(b))
        layers.append(act())
    return nn.Sequential(*layers)


def gat_widths(width: int, depth: int) -> List[int]:
    """Channel schedule of the encoder (models.py:68-88): halve ``depth`` times,
    then double ``depth`` times from the bottom width."""
    chans = [width]
    for _ in range(depth):
        chans.append(chans[-1] // 2)
    for _ in range(depth):
        chans.append(chans[-1] * 2)
    return chans


def _gat_stack(width: int, depth: int, dropout: float) -> pyg.Sequential:
    entries = []
    chans = gat_widths(width, depth)
    for cin, cout in zip(chans[:-1], chans[1:]):
        entries.append((pyg.GATConv(cin, cout), "x, edge_index -> x"))
        entries.append(pyg.GraphNorm(cout))
        entries.append(nn.ReLU(True))
        entries.append(nn.Dropout(dropout))
    return pyg.Sequential("x, edge_index", entries)


class Generator(nn.Module):
    def __init__(self, cfg, local_dim: int = 17, voxel_dim: int = 12):
        super().__init__()
        hid_l, hid_g, zdim = cfg.LOCAL_ENCODER_HIDDEN_DIM, cfg.GENERATOR_HIDDEN_DIM, cfg.Z_DIM
        lrelu = lambda: nn.LeakyReLU(0.2)  # noqa: E731
        self.matched_features_encoder = _mlp_block(
            [local_dim] + [hid_l] * (cfg.LOCAL_GRAPH_ENCODER_REPEAT + 1), True, lrelu)
        self.mlp_encoder = _mlp_block(
            [hid_l + voxel_dim + zdim] + [hid_g] * (cfg.GENERATOR_MLP_ENCODER_REPEAT + 1), True, lrelu)
        self.encoder = _gat_stack(hid_g, cfg.GENERATOR_ENCODER_REPEAT, 0.2)
        dec_in = hid_l + voxel_dim + zdim + gat_widths(hid_g, cfg.GENERATOR_ENCODER_REPEAT)[-1] + hid_g
        widths = [dec_in, hid_g, hid_g // 2, hid_g // 4, hid_g // 8]
        dec = list(_mlp_block(widths, True, lrelu).children())
        dec.append(nn.Linear(hid_g // 8, cfg.NUM_CLASSES))
        self.decoder = nn.Sequential(*dec)

    def forward(self, local_graph, voxel_graph, z, noise: Optional[torch.Tensor] = None):
        matched = type_matched_mean(local_graph.x, local_graph.type, voxel_graph.type)
        em = self.matched_features_encoder(matched)
        zz = z.squeeze(0)
        x = self.mlp_encoder(torch.cat([em, voxel_graph.x, zz], dim=-1))
        enc = self.encoder(x, voxel_graph.edge_index)
        logits = self.decoder(torch.cat([enc, x, em, voxel_graph.x, zz], dim=-1))
        # F.gumbel_softmax(logits, tau=1.0, hard=False) with the same draw
        if noise is None:
            noise = torch.empty_like(logits, memory_format=torch.legacy_contiguous_format).exponential_()
        soft = ((logits - noise.log()) / 1.0).softmax(-1)
        hard = torch.zeros_like(soft).scatter_(-1, soft.argmax(dim=1, keepdim=True), 1.0)
        hard = hard - soft.detach() + soft
        return logits, hard, soft


class Discriminator(nn.Module):
    def __init__(self, cfg, local_dim: int = 17, voxel_dim: int = 12):
        super().__init__()
        hid = cfg.DISCRIMINATOR_HIDDEN_DIM
        self.mlp_encoder = _mlp_block([local_dim + voxel_dim + cfg.NUM_CLASSES, hid, hid], False,
                                      lambda: nn.ReLU(True))
        self.encoder = _gat_stack(hid, cfg.DISCRIMINATOR_ENCODER_REPEAT, 0.2)
        dec = list(_mlp_block([hid, hid // 2, hid // 4, hid // 8], False, lambda: nn.ReLU(True)).children())
        dec.append(nn.Linear(hid // 8, 1))
        if not cfg.USE_WGANGP:
            dec.append(nn.Sigmoid())
        self.decoder = nn.Sequential(*dec)

    def forward(self, local_graph, voxel_graph, label):
        matched = type_matched_mean(local_graph.x, local_graph.type, voxel_graph.type)
        feats = torch.cat([matched, voxel_graph.x, label.squeeze(0)], dim=-1)
        return self.decoder(self.encoder(self.mlp_encoder(feats), voxel_graph.edge_index))


# --------------------------------------------------------------------- losses
def gradient_penalty(D, cfg, local_graph, voxel_graph, label_soft, eps: Optional[torch.Tensor] = None):
    """trainer.py:291-316 (eps drawn with torch.rand(N, 1) on the CPU generator)."""
    if eps is None:
        eps = torch.rand(voxel_graph.types_onehot.shape[0], 1)
    mix = (eps * voxel_graph.types_onehot + (1 - eps) * label_soft.squeeze(0)).requires_grad_(True)
    score = D(local_graph, voxel_graph, mix.unsqueeze(0))
    (grad,) = torch.autograd.grad(score, mix, torch.ones_like(score), create_graph=True, only_inputs=True)
    return ((grad.norm(dim=1) - 1) ** 2).mean() * cfg.LAMBDA_GP


def discriminator_loss(D, cfg, local_graph, voxel_graph, label_hard, label_soft):
    d_real = D(local_graph, voxel_graph, voxel_graph.types_onehot.unsqueeze(0))
    d_fake = D(local_graph, voxel_graph, label_hard)
    if cfg.USE_WGANGP:
        return d_fake.mean() - d_real.mean() + gradient_penalty(D, cfg, local_graph, voxel_graph, label_soft)
    return (F.binary_cross_entropy(d_fake, torch.zeros_like(d_fake))
            + F.binary_cross_entropy(d_real, torch.ones_like(d_real)))


def far_pairs(cfg, voxel_graph, label_hard):
    """Per-building (FAR, generated FAR) -- trainer.py:357-378."""
    pred = label_hard.squeeze(0).argmax(dim=1)
    target, generated = [], []
    lo = 0
    for gi in range(voxel_graph.num_graphs):
        g = voxel_graph[gi]
        hi = lo + g.num_nodes
        dims = g.x[:, 3:6] * cfg.NORMALIZATION_FACTOR_DIMENSION
        used = dims[pred[lo:hi] != cfg.VOID]
        generated.append((used[:, 1] * used[:, 2]).sum() / g.site_area[0])
        target.append(g.x[0][9])
        lo = hi
    return torch.tensor(generated), torch.tensor(target)


def generator_loss(D, cfg, local_graph, voxel_graph, logits, label_hard):
    """trainer.py:334-385."""
    d_fake = D(local_graph, voxel_graph, label_hard)
    if cfg.USE_WGANGP:
        adv = -d_fake.mean()
    else:
        adv = F.binary_cross_entropy(d_fake, torch.ones_like(d_fake))
    adv = adv * cfg.LAMBDA_ADV
    ce = F.cross_entropy(logits, voxel_graph.type) * cfg.LAMBDA_LABEL
    n = voxel_graph.num_nodes
    ratio_gen = label_hard.squeeze(0).sum(dim=0) / n
    ratio_ref = voxel_graph.types_onehot.sum(dim=0) / n
    ratio = F.mse_loss(ratio_gen[:-2], ratio_ref[:-2]) * cfg.LAMBDA_RATIO
    ratio_void = F.mse_loss(ratio_gen[-2:], ratio_ref[-2:]) * cfg.LAMBDA_RATIO_VOID
    gen_far, ref_far = far_pairs(cfg, voxel_graph, label_hard)
    far = F.mse_loss(gen_far, ref_far) * cfg.LAMBDA_FAR
    return adv + ratio + ce + ratio_void + far


def metrics(cfg, voxel_graph, label_hard):
    """trainer.py:387-443 (sklearn macro scores + per-building F1)."""
    from sklearn import metrics as skm

    truth = voxel_graph.type.cpu()
    pred = label_hard.squeeze(0).argmax(dim=1).cpu()
    avg = cfg.METRICS_AVERAGE
    f1 = skm.f1_score(truth, pred, average=avg, zero_division=0)
    prec = skm.precision_score(truth, pred, average=avg, zero_division=0)
    rec = skm.recall_score(truth, pred, average=avg, zero_division=0)
    acc = skm.accuracy_score(truth, pred)
    per_graph = []
    lo = 0
    for gi in range(voxel_graph.num_graphs):
        hi = lo + voxel_graph[gi].num_nodes
        per_graph.append(skm.f1_score(truth[lo:hi], pred[lo:hi], average=avg, zero_division=0))
        lo = hi
    return f1, per_graph, prec, rec, acc


def train_step(G, D, opt_g, opt_d, cfg, local_graph, voxel_graph, with_metrics: bool = False) -> Dict:
    """One full G+D step, trainer.py:467-502, CPU generator order preserved."""
    d_losses = []
    for _ in range(cfg.N_CRITIC):
        with torch.no_grad():
            z = torch.randn(1, voxel_graph.num_nodes, cfg.Z_DIM)
            _, hard, soft = G(local_graph, voxel_graph, z)
            hard, soft = hard.unsqueeze(0), soft.unsqueeze(0)
        opt_d.zero_grad()
        d_loss = discriminator_loss(D, cfg, local_graph, voxel_graph, hard, soft)
        d_loss.backward()
        d_losses.append(d_loss.item())
        opt_d.step()
    z = torch.randn(1, voxel_graph.num_nodes, cfg.Z_DIM)
    logits, hard, soft = G(local_graph, voxel_graph, z)
    hard, soft = hard.unsqueeze(0), soft.unsqueeze(0)
    opt_g.zero_grad()
    g_loss = generator_loss(D, cfg, local_graph, voxel_graph, logits, hard)
    g_loss.backward()
    out = {"d_losses": d_losses, "g_loss": g_loss.item(), "label_hard": hard.detach()}
    opt_g.step()
    if with_metrics:
        out["metrics"] = metrics(cfg, voxel_graph, hard)
    return out
