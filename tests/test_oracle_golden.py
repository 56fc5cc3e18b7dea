"""The CPU oracle against fixtures produced by EXECUTING the reference code.

The fixtures (tests/golden/make_golden.py) come from the reference's own
models.py / trainer.py run on the CPU; these tests pin the oracle's restatement
of the reference orchestration bit-for-bit, and cross-check the restated
torch-geometric operators against an independent dense derivation.
"""
import pytest
import torch

from oracle import dense, pyg
from oracle import reference as R
from parity_util import load_fixture, oracle_batches, tiny_config
from vgan.config import Configuration


def _run_step(name):
    f = load_fixture(name)
    cfg = Configuration(sanity_checking=(name == "step_sanity.pt"))
    if name == "step_tiny.pt":
        tiny_config(cfg)
    local, voxel = oracle_batches(f["batch"])
    G, D = R.Generator(cfg), R.Discriminator(cfg)
    G.load_state_dict(f["G0"])
    D.load_state_dict(f["D0"])
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    torch.manual_seed(int(f["step_seed"]))
    out = R.train_step(G, D, og, od, cfg, local, voxel, with_metrics=True)
    return f, out, G, D


@pytest.mark.parametrize("name", ["step_sanity.pt", "step_tiny.pt"])
def test_oracle_step_matches_reference_bitwise(name):
    f, out, G, D = _run_step(name)
    assert out["d_losses"] == f["d_losses"].tolist()
    assert out["g_loss"] == float(f["g_loss"][0])
    for k, v in f["G1"].items():
        assert torch.equal(G.state_dict()[k], v), k
    for k, v in f["D1"].items():
        assert torch.equal(D.state_dict()[k], v), k
    f1, per_graph, prec, rec, acc = out["metrics"]
    ref = f["epoch_result"].tolist()
    # the reference averages through torch.tensor(list).mean() -> float32 rounding
    assert f1 == pytest.approx(ref[2], rel=1e-6)
    assert min(per_graph) == pytest.approx(ref[3], rel=1e-12)
    assert (prec, rec, acc) == pytest.approx(tuple(ref[4:7]), abs=1e-7)


def test_oracle_forward_eval_matches_reference():
    f = load_fixture("forward_eval.pt")
    cfg = Configuration()
    local, voxel = oracle_batches(f["batch"])
    G, D = R.Generator(cfg), R.Discriminator(cfg)
    G.load_state_dict(f["G"])
    D.load_state_dict(f["D"])
    G.eval()
    D.eval()
    with torch.no_grad():
        logits, hard, soft = G(local, voxel, f["z"], noise=f["gumbel_noise"])
    assert torch.equal(logits, f["logits"])
    assert torch.equal(soft, f["label_soft"])
    assert torch.equal(hard, f["label_hard"])
    D.zero_grad()
    d_real = D(local, voxel, voxel.types_onehot.unsqueeze(0))
    d_fake = D(local, voxel, hard.unsqueeze(0))
    d_loss = d_fake.mean() - d_real.mean() + R.gradient_penalty(D, cfg, local, voxel, soft.unsqueeze(0),
                                                                 eps=f["gp_eps"])
    d_loss.backward()
    assert torch.equal(d_loss.detach(), f["d_loss"])
    for k, p in D.named_parameters():
        assert torch.equal(p.grad, f["d_grads"][k]), k


@pytest.mark.parametrize("idx", range(6))
def test_oracle_gat_matches_fixture_and_dense(idx):
    f = load_fixture("ops_small.pt")
    g = f["gat"][idx]
    _, voxel = oracle_batches(f["batch"])
    cin, cout = g["x"].shape[1], g["out"].shape[1]
    conv = pyg.GATConv(cin, cout).double()
    with torch.no_grad():
        conv.lin.weight.copy_(g["lin_weight"].double())
        conv.att_src.copy_(g["att_src"].double())
        conv.att_dst.copy_(g["att_dst"].double())
        conv.bias.copy_(g["bias"].double())
    x = g["x"].double()
    y = conv(x, voxel.edge_index)
    assert torch.allclose(y.float(), g["out"], atol=1e-6)
    yd, p = dense.gat_dense(x, conv.lin.weight, conv.att_src, conv.att_dst, conv.bias, voxel.edge_index)
    assert torch.allclose(y, yd, atol=1e-10)
    assert torch.allclose(p.sum(1), torch.ones(p.shape[0], dtype=p.dtype))


def test_oracle_graphnorm_matches_dense_and_zero_variance():
    f = load_fixture("ops_small.pt")["graphnorm"]
    gn = pyg.GraphNorm(16).double()
    with torch.no_grad():
        gn.weight.copy_(f["weight"].double())
        gn.bias.copy_(f["bias"].double())
        gn.mean_scale.copy_(f["mean_scale"].double())
    x = f["x"].double().requires_grad_(True)
    y = gn(x)
    assert torch.allclose(y.float(), f["out"], atol=1e-5)
    assert torch.allclose(y, dense.graphnorm_dense(x, gn.weight, gn.bias, gn.mean_scale), atol=1e-10)
    # a constant column: var(o) = ((1 - ms) mu)^2, finite gradients (eps inside the sqrt)
    xc = torch.randn(50, 3, dtype=torch.float64)
    xc[:, 1] = 2.5
    xc.requires_grad_(True)
    gn3 = pyg.GraphNorm(3).double()
    gn3(xc).sum().backward()
    assert torch.isfinite(xc.grad).all()
    # the published semantics: variance of o = x - ms * mu itself, eps under the
    # square root (torch_geometric 2.6.1 nn/norm/graph_norm.py); f64 gradgradcheck
    # of the oracle at mean_scale != 1 against the dense derivation's autograd
    gn4 = pyg.GraphNorm(4).double()
    with torch.no_grad():
        gn4.mean_scale.copy_(torch.tensor([0.3, 0.8, 1.0, 1.4], dtype=torch.float64))
        gn4.weight.uniform_(0.5, 1.5)
    x4 = (torch.randn(40, 4, dtype=torch.float64) * 0.2 + 0.5).requires_grad_(True)
    o = x4.detach() - x4.detach().mean(0) * gn4.mean_scale.detach()
    want = gn4.weight.detach() * o / (o.pow(2).mean(0) + 1e-5).sqrt() + gn4.bias.detach()
    assert torch.allclose(gn4(x4), want, atol=1e-12)
    params = (x4, gn4.weight, gn4.bias, gn4.mean_scale)
    dense_fn = lambda x, w, b, s: dense.graphnorm_dense(x, w, b, s)  # noqa: E731
    assert torch.autograd.gradgradcheck(dense_fn, params)
    g1 = torch.autograd.grad(gn4(x4).pow(2).sum(), params, create_graph=True)
    g2 = torch.autograd.grad(dense_fn(*params).pow(2).sum(), params, create_graph=True)
    for a, b in zip(g1, g2):
        assert torch.allclose(a, b, atol=1e-10)


def test_oracle_type_mean_fixture():
    f = load_fixture("ops_small.pt")
    local, voxel = oracle_batches(f["batch"])
    got = R.type_matched_mean(local.x, local.type, voxel.type)
    assert torch.equal(got, f["type_mean"])
    # voxels of a type with no program node (VOID = 6 never appears in programs) stay 0
    assert (got[voxel.type == 6] == 0).all()


def test_configuration_matches_reference_values():
    ref = load_fixture("step_sanity.pt")["config"]
    cfg = Configuration(sanity_checking=True)
    cfg.DATA_POINT = 4001
    mine = cfg.to_dict()
    skip = {"DATA_PATH", "GLOBAL_GRAPH_DATA_PATH", "LOCAL_GRAPH_DATA_PATH", "VOXEL_GRAPH_DATA_PATH",
            "SAVE_DATA_PATH", "LOG_DIR", "DEVICE"}
    for k, v in ref.items():
        if k in skip:
            continue
        assert k in mine, k
        assert mine[k] == v, (k, mine[k], v)


@pytest.mark.parametrize("name", ["forward_b32.pt", "forward_b32_perturbed.pt"])
def test_oracle_matches_reference_at_batch_32(name):
    """The benchmarked size (configs[1], 32 buildings, ~12.7k voxels): the
    restatement reproduces the reference-executed forward_b32.pt -- logits,
    D scores, WGAN-GP loss with its second-order D gradients, generator loss
    with its G gradients -- bit for bit; and so at the perturbed, trained-like
    parameters of forward_b32_perturbed.pt (GraphNorm mean_scale != 1, GATConv
    biases != 0)."""
    from parity_util import b32_inputs

    f = load_fixture(name)
    inp = b32_inputs(f, device=None)
    local, voxel = inp["oracle"]
    cfg = Configuration()
    torch.manual_seed(int(f["init_seed"]))
    G, D = R.Generator(cfg), R.Discriminator(cfg)
    if "G" in f:
        G.load_state_dict(f["G"])
        D.load_state_dict(f["D"])
    G.eval()
    D.eval()
    with torch.no_grad():
        logits, hard, soft = G(local, voxel, inp["z"], noise=inp["noise"])
        d_real = D(local, voxel, voxel.types_onehot.unsqueeze(0))
        d_hard = D(local, voxel, hard.unsqueeze(0))
    assert torch.equal(logits, f["logits"]) and torch.equal(soft, f["label_soft"])
    assert torch.equal(hard.argmax(1).to(torch.int8), f["label_argmax"])
    assert torch.equal(d_real, f["d_real"]) and torch.equal(d_hard, f["d_hard"])
    torch.manual_seed(int(f["gp_seed"]))  # the GP's eps = torch.rand(N, 1), trainer.py:298
    d_loss = R.discriminator_loss(D, cfg, local, voxel, hard.unsqueeze(0), soft.unsqueeze(0))
    d_loss.backward()
    assert torch.equal(d_loss.detach(), f["d_loss"])
    for k, p in D.named_parameters():
        assert torch.equal(p.grad, f["d_grads"][k]), k
    D.zero_grad()
    logits_g, hard_g, _ = G(local, voxel, inp["z"], noise=inp["noise"])
    g_loss = R.generator_loss(D, cfg, local, voxel, logits_g, hard_g.unsqueeze(0))
    g_loss.backward()
    assert torch.equal(g_loss.detach(), f["g_loss"])
    for k, p in G.named_parameters():
        assert torch.equal(p.grad, f["g_grads"][k]), k


@pytest.mark.parametrize("name,f64name", [("forward_b32.pt", "forward_b32_f64.pt"),
                                           ("forward_b32_perturbed.pt", "forward_b32_perturbed_f64.pt")])
def test_oracle_matches_f64_reference_at_batch_32(name, f64name):
    """The restatement run in f64 (the f32-initialised -- and, for the
    perturbed fixture, perturbed -- models widened, the same draws) against
    the reference's own code run in f64 (forward_b32[_perturbed]_f64.pt): the
    generator loss and every G gradient, the WGAN-GP critic loss (on the f32
    forward's labels and the f32 GP eps, as the f64 job feeds it) and every
    second-order D gradient, to f64 rounding -- the baseline
    tests/test_b32_gpu.py measures f32 errors from."""
    from parity_util import b32_inputs

    f = load_fixture(name)
    f64 = load_fixture(f64name)
    assert torch.equal(f64["batch_checksum"], f["batch_checksum"])
    inp = b32_inputs(f, device=None)
    local, voxel = inp["oracle"]
    cfg = Configuration()
    torch.manual_seed(int(f["init_seed"]))
    G, D = R.Generator(cfg), R.Discriminator(cfg)
    if "G" in f:
        G.load_state_dict(f["G"])
        D.load_state_dict(f["D"])
    G.eval()
    D.eval()
    with torch.no_grad():
        _, hard32, soft32 = G(local, voxel, inp["z"], noise=inp["noise"])
    assert torch.equal(hard32.argmax(1).to(torch.int8), f64["label_argmax_f32"])
    G, D = G.double(), D.double()
    local.x, voxel.x = local.x.double(), voxel.x.double()
    voxel.types_onehot = voxel.types_onehot.double()
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        logits, hard, _ = G(local, voxel, inp["z"].double(), noise=inp["noise"].double())
        g_loss = R.generator_loss(D, cfg, local, voxel, logits, hard.unsqueeze(0))
        g_loss.backward()
        g_grads = {k: p.grad.clone() for k, p in G.named_parameters()}
        G.zero_grad()
        D.zero_grad()
        d_real = D(local, voxel, voxel.types_onehot.unsqueeze(0))
        d_fake = D(local, voxel, hard32.double().unsqueeze(0))
        d_loss = d_fake.mean() - d_real.mean() + R.gradient_penalty(D, cfg, local, voxel,
                                                                     soft32.double().unsqueeze(0),
                                                                     eps=inp["gp_eps"].double())
        d_loss.backward()
    finally:
        torch.set_default_dtype(prev)
    assert torch.equal(hard.argmax(1).to(torch.int8), f64["label_argmax"])
    for loss, want in ((g_loss, f64["g_loss"]), (d_loss, f64["d_loss"])):
        assert abs(float(loss) - float(want)) <= 1e-12 * abs(float(want))
    for got, want_all in ((g_grads, f64["g_grads"]), ({k: p.grad for k, p in D.named_parameters()}, f64["d_grads"])):
        scale = float(torch.cat([v.reshape(-1) for v in want_all.values()]).norm())
        for k, g in got.items():
            want = want_all[k]
            assert float((g - want).norm()) <= 1e-9 * float(want.norm()) + 1e-12 * scale, k
