"""Device-mode draws (vg_rng_fill, counter-based Philox): distribution moments,
fresh draws when the device counter advances, identical draws for the same
(seed, counter, salt), distinct streams per seed."""
import pytest
import torch

from vgan.rng import RNG

pytestmark = pytest.mark.gpu


def test_moments(cuda):
    r = RNG("device", seed=1234)
    r.reset()
    z = r.normal((1 << 20,), cuda)
    u = r.uniform((1 << 20,), cuda)
    e = r.exponential((1 << 20,), cuda)
    assert abs(float(z.mean())) < 5e-3 and abs(float(z.std()) - 1) < 5e-3
    assert float(u.min()) >= 0 and float(u.max()) < 1 and abs(float(u.mean()) - 0.5) < 2e-3
    assert float(e.min()) > 0 and abs(float(e.mean()) - 1) < 5e-3 and torch.isfinite(e).all()
    # odd sizes: every element written
    odd = r.normal((7, 3), cuda)
    assert torch.isfinite(odd).all() and odd.shape == (7, 3)


def test_exponential_strictly_positive(cuda):
    """The Gumbel noise g = -log(E) of the label head (models.py:150) is +inf
    at E = 0, and the label softmax NaN.  The device Exp(1) draw uses 23-bit
    midpoints u' = (x + 0.5) / 2^23: E in [2^-24, 16.7) for every draw.
    2^25 draws cover each 23-bit value ~4 times (the former -log(1 - u) with
    u = 0 returned 0 once per 2^24 draws: a NaN step every ~130 steps at 16
    buildings, tools/nan_probe.py)."""
    r = RNG("device", seed=77)
    lo, hi = float("inf"), 0.0
    for _ in range(4):
        r.reset()
        e = r.exponential((1 << 23,), cuda)
        lo, hi = min(lo, float(e.min())), max(hi, float(e.max()))
        assert torch.isfinite(e).all()
    assert lo >= 2.0 ** -24 * 0.99 and hi < 16.7, (lo, hi)


def test_counter_and_seed(cuda):
    a, b = RNG("device", seed=5), RNG("device", seed=5)
    a.reset()
    b.reset()
    x1, y1 = a.normal((1000,), cuda), b.normal((1000,), cuda)
    assert torch.equal(x1, y1)  # same seed, counter and salt
    a.reset()
    assert not torch.equal(a.normal((1000,), cuda), x1)  # counter advanced
    c = RNG("device", seed=6)
    c.reset()
    assert not torch.equal(c.normal((1000,), cuda), x1)  # another seed


@pytest.mark.parametrize("C", [1, 6, 64])
def test_inkernel_dropout_without_store(cuda, C):
    """GraphNorm + ReLU + in-kernel dropout (DropSpec) in a no-grad forward
    applies the same mask without storing it (vg_graphnorm_fwd_drop with
    keep_out NULL): y is bitwise the grad-mode y, whose stored mask has the
    Bernoulli(0.8) / 0.8 values."""
    from vgan import ops

    torch.manual_seed(C)
    n = 300
    x = torch.randn(n, C, device=cuda)
    w, b, ms = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda), torch.rand(C, device=cuda)
    r = RNG("device", seed=9)
    r.reset()
    spec = r.keep_mask((n, C), 0.2, cuda)
    xg = x.clone().requires_grad_(True)
    y_grad = ops.graphnorm_relu_dropout(xg, w, b, ms, spec, 1e-5)
    with torch.no_grad():
        y_nograd = ops.graphnorm_relu_dropout(x, w, b, ms, spec, 1e-5)
    assert torch.equal(y_grad.detach(), y_nograd)
    keep = y_grad.grad_fn.saved_tensors[4]
    vals = set(torch.unique(keep).tolist())
    assert vals <= {0.0, 1.25} and 0.0 in vals and abs(float((keep > 0).float().mean()) - 0.8) < 0.08
