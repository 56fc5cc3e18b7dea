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
    assert float(e.min()) >= 0 and abs(float(e.mean()) - 1) < 5e-3 and torch.isfinite(e).all()
    # odd sizes: every element written
    odd = r.normal((7, 3), cuda)
    assert torch.isfinite(odd).all() and odd.shape == (7, 3)


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
