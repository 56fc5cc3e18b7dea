"""The launches that open a training iteration, folded into one (round 3):
vg_iter_begin (RNG counter, Adam step count, zeroed gradient) and
vg_critic_input_drawn (the gradient-penalty eps drawn inside the critic-input
kernel).  Both must reproduce the separate launches they replace bit for bit."""
import pytest
import torch

from vgan._lib import LIB, check, ptr, stream_handle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 1, 7, 63_397, 274_185])
def test_iter_begin_counts_and_zeroes(cuda, n):
    ctr = torch.tensor([41], dtype=torch.int64, device=cuda)
    step = torch.tensor([6], dtype=torch.int32, device=cuda)
    grad = torch.randn(n + 4, device=cuda)  # 4 guard elements past n
    guard = grad[n:].clone()
    check(LIB.vg_iter_begin(ptr(ctr), ptr(step), ptr(grad), n, stream_handle(cuda)), "vg_iter_begin")
    torch.cuda.synchronize()
    assert int(ctr.item()) == 42 and int(step.item()) == 7
    assert torch.count_nonzero(grad[:n]).item() == 0 and torch.equal(grad[n:], guard)
    # every pointer optional
    check(LIB.vg_iter_begin(None, ptr(step), None, 0, stream_handle(cuda)), "vg_iter_begin")
    torch.cuda.synchronize()
    assert int(step.item()) == 8
    # misaligned gradient: refused
    assert LIB.vg_iter_begin(None, None, ptr(grad[1:]), 8, stream_handle(cuda)) != 0


@pytest.mark.parametrize("n", [1, 5, 4099, 13107])
def test_critic_input_drawn_equals_rng_fill(cuda, n):
    F, K = 17, 12
    g = torch.Generator(device=cuda).manual_seed(n)
    mvx = torch.randn(n, F, device=cuda, generator=g)
    real = torch.randn(n, K, device=cuda, generator=g)
    hard = torch.randn(n, K, device=cuda, generator=g)
    soft = torch.randn(n, K, device=cuda, generator=g)
    it = torch.tensor([123], dtype=torch.int64, device=cuda)
    seed, salt = 0x1234_5678_9ABC_DEF0, 0x40000003
    st = stream_handle(cuda)
    eps = torch.empty(n, device=cuda)
    check(LIB.vg_rng_fill(ptr(eps), n, 1, seed, ptr(it), salt, st), "vg_rng_fill")
    x1 = torch.empty(4 * n, F + K, device=cuda)
    x2 = torch.full_like(x1, float("nan"))
    check(LIB.vg_critic_input(ptr(mvx), n, F, ptr(real), ptr(hard), ptr(soft), ptr(eps), K, 4, ptr(x1), st),
          "vg_critic_input")
    check(LIB.vg_critic_input_drawn(ptr(mvx), n, F, ptr(real), ptr(hard), ptr(soft), seed, ptr(it), salt, K, 4,
                                    ptr(x2), st), "vg_critic_input_drawn")
    torch.cuda.synchronize()
    assert torch.equal(x1, x2)
    assert LIB.vg_critic_input_drawn(ptr(mvx), n, F, ptr(real), ptr(hard), ptr(soft), seed, None, salt, K, 4,
                                     ptr(x2), st) != 0
