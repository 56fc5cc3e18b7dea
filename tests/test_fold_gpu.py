"""Deferred parameter-gradient folds: vg_fold_batch and its two-level form
vg_fold_batch_split (csrc/fold.hip), against f64 column sums."""
import ctypes

import pytest
import torch

from vgan._lib import LIB, VgFold, VgFoldSrc, check
from vgan import ops


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _folds(cuda, specs, seed):
    """specs: (rows0, rows1 or 0, width, k, accumulate); returns (descriptors, outs, expected)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    keep, outs, want = [], [], []
    arr = (VgFold * len(specs))()
    for i, (r0, r1, width, k, acc) in enumerate(specs):
        ldo = k + 3
        rows_out = (width + k - 1) // k
        out = torch.randn(rows_out, ldo, generator=g).to(cuda)
        base = out.double().clone()
        srcs = [torch.randn(r, width + 5, generator=g).to(cuda) for r in ((r0, r1) if r1 else (r0,))]
        keep += srcs
        f = arr[i]
        f.out, f.width, f.k, f.ldo, f.accumulate, f.nsrc = out.data_ptr(), width, k, ldo, acc, len(srcs)
        for j, t in enumerate(srcs):
            f.src[j] = VgFoldSrc(t.data_ptr(), t.shape[0], t.shape[1])
        tot = sum(t[:, :width].double().sum(0) for t in srcs)
        exp = base.clone()
        flat = torch.zeros(rows_out * k, dtype=torch.float64, device=cuda)
        flat[:width] = tot
        grid = flat.view(rows_out, k)
        exp[:, :k] = (exp[:, :k] if acc else 0) + grid
        outs.append(out)
        want.append(exp)
    return arr, outs, want, keep


@pytest.mark.gpu
@pytest.mark.parametrize("ws_scale", [1.0, 0.3, 0.0])
def test_fold_batch_split_matches_f64(cuda, ws_scale):
    """Short and long folds, one and two sources, narrow and wide, with and
    without accumulation, in one batch: the two-level split (long folds'
    128-row chunk sums, then their fold) and the one-level batch both equal
    the f64 column sums to f32 rounding; a workspace too small for some (or
    all) long folds leaves those in one level, still correct."""
    specs = [(100, 0, 4, 4, 1), (2717, 2717, 64, 64, 1), (1359, 1359, 32, 32, 1), (900, 0, 16, 16, 0),
             (3001, 0, 128, 64, 1), (256, 0, 4096, 64, 1), (769, 700, 8, 8, 0), (2000, 0, 1, 1, 1),
             (1191, 0, 200, 100, 1), (64, 64, 512, 512, 1)]
    st = ops.stream_handle(cuda)
    arr, outs, want, keep = _folds(cuda, specs, 5)
    need = int(LIB.vg_fold_split_ws_floats(arr, len(specs)))
    assert need > 0
    ws = torch.empty(max(1, int(need * ws_scale)), device=cuda)
    check(LIB.vg_fold_batch_split(arr, len(specs), ctypes.c_void_p(ws.data_ptr()), int(need * ws_scale), st),
          "vg_fold_batch_split")
    torch.cuda.synchronize()
    for o, w in zip(outs, want):
        assert torch.allclose(o.double(), w, rtol=1e-5, atol=1e-3), (o.double() - w).abs().max()
    arr2, outs2, want2, keep2 = _folds(cuda, specs, 5)
    check(LIB.vg_fold_batch(arr2, len(specs), st), "vg_fold_batch")
    torch.cuda.synchronize()
    for a, b in zip(outs, outs2):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-3)
    if ws_scale == 0.0:  # nothing split: the same launch as vg_fold_batch, bit for bit
        for a, b in zip(outs, outs2):
            assert torch.equal(a, b)


@pytest.mark.gpu
def test_full_fold_batch_every_workgroup_finds_its_fold(cuda):
    """VG_FOLD_MAX folds in one launch (the descriptors in the kernel
    arguments, each workgroup's fold found by binary search over block0),
    mixed sizes including one-workgroup folds between many-workgroup ones:
    every destination equals its f64 column sums, split and unsplit alone;
    one fold more is refused."""
    from vgan._lib import VG_FOLD_MAX
    shapes = [(5, 0, 4, 4, 1), (900, 300, 64, 64, 1), (40, 0, 300, 100, 0), (1300, 0, 16, 16, 1), (7, 7, 1, 1, 1)]
    specs = [shapes[i % len(shapes)] for i in range(VG_FOLD_MAX)]
    st = ops.stream_handle(cuda)
    for split in (False, True):
        arr, outs, want, keep = _folds(cuda, specs, 11)
        if split:
            need = int(LIB.vg_fold_split_ws_floats(arr, len(specs)))
            ws = torch.empty(max(1, need), device=cuda)
            check(LIB.vg_fold_batch_split(arr, len(specs), ctypes.c_void_p(ws.data_ptr()), need, st),
                  "vg_fold_batch_split")
        else:
            check(LIB.vg_fold_batch(arr, len(specs), st), "vg_fold_batch")
        torch.cuda.synchronize()
        for i, (o, w) in enumerate(zip(outs, want)):
            assert torch.allclose(o.double(), w, rtol=1e-5, atol=1e-3), (split, i, (o.double() - w).abs().max())
    big = (VgFold * (VG_FOLD_MAX + 1))()
    assert LIB.vg_fold_batch(big, VG_FOLD_MAX + 1, st) != 0
