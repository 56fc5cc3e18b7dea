"""Data path on the GPU: the host collate's CSR/CSC equals csr.hip's device
build, the prefetching loader delivers device-resident batches whose CSR the
model adopts as-is, and a generator forward over such a batch is bit-identical
to one over a ``from_data_list`` batch."""
import pytest
import torch

from vgan import data, ops, store
from vgan.config import Configuration
from vgan.loader import GraphLoader
from vgan.models import VoxelGNNGenerator
from vgan.synth import SyntheticDataset

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ds_store(tmp_path_factory):
    ds = SyntheticDataset(12, seed=21)
    return ds, store.write_store(str(tmp_path_factory.mktemp("store")), ds)


def _same(a, b, what):
    assert a.dtype == b.dtype and a.shape == b.shape, what
    assert torch.equal(a, b), what


def test_host_csr_matches_device_build(cuda, ds_store):
    _, st = ds_store
    _, vox = st.collate([5, 0, 11, 3, 7, 7], pin=True)
    arrays = [t.to(cuda) for t in vox.derived("csr_arrays")]
    dev = ops.CSR(vox.edge_index.to(cuda), vox.x.shape[0])
    for name, got, want in zip(("row_ptr", "col", "csc_ptr", "csc_slot", "csc_dst"), arrays,
                               (dev.row_ptr, dev.col, dev.csc_ptr, dev.csc_slot, dev.csc_dst)):
        _same(got, want, name)


@pytest.mark.parametrize("workers", [1, 3])
def test_loader_delivers_device_batches(cuda, ds_store, workers):
    """Every batch in plan order, device-resident, equal to the reference
    collate -- with one collating thread and with three (round-robin)."""
    ds, st = ds_store
    loader = GraphLoader(st, list(range(len(st))), batch_size=5, shuffle=True, device=cuda, prefetch=2,
                         workers=workers)
    torch.manual_seed(9)
    plan = loader.batches()
    torch.manual_seed(9)  # the iteration below draws the same plan
    seen = 0
    for (loc, vox), idx in zip(loader, plan):
        ref_loc, ref_vox = ds.collate_fn([ds[i] for i in idx])
        for got, want in ((loc, ref_loc), (vox, ref_vox)):
            assert got.keys() == want.keys()
            for k in got.keys():
                g, w = getattr(got, k), getattr(want, k)
                if torch.is_tensor(g):
                    assert g.is_cuda, k
                    _same(g.cpu(), w, k)
                else:
                    assert g == w, k
        assert loc.to(cuda) is loc  # the trainer's .to(DEVICE) is a no-op
        prep = data.prepared(loc, vox, 7)
        arrays = vox.derived("csr_arrays")
        assert prep.csr.row_ptr is arrays[0]  # adopted, not rebuilt
        seen += len(idx)
    assert seen == len(st)


def test_generator_forward_identical_on_loader_batch(cuda, ds_store):
    ds, st = ds_store
    cfg = Configuration()
    torch.manual_seed(3)
    G = VoxelGNNGenerator(cfg, 17, 12).to(cuda).eval()
    idx = [4, 9, 1]
    loc_a, vox_a = (g.to(cuda) for g in ds.collate_fn([ds[i] for i in idx]))
    loc_b, vox_b = (g.to(cuda, non_blocking=True) for g in st.collate(idx, pin=True))
    n = vox_a.num_nodes
    z = torch.randn(1, n, cfg.Z_DIM, device=cuda)
    noise = torch.empty(n, 7, device=cuda).exponential_()
    with torch.no_grad():
        out_a = G(loc_a, vox_a, z, noise=noise)
        out_b = G(loc_b, vox_b, z, noise=noise)
    assert data.prepared(loc_b, vox_b, 7).csr.row_ptr is vox_b.derived("csr_arrays")[0]
    for a, b in zip(out_a, out_b):
        _same(a, b, "generator output")


def test_host_prepared_batch_equals_device_build(cuda, ds_store):
    """A batch from the loader with ``prepare``: one host-to-device copy of the
    pair's buffer, and vgan.data adopts the host-built structures -- each bit
    for bit what the device builds from the same batch (vg_type_mean, the
    float one-hot, vg_csr_ell, CSR.stacked(3) and its padded columns, the
    critic's seeds); a step on it equals a step on the device-built batch."""
    from vgan.critic import CriticEngine  # noqa: F401  (prepare_batch semantics)

    _, st = ds_store
    loader = GraphLoader(st, [2, 7, 5, 0, 9], batch_size=5, shuffle=False, device=cuda, prefetch=1, prepare=7)
    (loc, vox), = list(loader)
    blob = vox.derived("device_blob")
    assert blob is not None and loc.derived("device_blob") is blob
    prep = data.prepared(loc, vox, 7)
    v = vox.derived("prepared_arrays")["views"]
    assert prep.matched_voxel_x is v["matched_voxel_x"] and prep.consts["critic_seeds4"] is v["critic_seeds4"]
    # the same batch rebuilt on the device
    loc2 = type(loc)(**{k: (getattr(loc, k).clone() if torch.is_tensor(getattr(loc, k)) else getattr(loc, k))
                        for k in loc.keys()})
    vox2 = type(vox)(**{k: (getattr(vox, k).clone() if torch.is_tensor(getattr(vox, k)) else getattr(vox, k))
                        for k in vox.keys()})
    ref = data.prepared(loc2, vox2, 7)
    assert "critic_seeds4" not in ref.consts
    from vgan.critic import CriticEngine as CE

    CE._seeds(ref)  # the device build of prepare_batch's constants
    ref.csr.stacked(3).ell()
    _same(prep.matched_voxel_x, ref.matched_voxel_x, "type-matched mean | voxel.x")
    _same(prep.matched_x, ref.matched_x, "matched_x")
    _same(prep.onehot_f, ref.onehot_f, "onehot_f")
    _same(prep.consts["critic_seeds4"], ref.consts["critic_seeds4"], "seeds")
    for name in ("row_ptr", "col", "csc_ptr", "csc_slot", "csc_dst"):
        _same(getattr(prep.csr, name), getattr(ref.csr, name), name)
    e1, w1 = prep.csr.ell()
    e2, w2 = ref.csr.ell()
    assert w1 == w2 == 8
    _same(e1, e2, "ell")
    s1, s2 = prep.csr.stacked(3), ref.csr.stacked(3)
    for name in ("row_ptr", "col", "csc_ptr", "csc_slot", "csc_dst"):
        _same(getattr(s1, name), getattr(s2, name), "stacked " + name)
    assert s1.seg_rows == s2.seg_rows == vox.num_nodes
    _same(s1.ell()[0], s2.ell()[0], "stacked ell")
    # an in-place edit of the batch invalidates the host-built structures
    vox.x.mul_(1.0)
    assert data.prepared(loc, vox, 7).matched_voxel_x is not v["matched_voxel_x"]
