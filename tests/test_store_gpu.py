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


def test_loader_delivers_device_batches(cuda, ds_store):
    ds, st = ds_store
    loader = GraphLoader(st, list(range(len(st))), batch_size=5, shuffle=True, device=cuda, prefetch=2)
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
