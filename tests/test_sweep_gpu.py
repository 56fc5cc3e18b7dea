"""configs[4]'s inference sweep over a STREAM of distinct buildings (the
reference's test loop, trainer.py:749-806, over a whole split; Gumbel tau
annealed, models.py:150): every batch comes through the native loader (host
collate + host-built per-batch structures + one upload), its stacked forward
launched eagerly (run_stream's default) or recorded as a hipGraph with an
executable graph updated in place per batch (InferenceSweep.run_fresh,
VGAN_SWEEP_STREAM=record).  The predictions equal, bit for bit, the
eager forward over the same batches from the same device-RNG state -- f16 and
f32, batches of varying size (updates and re-instantiations), back to back
with no host synchronisation."""
import pytest
import torch

from vgan.config import Configuration
from vgan.infer import InferenceSweep, geometric_taus
from vgan.loader import GraphLoader
from vgan.models import VoxelGNNGenerator
from vgan.rng import RNG
from vgan.store import write_store
from vgan.synth import SyntheticDataset

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stream", ["eager", "record"])
@pytest.mark.parametrize("dtype", ["f16", "f32"])
def test_stream_sweep_equals_eager(cuda, tmp_path, dtype, stream, monkeypatch):
    from vgan import infer

    monkeypatch.setattr(infer, "_STREAM", stream)
    st = write_store(str(tmp_path / "s"), SyntheticDataset(23, seed=17))
    cfg = Configuration()
    cfg.DEVICE = str(cuda)
    torch.manual_seed(5)
    G = VoxelGNNGenerator(cfg, 17, 12).to(cuda)
    taus = geometric_taus(1.0, 0.1, 4)

    def loader():
        return GraphLoader(st, list(range(len(st))), batch_size=5, shuffle=False, device=cuda, prefetch=2,
                           prepare=(7, ()))

    G.rng = RNG("device", seed=99)
    res = InferenceSweep(G, taus, dtype=dtype).run_stream(loader(), collect=True)
    torch.cuda.synchronize()
    assert res["batches"] == 5 and res["graphs"] == 23 and res["samples"] == 23 * len(taus)
    G.rng = RNG("device", seed=99)
    ref = InferenceSweep(G, taus, graphed=False, dtype=dtype).run(loader(), collect=True)
    torch.cuda.synchronize()
    for a, b in zip(res["predictions"], ref["predictions"]):
        assert a.shape == b.shape and torch.equal(a, b)


@pytest.mark.parametrize("copies", [1, 4])
def test_native_f16_sweep_equals_python_path(cuda, tmp_path, monkeypatch, copies):
    """The f16 sweep forward of a batch as one native call (vg_hgen_sweep,
    csrc/hgen_engine.hip) against the Python path over the same kernels
    (VGAN_HGEN_NATIVE=0): the int8 labels and the logits bit for bit, batch
    after batch from one device-RNG stream (the counter advanced in the
    engine's first launch, salts as RNG.normal / RNG.exponential), on one
    temperature and on a stacked schedule; the RNG state afterwards is the
    same."""
    from vgan import infer

    st = write_store(str(tmp_path / "s"), SyntheticDataset(17, seed=23))
    cfg = Configuration()
    cfg.DEVICE = str(cuda)
    torch.manual_seed(6)
    G = VoxelGNNGenerator(cfg, 17, 12).to(cuda)
    taus = geometric_taus(1.0, 0.1, copies)

    def run(native):
        monkeypatch.setattr(infer, "_NATIVE", native)
        G.rng = RNG("device", seed=41)
        sw = InferenceSweep(G, taus, dtype="f16")
        loader = GraphLoader(st, list(range(len(st))), batch_size=6, shuffle=False, device=cuda, prefetch=2,
                             prepare=(7, ()))
        out = sw.run_stream(loader, collect=True)["predictions"]
        torch.cuda.synchronize()
        return out, G.rng.state_dict(), G.rng._salt

    got, st_n, salt_n = run(True)
    want, st_p, salt_p = run(False)
    assert len(got) == len(want) == 3
    for a, b in zip(got, want):
        assert a.dtype == torch.int8 and a.shape == b.shape and torch.equal(a, b)
    assert st_n == st_p and salt_n == salt_p
    # the logits of one batch, native against HalfGenerator.logits from the same state
    from vgan import data as vdata
    from vgan.half import HalfGenerator

    loc, vox = next(iter(GraphLoader(st, [3, 1, 4, 1, 5], batch_size=5, shuffle=False, device=cuda, prefetch=1,
                                     prepare=(7, ()))))
    G.eval()
    hg = HalfGenerator(G)
    n = vdata.prepared(loc, vox, 7).voxel_x.shape[0]
    tt = torch.tensor(taus, device=cuda)
    G.rng = RNG("device", seed=3)
    G.rng.reset()
    lg = torch.empty(copies * n, 7, device=cuda)
    hg.sweep_labels(loc, vox, copies, tt, logits=lg)
    G.rng = RNG("device", seed=3)
    G.rng.reset()
    G.rng.reset()
    z = G.rng.normal((copies, n, cfg.Z_DIM), cuda)
    ref = hg.logits(loc, vox, z)
    torch.cuda.synchronize()
    assert torch.equal(lg, ref)


@pytest.mark.gpu
def test_graphed_native_sweep_equals_direct(cuda, tmp_path):
    """vg_hgen_sweep_graphed (the native call captured into a hipGraph, one of
    two executable graphs updated in place per batch) against vg_hgen_sweep
    launching the same kernels: labels and logits bit for bit over batches of
    varying size from one device-RNG stream, the RNG state after equal; the
    executable graphs are mostly updated in place (a batch whose shape picks
    another kernel variant re-instantiates its slot)."""
    from vgan import data as vdata
    from vgan.half import HalfGenerator

    st = write_store(str(tmp_path / "s"), SyntheticDataset(23, seed=31))
    cfg = Configuration()
    cfg.DEVICE = str(cuda)
    torch.manual_seed(9)
    G = VoxelGNNGenerator(cfg, 17, 12).to(cuda)
    G.eval()
    taus = torch.tensor(geometric_taus(1.0, 0.1, 4), device=cuda)
    plan = [[0, 1, 2], [3, 4, 5, 6, 7], [8], [9, 10, 11, 12], [13, 14], [15, 16, 17, 18, 19, 20], [21, 22]]

    def run(graph):
        G.rng = RNG("device", seed=77)
        hg = HalfGenerator(G)
        outs = []
        for idx in plan:
            loc, vox = next(iter(GraphLoader(st, idx, batch_size=len(idx), shuffle=False, device=cuda, prefetch=1,
                                             prepare=(7, ()))))
            n = vdata.prepared(loc, vox, 7).voxel_x.shape[0]
            lg = torch.empty(4 * n, 7, device=cuda)
            lab = hg.sweep_labels(loc, vox, 4, taus, logits=lg, graph=graph)
            outs.append((lab, lg))
        torch.cuda.synchronize()
        return outs, G.rng.state_dict(), hg.graph_stats()

    got, st_g, (inst, upd) = run(True)
    want, st_d, (inst_d, upd_d) = run(False)
    assert (inst_d, upd_d) == (0, 0)
    for (la, ga), (lb, gb) in zip(got, want):
        assert torch.equal(la, lb) and torch.equal(ga, gb)
    assert st_g == st_d
    assert inst + upd == len(plan) and upd >= len(plan) // 2, (inst, upd)
