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
