"""sys.modules shim so the reference's own models.py / trainer.py import here.

Used ONLY by ``tests/golden/make_golden.py`` in the build container (the
reference never travels to the GPU box).  It maps the third-party modules the
reference imports but this image lacks onto the oracle restatement or no-ops:

* ``torch_geometric.nn`` (GATConv, GraphNorm via ``.norm``, Sequential) and
  ``torch_geometric.data`` (Data, Dataset, Batch)  -> ``oracle.pyg``
* ``torch.utils.tensorboard.SummaryWriter``        -> no-op writer
* ``IPython.display.clear_output``                 -> no-op
"""
from __future__ import annotations

import importlib
import os
import sys
import types

REFERENCE_ROOT = os.environ.get("VGAN_REFERENCE_ROOT", "/root/reference")


class _NullWriter:
    def __init__(self, *args, **kwargs):
        pass

    def __getattr__(self, name):
        return lambda *a, **k: None


def install() -> None:
    from . import pyg

    tg = types.ModuleType("torch_geometric")
    tg_nn = types.ModuleType("torch_geometric.nn")
    tg_norm = types.ModuleType("torch_geometric.nn.norm")
    tg_data = types.ModuleType("torch_geometric.data")
    tg_nn.GATConv = pyg.GATConv
    tg_nn.Sequential = pyg.Sequential
    tg_nn.GraphNorm = pyg.GraphNorm
    tg_norm.GraphNorm = pyg.GraphNorm
    tg_nn.norm = tg_norm
    tg_data.Data = pyg.Data
    tg_data.Batch = pyg.Batch
    tg_data.Dataset = pyg.Dataset
    tg.nn, tg.data = tg_nn, tg_data
    sys.modules.update({
        "torch_geometric": tg,
        "torch_geometric.nn": tg_nn,
        "torch_geometric.nn.norm": tg_norm,
        "torch_geometric.data": tg_data,
    })
    if importlib.util.find_spec("IPython") is None:
        ipy = types.ModuleType("IPython")
        ipy_display = types.ModuleType("IPython.display")
        ipy_display.clear_output = lambda *a, **k: None
        ipy.display = ipy_display
        sys.modules.update({"IPython": ipy, "IPython.display": ipy_display})
    try:
        import torch.utils.tensorboard  # noqa: F401
    except Exception:
        tb = types.ModuleType("torch.utils.tensorboard")
        tb.SummaryWriter = _NullWriter
        sys.modules["torch.utils.tensorboard"] = tb
    if REFERENCE_ROOT not in sys.path:
        sys.path.insert(0, REFERENCE_ROOT)


def import_reference():
    """Return the reference modules (config, models, trainer) imported via the shim."""
    install()
    config = importlib.import_module("building_gan.src.config")
    models = importlib.import_module("building_gan.src.models")
    trainer = importlib.import_module("building_gan.src.trainer")
    return config, models, trainer
