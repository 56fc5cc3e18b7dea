"""Drop-in configuration for the voxel-graph GAN path.

Mirrors the attribute surface of the reference ``Configuration``
(``building_gan/src/config.py:9-135``) so that code written against the
reference (``cfg.GENERATOR_HIDDEN_DIM``, ``cfg.N_CRITIC``, ``cfg.VOID`` ...)
keeps working unchanged.  Build-only knobs live in ``Configuration.runtime``
(a plain dict) and never shadow a reference attribute.
"""
from __future__ import annotations

import os
import random
from typing import Dict, List

import numpy as np
import torch

# program types (reference ProgramMap, config.py:9-30)
_PROGRAM_TYPES = (
    ("LOBBY_CORRIDOR", 0, "brown"),
    ("RESTROOM", 1, "red"),
    ("STAIRS", 2, "yellow"),
    ("ELEVATOR", 3, "green"),
    ("OFFICE", 4, "blue"),
    ("MECHANICAL_ROOM", 5, "orange"),
    ("VOID", 6, "gray"),
)

# feature normalisers (reference DataConfiguration, config.py:41-45)
_NORMALISERS = dict(
    NORMALIZATION_FACTOR_FLOOR_LEVEL=10,
    NORMALIZATION_FACTOR_DIMENSION=11,
    NORMALIZATION_FACTOR_LOCATION=11,
    NORMALIZATION_FACTOR_COORDINATE=42,
    NORMALIZATION_FACTOR_SITE=1600,
)

# model / optimisation hyper-parameters (reference ModelConfiguration, config.py:51-106)
_MODEL_DEFAULTS = dict(
    NUM_WORKERS=3,
    EPOCHS=5000,
    SEED=777,
    TRAIN_SPLIT_RATIO=0.65,
    VALIDATION_SPLIT_RATIO=0.25,
    TEST_SPLIT_RATIO=0.10,
    DATA_POINT=None,
    DATA_SLICER=int(1e10),
    BATCH_SIZE=512,
    N_CRITIC=5,
    LEARNING_RATE_GENERATOR=0.0002,
    LEARNING_RATE_DISCRIMINATOR=0.0002,
    LAMBDA_RATIO=0.1,
    LAMBDA_RATIO_VOID=0.1,
    LAMBDA_LABEL=0.0,
    LAMBDA_ADV=1.0,
    LAMBDA_FAR=0.1,
    LAMBDA_GP=10.0,
    BETAS=(0.5, 0.999),
    F1_SCORE_TRAIN_WEIGHT=0.05,
    F1_SCORE_VALIDATION_WEIGHT=1.0,
    METRICS_AVERAGE="macro",
    GENERATOR_CONV_TYPE="GATCONV",
    GENERATOR_ENCODER_REPEAT=7,
    GENERATOR_HIDDEN_DIM=128,
    DISCRIMINATOR_CONV_TYPE="GATCONV",
    DISCRIMINATOR_ENCODER_REPEAT=3,
    DISCRIMINATOR_HIDDEN_DIM=64,
    Z_DIM=128,
    LOCAL_GRAPH_ENCODER_REPEAT=4,
    LOCAL_ENCODER_HIDDEN_DIM=128,
    ENCODER_DROPOUT_RATE=0.2,
    GENERATOR_MLP_ENCODER_REPEAT=4,
    INPUT_ARGS="x, edge_index",
    USE_WGANGP=True,
    LOCAL_DATA_SUFFIX="_local.pt",
    VOXEL_DATA_SUFFIX="_voxel.pt",
)


class ProgramMap:
    VOID_OLD = -1
    COLORS: Dict[int, str] = {}


for _name, _idx, _color in _PROGRAM_TYPES:
    setattr(ProgramMap, _name, _idx)
    ProgramMap.COLORS[_idx] = _color
ProgramMap.NUM_CLASSES = len(_PROGRAM_TYPES)


class Configuration(ProgramMap):
    """Same attribute names and defaults as the reference configuration.

    ``Configuration(sanity_checking=True)`` reproduces ``config.py:112-117``
    (batch 1, DATA_POINT 77).  ``runtime`` holds build-side switches:

    * ``rng``: ``"device"`` (draw z / dropout / Gumbel / GP noise on the GPU)
      or ``"host"`` (draw them on the CPU default generator in the reference's
      order, then copy -- used for bit-identical parity with the CPU path).
    * ``critic``: ``"engine"`` (default; the explicit four-pass WGAN-GP
      gradient of ``vgan.critic``) or ``"autograd"`` (double backward through
      the differentiable HIP ops).
    * ``skip_dead_d_grads``: skip D's parameter gradients in the generator
      iteration (the next critic iteration zeroes them, ``trainer.py:475``).
    * ``world_size`` / ``rank``: data-parallel layout (set by ``vgan.dist``).
    * ``precision``: ``"f32"`` (default; the reference's arithmetic) or
      ``"bf16"`` (BASELINE configs[2]: every dense product -- nn.Linear and
      GATConv.lin, forward, input and weight gradients -- with bf16 operands
      and f32 accumulation; everything else f32).
    """

    _DATA_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "data"))
    DATA_PATH = os.path.join(_DATA_ROOT, "6types-raw_data")
    GLOBAL_GRAPH_DATA_PATH = os.path.join(DATA_PATH, "global_graph_data")
    LOCAL_GRAPH_DATA_PATH = os.path.join(DATA_PATH, "local_graph_data")
    VOXEL_GRAPH_DATA_PATH = os.path.join(DATA_PATH, "voxel_data")
    SAVE_DATA_PATH = os.path.join(_DATA_ROOT, "6types-processed_data")
    LOG_DIR = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "runs"))
    DEVICE = "cuda" if torch.cuda.is_available() else "cpu"

    def __init__(self, sanity_checking: bool = False):
        self.SANITY_CHECKING = sanity_checking
        self.runtime = {"rng": "device", "world_size": 1, "rank": 0, "precision": "f32"}
        if sanity_checking:
            self.BATCH_SIZE = 1
            self.DATA_SLICER = int(1e10)
            self.DATA_POINT = 77

    @property
    def SPLIT_RATIOS(self) -> List[float]:
        return [self.TRAIN_SPLIT_RATIO, self.VALIDATION_SPLIT_RATIO, self.TEST_SPLIT_RATIO]

    def to_dict(self) -> Dict[str, object]:
        """Class-level settings, like the reference (config.py:119-135 reads the
        classes' ``vars``, so per-instance overrides are not reported)."""
        out: Dict[str, object] = {}
        for klass in reversed(type(self).__mro__):
            for key, value in vars(klass).items():
                if key.startswith("_") or callable(value) or isinstance(value, (property, staticmethod)):
                    continue
                out[key] = value
        out["SPLIT_RATIOS"] = self.SPLIT_RATIOS
        return out

    @staticmethod
    def set_seed(seed: int = _MODEL_DEFAULTS["SEED"]) -> None:
        """Seed every generator the path draws from (reference config.py:137-157)."""
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(seed)
        np.random.seed(seed)
        random.seed(seed)
        Configuration.SEED = seed


for _k, _v in {**_NORMALISERS, **_MODEL_DEFAULTS}.items():
    setattr(Configuration, _k, _v)
