"""vgan -- MI355X-native voxel-graph GAN training path (drop-in for building_gan.src).

Submodules importable without a GPU: ``config``, ``graph``, ``synth``, ``rng``,
``metrics``, ``dist``.  ``ops`` / ``models`` / ``trainer`` load the HIP library
``libvgan_hip.so`` and raise if it is missing (no CPU fallback).
"""
from .config import Configuration, ProgramMap  # noqa: F401
from .graph import GraphBatch, GraphData  # noqa: F401

__all__ = ["Configuration", "ProgramMap", "GraphBatch", "GraphData"]
