"""libpga_amd — MI355X-native parallel genetic-algorithm engine.

Layers (bottom to top):
  csrc/kernels   hand-written gfx950 HIP kernels (fused generation, init, eval,
                 top-k, roulette prefix, migration gather/scatter)
  csrc/cpu       CPU reference backend (bit-exact for BINARY/PERMUTATION)
  csrc/engine    native Island runtime (memory, stages, checkpoint)
  csrc/capi      reference-compatible C API (include/pga.h) -> build/libpga.so
  libpga_amd     python: problems (models/), ops/, GeneticAlgorithm,
                 island model over torch.distributed/RCCL (parallel/), utils/
"""
from ._ext import C as _C  # noqa: F401  (fails loudly if the extension is missing)
from . import models, ops, parallel, utils  # noqa: F401
from .ga import GeneticAlgorithm, default_device  # noqa: F401
from .models.base import Operators, Problem  # noqa: F401

__version__ = "0.1.0"
