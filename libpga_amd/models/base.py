"""Problem (model-family) base class.

A *problem* is the GA analogue of a model architecture: it fixes the genome
encoding and length, the fused objective the native kernels evaluate, the
problem data uploaded to the device, and sensible default operators.  Every
built-in problem also carries a plain-PyTorch ``reference_fitness`` used by the
test-suite as the fp32 oracle of the fused HIP objective.

Reference: the reference has exactly one "problem" interface, a device
function pointer ``obj_f(gene*, unsigned)`` (include/pga.h:46), with examples
E1 (sum of float genes), E2 (knapsack) and E3 (TSP) in test*/test.cu.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Optional

import torch

from .._ext import C

ENCODINGS = {"binary": C.ENC_BINARY, "real": C.ENC_REAL, "permutation": C.ENC_PERMUTATION}


@dataclass
class Operators:
    selection: str = "tournament"
    tournament_k: int = 2
    crossover: str = "uniform"
    crossover_prob: float = 1.0
    blend_alpha: float = 0.5
    mutation: str = "bit_flip"
    mutation_rate: Optional[float] = None  # None: 1/L per gene, 0.01 per individual
    sigma: float = 0.1
    elitism: int = 0
    rank_pressure: float = 1.5  # selection="rank": linear ranking pressure in [1, 2]


class Problem:
    """Base class.  Subclasses set the attributes below in ``__init__``."""

    encoding: str = "binary"
    length: int = 0
    objective: int = 0  # C.OBJ_*
    obj_i: int = 0
    obj_f0: float = 0.0
    obj_f1: float = 0.0
    lo: float = 0.0
    hi: float = 1.0
    optimum: Optional[float] = None  # best achievable score, when known

    def data(self) -> Optional[torch.Tensor]:
        """Objective data slot 0 (uploaded once to the device)."""
        return None

    def data2(self) -> Optional[torch.Tensor]:
        return None

    def default_operators(self) -> Operators:
        return Operators()

    # custom (non-fused) objectives override this; it receives decoded genomes
    torch_objective: Optional[Callable[[torch.Tensor], torch.Tensor]] = None

    # ---- decoding ----
    def decode(self, rows: torch.Tensor) -> torch.Tensor:
        """rows: int32 [N, row_words] -> genomes [N, L] (bits as uint8, genes as f32/int64)."""
        from ..ops.codec import decode

        return decode(rows, self.encoding, self.length)

    def encode(self, genomes: torch.Tensor, row_words: int) -> torch.Tensor:
        from ..ops.codec import encode

        return encode(genomes, self.encoding, self.length, row_words)

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        """Plain-PyTorch fp32 fitness of decoded genomes (test oracle)."""
        raise NotImplementedError

    def describe(self) -> dict:
        return {"problem": type(self).__name__, "encoding": self.encoding, "length": self.length}
