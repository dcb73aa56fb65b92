"""Bit-string (BINARY encoding) problem family.

All objectives are fused into the generation kernel (csrc/kernels/binary.hip);
``reference_fitness`` is the plain-PyTorch fp32 oracle used by the tests.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .._ext import C
from .base import Operators, Problem


class OneMax(Problem):
    """Maximise the number of one bits (headline benchmark: L = 1024).

    The bit-packed analogue of the reference's "continuous OneMax" example
    (test/test.cu:24-30, sum of float genes)."""

    def __init__(self, length: int = 1024):
        self.encoding = "binary"
        self.length = int(length)
        self.objective = C.OBJ_ONEMAX
        self.optimum = float(length)

    def default_operators(self) -> Operators:
        return Operators(selection="tournament", tournament_k=2, crossover="uniform", mutation="bit_flip")

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        return genomes.to(torch.float32).sum(-1)


class Knapsack01(Problem):
    """0/1 knapsack; infeasible solutions score ``capacity - weight`` (< 0),
    the penalty of the reference's knapsack example (test2/test.cu:35)."""

    def __init__(self, values: Sequence[float], weights: Sequence[float], capacity: float):
        self.encoding = "binary"
        self.values = torch.as_tensor(values, dtype=torch.float32)
        self.weights = torch.as_tensor(weights, dtype=torch.float32)
        if self.values.shape != self.weights.shape or self.values.ndim != 1:
            raise ValueError("values and weights must be 1-D of equal length")
        self.length = int(self.values.numel())
        self.capacity = float(capacity)
        self.objective = C.OBJ_KNAPSACK
        self.obj_f0 = self.capacity

    def data(self) -> torch.Tensor:
        return torch.cat([self.values, self.weights])

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        g = genomes.to(torch.float32)
        v = g @ self.values.to(g.device)
        w = g @ self.weights.to(g.device)
        return torch.where(w <= self.capacity, v, self.capacity - w)

    @staticmethod
    def random(n: int, seed: int = 0, capacity_ratio: float = 0.5) -> "Knapsack01":
        gen = torch.Generator().manual_seed(seed)
        v = torch.randint(1, 100, (n,), generator=gen).float()
        w = torch.randint(1, 100, (n,), generator=gen).float()
        return Knapsack01(v, w, float(w.sum()) * capacity_ratio)


class Trap(Problem):
    """Concatenated deceptive trap functions of order k (k in {2,4,8,16,32}).

    Each k-bit block with u ones scores k if u == k else k - 1 - u."""

    def __init__(self, length: int = 1024, k: int = 4):
        if k not in (2, 4, 8, 16, 32):
            raise ValueError("trap order must divide 32")
        if length % k:
            raise ValueError("length must be a multiple of the trap order")
        self.encoding = "binary"
        self.length = int(length)
        self.k = int(k)
        self.objective = C.OBJ_TRAP
        self.obj_i = self.k
        self.optimum = float(length)

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        u = genomes.to(torch.int64).reshape(genomes.shape[0], -1, self.k).sum(-1)
        f = torch.where(u == self.k, torch.full_like(u, self.k), self.k - 1 - u)
        return f.sum(-1).to(torch.float32)


class LeadingOnes(Problem):
    """Number of consecutive one bits from bit 0."""

    def __init__(self, length: int = 256):
        self.encoding = "binary"
        self.length = int(length)
        self.objective = C.OBJ_LEADING_ONES
        self.optimum = float(length)

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        g = genomes.to(torch.int64)
        zeros = (g == 0).to(torch.int64)
        idx = torch.arange(g.shape[1], device=g.device).expand_as(g)
        first0 = torch.where(zeros.bool(), idx, torch.full_like(idx, g.shape[1])).min(-1).values
        return first0.to(torch.float32)


class BinaryTorchObjective(Problem):
    """User objective written in PyTorch over decoded bit genomes ``[N, L]``.

    Selection/crossover/mutation still run in the fused HIP kernel; the
    objective is evaluated by ``fn`` once per generation (vectorised over the
    whole population)."""

    def __init__(self, length: int, fn, optimum: Optional[float] = None):
        self.encoding = "binary"
        self.length = int(length)
        self.objective = C.OBJ_NONE
        self.torch_objective = fn
        self.optimum = optimum

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        return self.torch_objective(genomes).to(torch.float32)
