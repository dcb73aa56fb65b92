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


class QUBO(Problem):
    """Quadratic unconstrained binary optimisation: ``sign * x^T Q x``.

    ``Q`` is an ``L x L`` integer matrix with entries in [-128, 127]
    (L <= 1024).  On the GPU the population is scored on the int8 matrix
    cores (``v_mfma_i32_16x16x64_i8``, csrc/kernels/qubo.hip) with exact i32
    accumulation, so GPU and CPU scores agree bit for bit.  ``maximize=False``
    (the QUBO convention) scores ``-x^T Q x``."""

    def __init__(self, Q, maximize: bool = False):
        q = torch.as_tensor(Q)
        if q.ndim != 2 or q.shape[0] != q.shape[1]:
            raise ValueError("Q must be a square matrix")
        if q.shape[0] > 1024:
            raise ValueError("QUBO supports at most 1024 variables")
        qf = q.to(torch.float64)
        if not torch.equal(qf, qf.round()) or qf.min() < -128 or qf.max() > 127:
            raise ValueError("Q entries must be integers in [-128, 127] (int8 matrix cores)")
        self.encoding = "binary"
        self.Q = q.to(torch.float32).contiguous()
        self.length = int(q.shape[0])
        self.objective = C.OBJ_QUBO
        self.sign = 1.0 if maximize else -1.0
        self.obj_f0 = self.sign

    def data(self) -> torch.Tensor:
        return self.Q.reshape(-1)

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        g = genomes.to(torch.float64)
        q = self.Q.to(device=g.device, dtype=torch.float64)
        f = ((g @ q) * g).sum(-1)
        return (self.sign * f.to(torch.int64).to(torch.float32))

    @staticmethod
    def random(n: int, seed: int = 0, lo: int = -8, hi: int = 8, maximize: bool = False) -> "QUBO":
        gen = torch.Generator().manual_seed(seed)
        return QUBO(torch.randint(lo, hi + 1, (n, n), generator=gen), maximize=maximize)


class MaxCut(QUBO):
    """Maximum cut of an undirected graph with integer edge weights, as the
    QUBO ``cut(x) = x^T (diag(deg) - W) x`` (maximised).  Weighted degrees
    must stay within 127 (int8 diagonal)."""

    def __init__(self, W):
        w = torch.as_tensor(W).to(torch.int64)
        if w.ndim != 2 or w.shape[0] != w.shape[1] or not torch.equal(w, w.T):
            raise ValueError("W must be a symmetric square matrix")
        w = w.clone()
        w.fill_diagonal_(0)
        deg = w.sum(1)
        if deg.max() > 127 or w.min() < -128:
            raise ValueError("weighted degrees must be <= 127 for the int8 QUBO form")
        self.W = w
        super().__init__(torch.diag(deg) - w, maximize=True)

    def cut_value(self, genomes: torch.Tensor) -> torch.Tensor:
        g = genomes.to(torch.int64)
        w = self.W.to(g.device)
        diff = (g[:, :, None] != g[:, None, :]).to(torch.int64)
        return (diff * w).sum((1, 2)) // 2

    @staticmethod
    def random_graph(n: int, degree: float = 8.0, seed: int = 0) -> "MaxCut":
        gen = torch.Generator().manual_seed(seed)
        p = min(1.0, degree / max(1, n - 1))
        upper = (torch.rand(n, n, generator=gen) < p).triu(1).to(torch.int64)
        w = upper + upper.T
        over = w.sum(1) > 127
        if over.any():  # drop edges of over-full vertices (dense graphs)
            w[over] = 0
            w[:, over] = 0
        return MaxCut(w)


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
