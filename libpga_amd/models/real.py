"""Real-valued (REAL encoding, f32 genes) problem family.

Benchmark functions are posed as minimisation problems f(z) with
z = M (x - o) (optional CEC-style shift o and rotation M); the engine always
maximises, so the fused score is -f.  Rotated variants evaluate M (x - o) for
a whole tile of children at once on MFMA (csrc/kernels/real.hip).

The reference examples are also here: ``SumGenes`` (test/test.cu:24-30),
``ReferenceKnapsack`` (test2/test.cu:22-36) and ``RandomKeyTSP``
(test3/test.cu:26-46).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch

from .._ext import C
from .base import Operators, Problem


def random_rotation(dim: int, seed: int = 0) -> torch.Tensor:
    """Haar-random orthogonal matrix (QR of a gaussian, sign-fixed)."""
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(dim, dim, generator=g, dtype=torch.float64)
    q, r = torch.linalg.qr(a)
    q = q * torch.sign(torch.diagonal(r)).unsqueeze(0)
    return q.to(torch.float32)


class _Benchmark(Problem):
    objective_id = 0
    default_bounds = (-5.12, 5.12)
    optimum = 0.0

    def __init__(self, dim: int = 30, *, rotate: bool = False, shift: bool = False, seed: int = 0,
                 bounds: Optional[Sequence[float]] = None):
        self.encoding = "real"
        self.length = int(dim)
        self.objective = self.objective_id
        lo, hi = bounds if bounds is not None else self.default_bounds
        self.lo, self.hi = float(lo), float(hi)
        self.rotation = random_rotation(dim, seed) if rotate else None
        if rotate and dim > 128:
            raise ValueError("rotated objectives support at most 128 dimensions")
        g = torch.Generator().manual_seed(seed + 7)
        self.shift = (torch.rand(dim, generator=g) * 1.6 - 0.8) * (self.hi - self.lo) / 2 if shift else None
        self.obj_i = (1 if shift else 0) | (2 if rotate else 0)

    def data(self):
        return self.rotation.reshape(-1) if self.rotation is not None else None

    def data2(self):
        return self.shift

    def default_operators(self) -> Operators:
        return Operators(selection="tournament", tournament_k=2, crossover="blend", blend_alpha=0.3,
                         mutation="gaussian", sigma=0.05 * (self.hi - self.lo))

    def transform(self, x: torch.Tensor) -> torch.Tensor:
        z = x.to(torch.float32)
        if self.shift is not None:
            z = z - self.shift.to(z.device)
        if self.rotation is not None:
            z = z @ self.rotation.to(z.device).T
        return z

    def f(self, z: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        return -self.f(self.transform(genomes))


class Sphere(_Benchmark):
    objective_id = C.OBJ_SPHERE

    def f(self, z):
        return (z * z).sum(-1)


class Rastrigin(_Benchmark):
    """Rastrigin; ``Rastrigin(30, rotate=True)`` is BASELINE config 3."""
    objective_id = C.OBJ_RASTRIGIN

    def f(self, z):
        return (z * z - 10.0 * torch.cos(2 * math.pi * z) + 10.0).sum(-1)


class Rosenbrock(_Benchmark):
    objective_id = C.OBJ_ROSENBROCK
    default_bounds = (-2.048, 2.048)

    def f(self, z):
        return (100.0 * (z[:, 1:] - z[:, :-1] ** 2) ** 2 + (1.0 - z[:, :-1]) ** 2).sum(-1)


class Ackley(_Benchmark):
    objective_id = C.OBJ_ACKLEY
    default_bounds = (-32.768, 32.768)

    def f(self, z):
        d = z.shape[1]
        return (-20.0 * torch.exp(-0.2 * torch.sqrt((z * z).sum(-1) / d))
                - torch.exp(torch.cos(2 * math.pi * z).sum(-1) / d) + 20.0 + math.e)


class Griewank(_Benchmark):
    objective_id = C.OBJ_GRIEWANK
    default_bounds = (-600.0, 600.0)

    def f(self, z):
        i = torch.arange(1, z.shape[1] + 1, device=z.device, dtype=torch.float32)
        return 1.0 + (z * z).sum(-1) / 4000.0 - torch.cos(z / torch.sqrt(i)).prod(-1)


class Schwefel(_Benchmark):
    objective_id = C.OBJ_SCHWEFEL
    default_bounds = (-500.0, 500.0)

    def f(self, z):
        return 418.9828872724339 * z.shape[1] - (z * torch.sin(torch.sqrt(z.abs()))).sum(-1)


class SumGenes(Problem):
    """Reference E1 "continuous OneMax": maximise the sum of genes in [0, 1]
    (test/test.cu:24-30).  Optional weights give a general linear objective."""

    def __init__(self, dim: int = 100, weights: Optional[Sequence[float]] = None):
        self.encoding = "real"
        self.length = int(dim)
        self.objective = C.OBJ_LINEAR
        self.lo, self.hi = 0.0, 1.0
        self.weights = None if weights is None else torch.as_tensor(weights, dtype=torch.float32)
        self.optimum = float(dim) if weights is None else float(self.weights.clamp(min=0).sum())

    def data(self):
        return self.weights

    def default_operators(self) -> Operators:
        # reference semantics: binary tournament, uniform crossover, 1% single-gene reset
        return Operators(selection="tournament", tournament_k=2, crossover="uniform", mutation="reset_one",
                         mutation_rate=0.01)

    def reference_fitness(self, genomes):
        g = genomes.to(torch.float32)
        return g.sum(-1) if self.weights is None else g @ self.weights.to(g.device)


class ReferenceKnapsack(Problem):
    """Reference E2 bounded knapsack: gene g encodes count = (int)(g * max_count);
    infeasible -> capacity - weight (test2/test.cu:22-36).  The default
    instance has the known optimum 285 (items 2 and 3)."""

    def __init__(self, values=(75, 150, 250, 35, 10, 100), weights=(7, 8, 6, 4, 3, 9), capacity: float = 10.0,
                 max_count: int = 2):
        self.encoding = "real"
        self.values = torch.as_tensor(values, dtype=torch.float32)
        self.weights = torch.as_tensor(weights, dtype=torch.float32)
        self.length = int(self.values.numel())
        self.objective = C.OBJ_KNAPSACK_REAL
        self.obj_i = int(max_count)
        self.obj_f0 = float(capacity)
        self.capacity = float(capacity)
        self.max_count = int(max_count)
        self.lo, self.hi = 0.0, 1.0

    def data(self):
        return torch.cat([self.values, self.weights])

    def default_operators(self) -> Operators:
        return Operators(selection="tournament", tournament_k=2, crossover="uniform", mutation="reset_one",
                         mutation_rate=0.01)

    def counts(self, genomes):
        return (genomes.to(torch.float32) * self.max_count).to(torch.int64)

    def reference_fitness(self, genomes):
        c = self.counts(genomes).to(torch.float32)
        v = c @ self.values.to(c.device)
        w = c @ self.weights.to(c.device)
        return torch.where(w <= self.capacity, v, self.capacity - w)


class RandomKeyTSP(Problem):
    """Reference E3 TSP on float genes: city_i = (int)(g_i * n); score =
    -(open path length + 10000 per duplicated ordered pair) (test3/test.cu:26-46).
    Decoded indices are clamped to n-1 (the reference can index n)."""

    def __init__(self, dist: torch.Tensor):
        self.encoding = "real"
        self.dist = torch.as_tensor(dist, dtype=torch.float32)
        n = self.dist.shape[0]
        if self.dist.shape != (n, n) or n > 256:
            raise ValueError("distance matrix must be square with n <= 256")
        self.length = n
        self.objective = C.OBJ_TSP_RANDOM_KEY
        self.lo, self.hi = 0.0, 1.0

    def data(self):
        return self.dist.reshape(-1)

    def default_operators(self) -> Operators:
        return Operators(selection="tournament", tournament_k=2, crossover="uniform", mutation="reset_one",
                         mutation_rate=0.01)

    def cities(self, genomes):
        n = self.length
        return (genomes.to(torch.float32) * n).to(torch.int64).clamp(0, n - 1)

    def reference_fitness(self, genomes):
        c = self.cities(genomes)
        d = self.dist.to(c.device)
        path = d[c[:, :-1], c[:, 1:]].sum(-1)
        eq = (c.unsqueeze(2) == c.unsqueeze(1)).sum((1, 2)) - c.shape[1]
        return -(path + 10000.0 * eq.to(torch.float32))

    @staticmethod
    def planted(n: int = 100, seed: int = 0) -> "RandomKeyTSP":
        """Reference gen.c instance: d[i][i+1] = 10, else U[10, 1010) — the path
        0 -> 1 -> ... -> n-1 (length 10 (n-1)) is planted (test3/gen.c:26-39)."""
        g = torch.Generator().manual_seed(seed)
        d = torch.randint(10, 1010, (n, n), generator=g).to(torch.float32)
        idx = torch.arange(n - 1)
        d[idx, idx + 1] = 10.0
        return RandomKeyTSP(d)


class RealTorchObjective(Problem):
    """User objective in PyTorch over decoded f32 genomes ``[N, D]``."""

    def __init__(self, dim: int, fn, bounds=(0.0, 1.0), optimum=None):
        self.encoding = "real"
        self.length = int(dim)
        self.objective = C.OBJ_NONE
        self.torch_objective = fn
        self.lo, self.hi = float(bounds[0]), float(bounds[1])
        self.optimum = optimum

    def default_operators(self) -> Operators:
        return Operators(crossover="blend", mutation="gaussian", sigma=0.05 * (self.hi - self.lo))

    def reference_fitness(self, genomes):
        return self.torch_objective(genomes).to(torch.float32)
