"""Permutation (PERMUTATION encoding, u16 city ids) problem family: TSP.

BASELINE config 5 ("TSP-256 permutation encoding (ordered/PMX crossover)").
Crossover PMX / OX1 and swap / inversion (2-opt) mutation run in the fused
kernel (csrc/kernels/perm.hip).
"""
from __future__ import annotations

import torch

from .._ext import C
from .base import Operators, Problem


class TSP(Problem):
    """Closed-tour TSP over a distance matrix (score = -tour length).
    ``open_path=True`` scores the open path (the reference E3 metric,
    test3/test.cu:30-34, without its duplicate penalty: tours are valid
    permutations by construction)."""

    def __init__(self, dist: torch.Tensor, open_path: bool = False):
        self.encoding = "permutation"
        self.dist = torch.as_tensor(dist, dtype=torch.float32)
        n = self.dist.shape[0]
        if self.dist.shape != (n, n):
            raise ValueError("distance matrix must be square")
        if n > 65535:
            raise ValueError("at most 65535 cities (u16 ids); on the GPU at most ~20400 (LDS-resident crossover)")
        self.length = n
        self.open_path = open_path
        self.objective = C.OBJ_TSP_OPEN if open_path else C.OBJ_TSP

    def data(self):
        return self.dist.reshape(-1)

    def default_operators(self) -> Operators:
        return Operators(selection="tournament", tournament_k=4, crossover="ox", mutation="inversion",
                         mutation_rate=0.3)

    def tour_length(self, tours: torch.Tensor) -> torch.Tensor:
        t = tours.to(torch.int64)
        d = self.dist.to(t.device)
        nxt = t[:, 1:] if self.open_path else torch.roll(t, -1, dims=1)
        cur = t[:, :-1] if self.open_path else t
        return d[cur, nxt].sum(-1)

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        return -self.tour_length(genomes)

    @staticmethod
    def random_integer_euclidean(n: int, seed: int = 0, scale: float = 1000.0, open_path: bool = False) -> "TSP":
        """Integer Euclidean instance (TSPLIB EUC_2D: nint of the distance of
        cities placed uniformly in [0, scale)^2): symmetric, integer-valued,
        so the GPU evaluates tours from a u16 copy of the matrix in LDS."""
        g = torch.Generator().manual_seed(seed)
        xy = torch.rand(n, 2, generator=g, dtype=torch.float64) * scale
        return TSP(torch.round(torch.cdist(xy, xy)).float(), open_path=open_path)

    @staticmethod
    def reference_e3(n: int = 100, seed: int = 0) -> "TSP":
        """The reference's E3 instance family (test3/gen.c:26-39): d[i][i+1] =
        10, every other entry uniform in [10, 1009] (asymmetric, integer), so
        the path 0 -> 1 -> ... -> n-1 of length 10 (n - 1) is planted.  The
        reference scores the open path (test3/test.cu:30-34)."""
        g = torch.Generator().manual_seed(seed)
        d = torch.randint(10, 1010, (n, n), generator=g).float()
        i = torch.arange(n - 1)
        d[i, i + 1] = 10.0
        return TSP(d, open_path=True)

    @staticmethod
    def random_euclidean(n: int, seed: int = 0, open_path: bool = False) -> "TSP":
        g = torch.Generator().manual_seed(seed)
        xy = torch.rand(n, 2, generator=g) * 1000.0
        return TSP(torch.cdist(xy.double(), xy.double()).float(), open_path=open_path)


class TSPEuclidean(Problem):
    """Closed-tour Euclidean TSP from city coordinates (staged in LDS; no
    distance matrix traffic)."""

    def __init__(self, coords: torch.Tensor):
        self.encoding = "permutation"
        self.coords = torch.as_tensor(coords, dtype=torch.float32)
        if self.coords.ndim != 2 or self.coords.shape[1] != 2:
            raise ValueError("coords must be [n, 2]")
        self.length = int(self.coords.shape[0])
        if self.length > 65535:
            raise ValueError("at most 65535 cities (u16 ids); on the GPU at most ~10200 (LDS-resident crossover)")
        self.objective = C.OBJ_TSP_EUC

    def data(self):
        return self.coords.reshape(-1)

    def default_operators(self) -> Operators:
        return Operators(selection="tournament", tournament_k=4, crossover="ox", mutation="inversion",
                         mutation_rate=0.3)

    def tour_length(self, tours: torch.Tensor) -> torch.Tensor:
        t = tours.to(torch.int64)
        c = self.coords.to(t.device)
        a, b = c[t], c[torch.roll(t, -1, dims=1)]
        return torch.sqrt(((a - b) ** 2).sum(-1)).sum(-1)

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        return -self.tour_length(genomes)

    @staticmethod
    def random(n: int, seed: int = 0) -> "TSPEuclidean":
        g = torch.Generator().manual_seed(seed)
        return TSPEuclidean(torch.rand(n, 2, generator=g) * 1000.0)

    @staticmethod
    def circle(n: int) -> "TSPEuclidean":
        """Cities on a circle: the optimal tour (length ~ 2 pi r) is known."""
        th = torch.arange(n, dtype=torch.float64) * (2 * torch.pi / n)
        return TSPEuclidean(torch.stack([500 + 400 * torch.cos(th), 500 + 400 * torch.sin(th)], 1).float())
