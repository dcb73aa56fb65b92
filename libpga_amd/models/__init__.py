"""Problem families (the GA analogue of model architectures)."""
from .base import Operators, Problem  # noqa: F401
from .binary import BinaryTorchObjective, Knapsack01, LeadingOnes, MaxCut, OneMax, QUBO, Trap  # noqa: F401
from .real import (  # noqa: F401
    Ackley, Griewank, RandomKeyTSP, Rastrigin, RealTorchObjective, ReferenceKnapsack, Rosenbrock, Schwefel, Sphere,
    SumGenes, random_rotation,
)
from .jit import JitObjective  # noqa: F401
from .permutation import TSP, TSPEuclidean  # noqa: F401
