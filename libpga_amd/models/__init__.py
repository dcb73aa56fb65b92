"""Problem families (the GA analogue of model architectures)."""
from .base import Operators, Problem  # noqa: F401
from .binary import BinaryTorchObjective, Knapsack01, LeadingOnes, OneMax, Trap  # noqa: F401
