"""Multi-GPU island model over torch.distributed (RCCL over xGMI)."""
from .islands import IslandModel, init_distributed, migrants_for  # noqa: F401
