"""Island models: across GPUs over torch.distributed (RCCL over xGMI) and
across HIP streams on one GPU."""
from .islands import IslandModel, init_distributed, migrants_for  # noqa: F401
from .local import LocalIslands  # noqa: F401
