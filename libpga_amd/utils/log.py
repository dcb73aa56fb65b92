"""Logging with a level taken from the ``PGA_LOG`` environment variable
(debug|info|warning|error; default warning).  Rank-aware: messages carry the
torch.distributed rank when a process group is up."""
from __future__ import annotations

import logging
import os

_CONFIGURED = False


class _RankFilter(logging.Filter):
    def filter(self, record: logging.LogRecord) -> bool:
        try:
            import torch.distributed as dist

            record.rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        except Exception:  # pragma: no cover
            record.rank = 0
        return True


def get_logger(name: str) -> logging.Logger:
    global _CONFIGURED
    if not _CONFIGURED:
        level = os.environ.get("PGA_LOG", "warning").upper()
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter("[pga r%(rank)s %(levelname)s %(name)s] %(message)s"))
        h.addFilter(_RankFilter())
        root = logging.getLogger("libpga_amd")
        root.addHandler(h)
        root.setLevel(getattr(logging, level, logging.WARNING))
        root.propagate = False
        _CONFIGURED = True
    return logging.getLogger(name)
