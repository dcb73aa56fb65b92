"""Utilities: logging, timing, profiling, checkpoints."""
from .checkpoint import load_model, save_model  # noqa: F401
from .log import get_logger  # noqa: F401
from .profiling import GpuTimer, trace_mark, trace_range, tracing_enabled  # noqa: F401
