"""Utilities: logging, timing, profiling, checkpoints."""
