"""Loader for the in-tree native extension ``libpga_amd/_C.so``.

The extension holds the gfx950 kernels, the native Island runtime and the CPU
reference backend.  There is deliberately NO pure-python fallback: if the
extension is missing, importing the package fails loudly with the build
command, so a GPU run can never silently execute something other than the
HIP kernels.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (loads libamdhip64 / libc10_hip before the extension)

_HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    try:
        return importlib.import_module("libpga_amd._C")
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        raise ImportError(
            "libpga_amd native extension is not built (expected "
            f"{os.path.join(_HERE, '_C.so')}). Build it with:  python tools/build.py"
        ) from e


C = load()
