"""Objectives written as HIP source and compiled at runtime (hipRTC).

    p = JitObjective("binary", 1024, '''
        __device__ float f(const unsigned int* w, unsigned int nbits, const float* data) {
            float s = 0.f;
            for (unsigned int i = 0; i < (nbits + 31) / 32; ++i) s += __popc(w[i]);
            return s;
        }''', name="f")

The function sees ONE individual's row (decoded layout of the encoding):
  binary       const unsigned int*  bit-packed words, bit i of the genome =
               bit (i % 32) of word i / 32 (padding bits are zero)
  real         const float*         n genes
  permutation  const unsigned short* n city ids
plus ``data`` = the problem data tensor (float32, uploaded once; may be
None).  The engine wraps it into a batched gfx950 evaluation kernel that
runs right after every fused generation kernel (csrc/engine/jit.cpp) — a
direct, inlined call instead of the reference's device function pointer
(include/pga.h:46, src/pga.cu:250-262) or a Python/torch objective.

``fallback`` (a torch function of decoded genomes) is what the CPU backend
uses, and what tests compare the compiled objective against.
"""
from __future__ import annotations

import hashlib
from typing import Callable, Dict, Optional

import torch

from .._ext import C
from .base import ENCODINGS, Operators, Problem

_CACHE: Dict[str, object] = {}


class JitObjective(Problem):
    def __init__(self, encoding: str, length: int, source: str, *, name: str = "objective",
                 data: Optional[torch.Tensor] = None, bounds=(0.0, 1.0),
                 fallback: Optional[Callable[[torch.Tensor], torch.Tensor]] = None,
                 operators: Optional[Operators] = None, optimum: Optional[float] = None,
                 options=()):
        if encoding not in ENCODINGS:
            raise ValueError(f"encoding must be one of {sorted(ENCODINGS)}")
        self.encoding = encoding
        self.length = int(length)
        self.objective = C.OBJ_NONE
        self.lo, self.hi = float(bounds[0]), float(bounds[1])
        self.jit_source = source
        self.jit_name = name
        self.jit_options = list(options)
        self._data = None if data is None else torch.as_tensor(data, dtype=torch.float32).contiguous().cpu()
        self.fallback = fallback
        self._ops = operators
        self.optimum = optimum

    def kernel(self):
        """Compiled kernel (cached per source / encoding / name / options)."""
        key = hashlib.sha256(repr((self.encoding, self.jit_name, self.jit_source, self.jit_options)).encode()).hexdigest()
        k = _CACHE.get(key)
        if k is None:
            k = C.jit_compile(ENCODINGS[self.encoding], self.jit_source, self.jit_name, self.jit_options)
            _CACHE[key] = k
        return k

    def data(self):
        return self._data

    def default_operators(self) -> Operators:
        if self._ops is not None:
            return Operators(**vars(self._ops))
        if self.encoding == "real":
            return Operators(crossover="blend", blend_alpha=0.3, mutation="gaussian", sigma=0.05 * (self.hi - self.lo))
        if self.encoding == "permutation":
            return Operators(tournament_k=4, crossover="ox", mutation="inversion", mutation_rate=0.3)
        return Operators()

    def reference_fitness(self, genomes: torch.Tensor) -> torch.Tensor:
        if self.fallback is None:
            raise NotImplementedError("no torch fallback given")
        return self.fallback(genomes).to(torch.float32)
