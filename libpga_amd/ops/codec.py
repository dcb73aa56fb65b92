"""Genome row codecs (pure torch, device-agnostic).

Row layout (shared with the kernels, csrc/include/pga/core.hpp):
  BINARY       bit b of the genome = bit (b % 32) of int32 word b // 32
  REAL         gene g = float32 word g
  PERMUTATION  gene g = uint16 half-word g (little endian)
Rows are padded to a multiple of 4 words (16 bytes); padding is zero.
"""
from __future__ import annotations

import torch


def decode(rows: torch.Tensor, encoding: str, length: int) -> torch.Tensor:
    if rows.dtype != torch.int32:
        raise TypeError("rows must be int32")
    if encoding == "binary":
        w = rows[:, : (length + 31) // 32].to(torch.int64) & 0xFFFFFFFF
        shifts = torch.arange(32, device=rows.device, dtype=torch.int64)
        bits = (w.unsqueeze(-1) >> shifts) & 1
        return bits.reshape(rows.shape[0], -1)[:, :length].to(torch.uint8)
    if encoding == "real":
        return rows.view(torch.float32)[:, :length]
    if encoding == "permutation":
        h = rows.contiguous().view(torch.int16)[:, :length]
        return h.to(torch.int64) & 0xFFFF
    raise ValueError(encoding)


def encode(genomes: torch.Tensor, encoding: str, length: int, row_words: int) -> torch.Tensor:
    n = genomes.shape[0]
    out = torch.zeros((n, row_words), dtype=torch.int32, device=genomes.device)
    if encoding == "binary":
        g = genomes.to(torch.int64)
        nw = (length + 31) // 32
        pad = nw * 32 - length
        if pad:
            g = torch.cat([g, torch.zeros((n, pad), dtype=torch.int64, device=g.device)], 1)
        g = g.reshape(n, nw, 32)
        shifts = torch.arange(32, device=g.device, dtype=torch.int64)
        w = (g << shifts).sum(-1)
        w = torch.where(w >= 2**31, w - 2**32, w)
        out[:, :nw] = w.to(torch.int32)
        return out
    if encoding == "real":
        out.view(torch.float32)[:, :length] = genomes.to(torch.float32)
        return out
    if encoding == "permutation":
        h = genomes.to(torch.int64)
        h = torch.where(h >= 2**15, h - 2**16, h).to(torch.int16)
        out.view(torch.int16)[:, :length] = h
        return out
    raise ValueError(encoding)
