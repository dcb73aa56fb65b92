"""Checkpoint / resume for single islands and multi-rank island models
(SURVEY.md §5.4 — absent in the reference).

A population checkpoint is the native ``PGACKPT1`` file (csrc/engine/
island.cpp: header with S, L, encoding, generation, migration epoch, island id
and seed, then the current rows and scores).  Because the RNG is counter-based
(Philox keyed by seed, counter = (island, generation, child, stream)), the
generation counter IS the RNG state: resuming reproduces the uninterrupted run
bit for bit.

For an island model every rank writes ``<prefix>.rank<R>.ckpt`` plus rank 0
writes ``<prefix>.json`` with the model-level state (world size, topology,
migration epoch and counters).
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict

import torch.distributed as dist


def rank_path(prefix: str, rank: int) -> str:
    return f"{prefix}.rank{rank}.ckpt"


def save_model(model, prefix: str) -> None:
    """Save an ``IslandModel`` (every rank calls this)."""
    model.flush()
    model.ga.save(rank_path(prefix, model.rank))
    if model.rank == 0:
        meta: Dict[str, Any] = {
            "format": "libpga_amd.island_model.v1",
            "world": model.world,
            "topology": model.topology,
            "migrate_every": model.migrate_every,
            "k": model.k,
            "epoch": model._epoch,
            "migrations": model.migrations,
            "generation": model.ga.generation,
        }
        tmp = prefix + ".json.tmp"
        with open(tmp, "w") as f:
            json.dump(meta, f)
        os.replace(tmp, prefix + ".json")
    if model.distributed:
        dist.barrier(group=model.group)


def load_model(model, prefix: str) -> Dict[str, Any]:
    """Restore an ``IslandModel`` saved by :func:`save_model` with the same
    world size; returns the metadata."""
    with open(prefix + ".json") as f:
        meta = json.load(f)
    if meta.get("format") != "libpga_amd.island_model.v1":
        raise ValueError("not an island-model checkpoint")
    if meta["world"] != model.world or meta["k"] != model.k:
        raise ValueError(f"checkpoint has world={meta['world']} k={meta['k']}, model has world={model.world} k={model.k}")
    model.flush()
    model.ga.load(rank_path(prefix, model.rank))
    model._epoch = int(meta["epoch"])
    model.migrations = int(meta["migrations"])
    return meta
