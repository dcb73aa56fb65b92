"""Several islands on ONE device, each evolving on its own HIP stream.

The single-device island model.  In the reference, up to 10
populations share a context, ``*_all`` loops run them serially and migration
is a stub (include/pga.h:44, src/pga.cu:272-276, :368-374, :393-395).  Here
the islands are independent ``GeneticAlgorithm`` objects (distinct island ids,
hence distinct Philox streams).  Same-shape BINARY islands with a built-in
integer objective run as ONE batched launch per generation (island = grid y,
Island::run_batched); other islands are enqueued on separate streams, so
small, latency-bound islands run side by side across the 256 CUs.
Every ``migrate_every`` generations the streams join on the caller's stream
and the top ``migrate_pct`` of each island replaces the worst of the next one
(ring, or a seeded random ring) with device-to-device gather/scatter kernels —
no host round trip.

The same migration protocol as the multi-GPU ``IslandModel``; the two
compose (several local islands per rank are not combined with ranks here).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from ..ga import GeneticAlgorithm
from ..models.base import Problem


def migration_policy(name: str) -> int:
    """"stripe" (default): the population is cut into k stripes; each stripe's
    best emigrates and its worst is replaced — one pass each.  "topk": the
    exact top-k emigrate and the bottom-k are replaced (two radix selections)."""
    from .._ext import C
    try:
        return {"stripe": C.MIG_STRIPE, "topk": C.MIG_TOPK}[name]
    except KeyError:
        raise ValueError("migration policy must be 'stripe' or 'topk'") from None


class LocalIslands:
    def __init__(self, problem: Problem, n_islands: int, pop_size: int, *, seed: Optional[int] = None,
                 device=None, migrate_every: int = 10, migrate_pct: float = 0.01, topology: str = "ring",
                 first_island: int = 0, policy: str = "topk", batched: bool = True, **op_overrides):
        if n_islands < 1:
            raise ValueError("n_islands must be >= 1")
        if topology not in ("ring", "random"):
            raise ValueError("topology must be 'ring' or 'random'")
        self.islands: List[GeneticAlgorithm] = [
            GeneticAlgorithm(problem, pop_size, seed=seed, island=first_island + i, device=device, **op_overrides)
            for i in range(n_islands)
        ]
        for ga in self.islands:
            ga.island.migration_policy = migration_policy(policy)
            if policy == "topk" and n_islands > 1:
                ga.island.fused_histogram = True  # exact selections without a histogram pass
        self.device = self.islands[0].device
        self.migrate_every = int(migrate_every)
        self.topology = topology
        self.seed = 0 if seed is None else int(seed)
        k = int(round(migrate_pct * pop_size))
        self.k = max(1, min(k, pop_size // 2)) if migrate_pct > 0 and n_islands > 1 else 0
        self.streams = ([torch.cuda.Stream(self.device) for _ in range(n_islands)]
                        if self.device.type == "cuda" else None)
        self.migrations = 0
        # batched launches (Island::run_batched) when the islands qualify:
        # BINARY, same shape, built-in integer objective, <= 10 islands
        self.batched = bool(batched)
        self.batched_generations = 0
        self._epoch = 0
        self._staging = {}

    @property
    def generation(self) -> int:
        return self.islands[0].generation

    def _order(self) -> List[int]:
        n = len(self.islands)
        if self.topology == "ring":
            return list(range(n))
        g = torch.Generator().manual_seed(self.seed * 1000003 + self._epoch)
        return torch.randperm(n, generator=g).tolist()

    def _evolve(self, n: int) -> None:
        if self.streams is None:
            for ga in self.islands:
                ga.run(n)
            return
        if self.batched and all(ga.torch_objective is None for ga in self.islands):
            # same-shape islands: ONE launch per generation (island = grid y)
            from .._ext import C
            if C.run_islands_batched([ga.island for ga in self.islands], int(n)):
                self.batched_generations += n
                return
        main = torch.cuda.current_stream(self.device)
        for ga, s in zip(self.islands, self.streams):
            s.wait_stream(main)
            with torch.cuda.stream(s):
                ga.run(n)
        for s in self.streams:
            main.wait_stream(s)

    def migrate(self) -> None:
        """Top-k of island order[i] replaces the worst k of order[i+1]."""
        if self.k == 0:
            return
        order = self._order()
        out = []
        for i in order:  # take every island's emigrants before any is replaced
            isl = self.islands[i].island
            if i not in self._staging:  # persistent per-island emigrant buffers
                self._staging[i] = (torch.empty(self.k * int(isl.row_words), dtype=torch.int32, device=self.device),
                                    torch.empty(self.k, dtype=torch.float32, device=self.device))
            rows, sc = self._staging[i]
            isl.emigrate(self.k, rows, sc)  # top-k selection, gather fused in
            out.append((rows, sc))
        n = len(order)
        for j, i in enumerate(order):
            dst = self.islands[order[(j + 1) % n]].island
            rows, sc = out[j]
            dst.immigrate(self.k, rows, sc)  # bottom-k selection, scatter fused in
        self._epoch += 1
        self.migrations += 1

    def run(self, generations: int) -> None:
        g = 0
        while g < generations:
            step = generations - g
            if self.migrate_every > 0:
                nxt = (self.generation // self.migrate_every + 1) * self.migrate_every
                step = min(step, nxt - self.generation)
            self._evolve(step)
            g += step
            if self.migrate_every > 0 and self.generation % self.migrate_every == 0:
                self.migrate()

    def best(self) -> Tuple[float, int, torch.Tensor]:
        """(score, island, decoded genome) of the best individual overall."""
        scores = [ga.best_score() for ga in self.islands]
        i = max(range(len(scores)), key=lambda j: scores[j])
        s, genome = self.islands[i].best()
        return s, i, genome

    def synchronize(self) -> None:
        for ga in self.islands:
            ga.synchronize()
