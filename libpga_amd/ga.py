"""High-level single-island genetic algorithm.

    import libpga_amd as pga
    ga = pga.GeneticAlgorithm(pga.models.OneMax(1024), pop_size=1 << 20, seed=0)
    ga.run(100)
    score, genome = ga.best()

One ``GeneticAlgorithm`` = one native ``Island`` (csrc/engine/island.cpp)
resident on one device ("cuda:N" → gfx950 kernels, "cpu" → the bit-exact CPU
reference backend).  ``run(n)`` enqueues n fused generation kernels on the
current torch stream with no host synchronisation.

Reference: ``pga_init`` / ``pga_create_population`` / ``pga_run`` /
``pga_get_best`` (include/pga.h:53-143, src/pga.cu:148-236, :376-391).
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Tuple, Union

import torch

from ._ext import C
from .models.base import ENCODINGS, Operators, Problem

SELECTIONS = {"tournament": C.SEL_TOURNAMENT, "roulette": C.SEL_ROULETTE, "random": C.SEL_RANDOM, "rank": C.SEL_RANK}
CROSSOVERS = {
    "uniform": C.XO_UNIFORM, "one_point": C.XO_ONE_POINT, "two_point": C.XO_TWO_POINT, "blend": C.XO_BLEND,
    "arithmetic": C.XO_ARITHMETIC, "pmx": C.XO_PMX, "ox": C.XO_OX, "none": C.XO_NONE,
}
MUTATIONS = {
    "bit_flip": C.MUT_BIT_FLIP, "gaussian": C.MUT_GAUSSIAN, "uniform": C.MUT_UNIFORM, "reset_one": C.MUT_RESET_ONE,
    "swap": C.MUT_SWAP, "inversion": C.MUT_INVERSION, "none": C.MUT_NONE,
}


def default_device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _device_index(device: torch.device) -> int:
    if device.type == "cpu":
        return -1
    if device.type != "cuda":
        raise ValueError(f"unsupported device {device}")
    return device.index if device.index is not None else torch.cuda.current_device()


class GeneticAlgorithm:
    def __init__(
        self,
        problem: Problem,
        pop_size: int,
        *,
        operators: Optional[Operators] = None,
        seed: Optional[int] = None,
        island: int = 0,
        device: Union[str, torch.device, None] = None,
        initialize: bool = True,
        **op_overrides,
    ):
        self.problem = problem
        ops = operators or problem.default_operators()
        for k, v in op_overrides.items():
            if not hasattr(ops, k):
                raise TypeError(f"unknown operator option {k!r}")
            setattr(ops, k, v)
        self.operators = ops
        if seed is None:
            seed = int(os.environ.get("PGA_SEED", "0"))
        self.device = torch.device(device) if device is not None else default_device()
        cfg = C.Config()
        cfg.encoding = ENCODINGS[problem.encoding]
        cfg.S = int(pop_size)
        cfg.L = int(problem.length)
        cfg.lo, cfg.hi = float(problem.lo), float(problem.hi)
        cfg.objective = int(problem.objective)
        cfg.obj_i, cfg.obj_f0, cfg.obj_f1 = int(problem.obj_i), float(problem.obj_f0), float(problem.obj_f1)
        cfg.seed = int(seed) & ((1 << 64) - 1)
        cfg.island = int(island)
        self._apply_ops(cfg, ops)
        self._island = C.Island(cfg, _device_index(self.device))
        d1, d2 = problem.data(), problem.data2()
        if d1 is not None:
            self._island.set_objective_data(d1, 0)
        if d2 is not None:
            self._island.set_objective_data(d2, 1)
        # the objective the Python layer evaluates (None: native, fused or JIT)
        self.torch_objective = problem.torch_objective
        if getattr(problem, "jit_source", None) is not None:
            if self.device.type == "cuda":
                self._island.set_jit_objective(problem.kernel())
            elif getattr(problem, "fallback", None) is not None:
                self.torch_objective = problem.fallback
            else:
                raise ValueError("a JIT objective needs a GPU (or a torch `fallback` for the CPU backend)")
        if initialize:
            self.initialize()

    # ------------------------------------------------------------ config ---
    @staticmethod
    def _apply_ops(cfg, ops: Operators) -> None:
        cfg.selection = SELECTIONS[ops.selection]
        cfg.tour_k = int(ops.tournament_k)
        cfg.crossover = CROSSOVERS[ops.crossover]
        cfg.xo_prob = float(ops.crossover_prob)
        cfg.blend_alpha = float(ops.blend_alpha)
        cfg.mutation = MUTATIONS[ops.mutation]
        cfg.mut_rate = -1.0 if ops.mutation_rate is None else float(ops.mutation_rate)
        cfg.sigma = float(ops.sigma)
        cfg.rank_pressure = float(ops.rank_pressure)
        cfg.n_elite = int(ops.elitism)

    def set_operators(self, **kw) -> None:
        for k, v in kw.items():
            if not hasattr(self.operators, k):
                raise TypeError(f"unknown operator option {k!r}")
            setattr(self.operators, k, v)
        cfg = self._island.config()
        self._apply_ops(cfg, self.operators)
        self._island.set_operators(cfg)

    @property
    def island(self):
        """The native ``_C.Island`` (advanced use: parallel/, ops/)."""
        return self._island

    @property
    def pop_size(self) -> int:
        return int(self._island.config().S)

    @property
    def generation(self) -> int:
        return int(self._island.generation)

    # ------------------------------------------------------------ stages ---
    def _custom_eval(self) -> None:
        fn = self.torch_objective
        if fn is None:
            return
        genomes = self.problem.decode(self._island.rows(0))
        self._island.scores(0).copy_(fn(genomes).to(torch.float32).reshape(-1))
        self._island.rebest()

    def initialize(self) -> None:
        self._island.initialize()
        self._custom_eval()

    def evaluate(self) -> None:
        if self.torch_objective is not None:
            self._custom_eval()
        else:
            self._island.evaluate()

    def step(self) -> None:
        self.run(1)

    def run(self, generations: int, *, callback: Optional[Callable[["GeneticAlgorithm"], bool]] = None,
            target: Optional[float] = None, check_every: int = 1) -> int:
        """Run ``generations`` fused generations.  With ``target`` (or a
        callback returning True) stop early; those checks synchronise every
        ``check_every`` generations.  Returns generations executed."""
        if self.torch_objective is None and callback is None and target is None:
            self._island.run(int(generations))
            return int(generations)
        if self.torch_objective is None and callback is None:
            # native loop: one stream sync per check, none per generation
            if self.best_score() >= target:
                return 0
            return int(self._island.run_until(int(generations), float(target), max(1, int(check_every))))
        done = 0
        while done < generations:
            n = min(check_every, generations - done)
            if self.torch_objective is None:
                self._island.run(n)
            else:
                for _ in range(n):
                    self._island.run(1)
                    self._custom_eval()
                    self._island.record_history_row()  # from the evaluated scores
            done += n
            if target is not None and self.best_score() >= target:
                break
            if callback is not None and callback(self):
                break
        return done

    # ----------------------------------------------------------- queries ---
    def best_score(self) -> float:
        return float(self._island.best()[0])

    def best_index(self) -> int:
        return int(self._island.best()[1])

    def best(self) -> Tuple[float, torch.Tensor]:
        score, idx = self._island.best()
        row = self._island.row(int(idx)).unsqueeze(0)
        return float(score), self.problem.decode(row)[0]

    def top(self, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Top-k (scores, decoded genomes), best first (pga_get_best_top)."""
        idx = self._island.topk(int(k), True).to(torch.int64)
        rows = self._island.rows(0).index_select(0, idx.to(self._island.rows(0).device))
        scores = self._island.scores(0).index_select(0, idx.to(self._island.scores(0).device))
        return scores.clone(), self.problem.decode(rows)

    def stats(self) -> dict:
        mn, mx, sm, n = self._island.stats()
        return {"min": mn, "max": mx, "mean": sm / max(n, 1.0), "generation": self.generation}

    def record_history(self, on: bool = True) -> None:
        """Start (clearing) or stop the per-generation statistics history:
        every generation appends {min, max, sum, count} on the device from
        its kernel's fused partials (no pass over the scores, no sync)."""
        # a torch objective scores each generation after its kernel: its rows
        # are appended once _custom_eval has run (GeneticAlgorithm.run)
        self._island.set_history_manual(self.torch_objective is not None)
        self._island.set_stats_history(bool(on))

    def history(self) -> torch.Tensor:
        """[generations, 4] float tensor of (min, max, mean, count) rows
        recorded since record_history()."""
        h = self._island.history()
        if h.numel():
            h[:, 2] = h[:, 2] / h[:, 3].clamp(min=1.0)
        return h

    @property
    def scores(self) -> torch.Tensor:
        """Zero-copy view of the current generation's scores."""
        return self._island.scores(0)

    @property
    def rows(self) -> torch.Tensor:
        """Zero-copy int32 view [S, row_words] of the current generation."""
        return self._island.rows(0)

    def genomes(self) -> torch.Tensor:
        return self.problem.decode(self._island.rows(0))

    def synchronize(self) -> None:
        self._island.synchronize()

    # ------------------------------------------------------- checkpoints ---
    def save(self, path: str) -> None:
        self._island.save(path)

    def load(self, path: str) -> None:
        self._island.load(path)
