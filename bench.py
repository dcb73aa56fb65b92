#!/usr/bin/env python3
"""Headline benchmark: generations/sec + evals/sec of the BASELINE configs.

Default (the driver's headline, BASELINE.json "metric"): one island of
pop=1M OneMax-1024 (bit-packed, tournament-2, uniform crossover, bit-flip
1/L, elitism 1) per GPU.  ``--problem`` selects the other multi-GPU BASELINE
configs under the same launcher:

  onemax           OneMax 1024-bit, pop=1M per GPU (configs 2 and 4)
  tsp256           TSP-256 permutation, pop=256K per GPU, --crossover ox|pmx
                   (config 5; symmetric f32 distance matrix of 256 random cities)
  rastrigin30      Rastrigin-30D float, pop=1M per GPU
  rastrigin30_rot  rotated Rastrigin-30D, fitness through MFMA tiles (config 3)

With N>1 GPUs the islands exchange their top 1% every 10 generations over
RCCL (ring), so the per-GPU work is fixed as N grows (weak scaling).  A
"step" is one generation of every island, fused selection + crossover +
mutation + evaluation included; migrations that fall in the timed window are
timed too.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--problem P]
    torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

Prints ONE JSON line (rank 0): value = total evals/s over all GPUs.  The line
also says how the islands migrated (transport, rccl_ranks, timed vs expected
migrations, degraded, failures); a run whose migration degraded or fell short
exits non-zero, so a number measured without migration can never pass as a
weak-scaling result.
Data: random-init population of the named architecture (synthetic; the GA has
no dataset).  The reference publishes no numbers, so
vs_baseline compares against the measured reference-semantics re-creation
(bench/refsem.hip) on the same hardware, times the GPU count.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import libpga_amd as pga  # noqa: E402
from libpga_amd.parallel import IslandModel, init_distributed  # noqa: E402

METRIC = "generations/sec + evals/sec, OneMax pop=1M 1024-bit, 1/2/4/8 MI355X"
# The reference publishes no numbers.  The comparison point is
# its execution structure re-created on the same MI355X (bench/refsem.hip,
# profiles/reference_semantics.jsonl), in evals/s on one GPU, scaled by the
# GPU count (perfect scaling credited to the reference, which has no
# multi-GPU code at all).  OneMax-1024 pop=1M: 1.91 gens/s; Rastrigin-30D
# pop=1M: 19.2 gens/s; TSP has no reference-semantics run (null).
REFSEM_EVALS_PER_SEC_PER_GPU = {"onemax": 2.00086e6, "rastrigin30": 19.2 * (1 << 20)}

PROBLEMS = ("onemax", "tsp256", "rastrigin30", "rastrigin30_rot")


def make_problem(name: str, length: int):
    """(problem, default pop per GPU, operator overrides, model label)."""
    M = pga.models
    if name == "onemax":
        return M.OneMax(length), 1 << 20, dict(selection="tournament", tournament_k=2, crossover="uniform",
                                               mutation="bit_flip"), f"OneMax-{length}bit"
    if name == "tsp256":
        # bench/bench_configs.py tsp256_*: 256 uniform random cities (seed 7),
        # exact pairwise distances (symmetric f32 matrix, zero diagonal)
        g = torch.Generator().manual_seed(7)
        xy = torch.rand(256, 2, generator=g)
        d = torch.cdist(xy, xy, compute_mode="donot_use_mm_for_euclid_dist")
        return M.TSP(d), 1 << 18, {}, "TSP-256"
    if name == "rastrigin30":
        return M.Rastrigin(30), 1 << 20, {}, "Rastrigin-30D"
    if name == "rastrigin30_rot":
        return M.Rastrigin(30, rotate=True, seed=1), 1 << 20, {}, "Rastrigin-30D-rotated"
    raise ValueError(name)


def expected_migrations(g0: int, steps: int, every: int) -> int:
    """Exchanges IslandModel.run starts in generations [g0, g0 + steps): one
    at every generation g > 0 with g % every == 0 (each completes one
    generation later, inside the window: run() and flush() leave none open)."""
    if every <= 0:
        return 0
    return sum(1 for g in range(g0, g0 + steps) if g > 0 and g % every == 0)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--problem", default="onemax", choices=PROBLEMS)
    ap.add_argument("--crossover", default=None, help="tsp256: ox (default) or pmx; others: the problem's default")
    ap.add_argument("--pop", type=int, default=None, help="population per GPU (default: the config's)")
    ap.add_argument("--length", type=int, default=1024, help="onemax chromosome bits")
    ap.add_argument("--migrate-every", type=int, default=10)
    ap.add_argument("--migrate-pct", type=float, default=0.01)
    ap.add_argument("--topology", default="ring")
    ap.add_argument("--transport", default="auto", choices=("auto", "engine", "torch"))
    ap.add_argument("--elitism", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--timeout-s", type=float, default=120.0, help="per-exchange deadline (degrades, never hangs)")
    ap.add_argument("--cpu", action="store_true", help="CPU reference backend (plumbing check)")
    ap.add_argument("--rccl-self", action="store_true",
                    help="one GPU, no torchrun: the island migrates with itself over a 1-rank RCCL communicator "
                         "(the per-GPU migration cost of an N-GPU run, minus the xGMI wire)")
    a = ap.parse_args()

    rank, world, device = init_distributed("gloo" if a.cpu else None)
    if a.rccl_self:
        if world != 1 or a.cpu:
            ap.error("--rccl-self runs one GPU process without torchrun")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=device)
    if a.cpu:
        device = torch.device("cpu")
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    problem, pop_default, ops, label = make_problem(a.problem, a.length)
    pop = a.pop or pop_default
    if a.crossover:
        if a.problem == "tsp256" and a.crossover not in ("ox", "pmx"):
            ap.error("tsp256 takes --crossover ox or pmx")
        ops["crossover"] = a.crossover
    ga = pga.GeneticAlgorithm(problem, pop, seed=a.seed, island=rank, device=device, elitism=a.elitism, **ops)
    model = IslandModel(ga, migrate_every=a.migrate_every, migrate_pct=a.migrate_pct, topology=a.topology,
                        transport=a.transport, timeout_s=a.timeout_s if world > 1 or a.rccl_self else None,
                        self_exchange=a.rccl_self)

    def barrier():
        if world > 1:
            dist.barrier()
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    model.connect()  # RCCL p2p connection setup happens outside the timed region
    model.run(a.warmup)
    barrier()
    g0, m0 = ga.generation, model.migrations
    t0 = time.perf_counter()
    model.run(a.steps)
    model.flush()
    barrier()
    dt = time.perf_counter() - t0
    migrations_timed = model.migrations - m0
    expected = expected_migrations(g0, a.steps, a.migrate_every) if model.world > 1 and model.k > 0 else 0

    # the slowest rank's time; every rank's migration health
    t = torch.tensor([dt, float(model.degraded), float(model.failures), float(expected - migrations_timed)],
                     dtype=torch.float64, device=device if dist.is_initialized() and device.type == "cuda" else "cpu")
    if model.world > 1 and not model.reduce_max(t):
        t[1] = 1.0  # the health reduction itself failed: this rank reports a degraded run
    dt, any_degraded, max_failures, max_short = float(t[0]), bool(t[1] > 0), int(t[2]), int(t[3])
    best = model.global_reduce_best()
    gens_per_sec = a.steps / dt
    evals = gens_per_sec * pop * world
    ref = REFSEM_EVALS_PER_SEC_PER_GPU.get(a.problem.replace("_rot", ""))
    healthy = not any_degraded and max_failures == 0 and max_short <= 0
    if rank == 0:
        xo = ops.get("crossover", ga.operators.crossover)
        out = {
            "metric": METRIC if a.problem == "onemax" else
            f"generations/sec + evals/sec, {label} ({xo}) pop={pop} per GPU, 1/2/4/8 MI355X",
            "value": evals,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": evals / (ref * world) if ref else None,
            "baseline": "reference-semantics re-creation on MI355X (bench/refsem.hip), x n_gpus" if ref else None,
            "dtype": "u1-bitpacked" if problem.encoding == "binary" else
            ("u16-permutation" if problem.encoding == "permutation" else "fp32"),
            "data": f"synthetic (random-init population, {label} objective)",
            "gens_per_sec": gens_per_sec,
            "best_fitness": best,
            # migration health: how the islands exchanged, and whether every
            # exchange of the timed window happened
            "transport": model.transport if model.world > 1 else "none",
            "self_exchange": a.rccl_self,
            "rccl_ranks": model.rccl_ranks,
            "migrations": model.migrations,
            "migrations_timed": migrations_timed,
            "migrations_expected": expected,
            "degraded": any_degraded,
            "failures": max_failures,
            "config": {
                "model": label,
                "global_batch": pop * world,
                "seq_len": problem.length,
                "parallelism": f"island{world}",
                "pop_per_gpu": pop,
                "selection": f"{ga.operators.selection}-{ga.operators.tournament_k}"
                if ga.operators.selection == "tournament" else ga.operators.selection,
                "crossover": xo,
                "mutation": ga.operators.mutation,
                "elitism": a.elitism,
                "migrate_every": a.migrate_every,
                "migrate_pct": a.migrate_pct,
                "topology": a.topology,
                "device": "cpu" if device.type == "cpu" else torch.cuda.get_device_name(device),
            },
        }
        print(json.dumps(out), flush=True)
        if not healthy:
            print(f"error: migration unhealthy (degraded={any_degraded}, failures={max_failures}, "
                  f"timed {migrations_timed} of {expected} expected on rank 0)", file=sys.stderr)
    if (world > 1 or a.rccl_self) and healthy:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if healthy else 3


if __name__ == "__main__":
    sys.exit(main())
