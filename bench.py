#!/usr/bin/env python3
"""Headline benchmark: generations/sec + evals/sec, OneMax pop=1M 1024-bit.

One island of pop=1M (1024-bit bit-packed OneMax, tournament-2, uniform
crossover, bit-flip mutation at 1/L, elitism 1) per GPU; with N>1 GPUs the
islands exchange their top 1% every 10 generations over RCCL (ring), so the
per-GPU work is fixed as N grows (weak scaling).  A "step" is one generation
of every island, fused selection+crossover+mutation+evaluation included;
migrations that fall in the timed window are timed too.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

Prints ONE JSON line (rank 0): value = total evals/s over all GPUs.
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
# profiles/reference_semantics.jsonl): 1.91 gens/s = 2.00e6 evals/s for
# OneMax-1024 pop=1M on one GPU.  Scaled by the GPU count (perfect scaling
# credited to the reference, which has no multi-GPU code at all).
REFSEM_EVALS_PER_SEC_PER_GPU = 2.00086e6


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--pop", type=int, default=1 << 20)
    ap.add_argument("--length", type=int, default=1024)
    ap.add_argument("--migrate-every", type=int, default=10)
    ap.add_argument("--migrate-pct", type=float, default=0.01)
    ap.add_argument("--topology", default="ring")
    ap.add_argument("--elitism", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--cpu", action="store_true", help="CPU reference backend (plumbing check)")
    a = ap.parse_args()

    rank, world, device = init_distributed("gloo" if a.cpu else None)
    if a.cpu:
        device = torch.device("cpu")
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    problem = pga.models.OneMax(a.length)
    ga = pga.GeneticAlgorithm(problem, a.pop, seed=a.seed, island=rank, device=device, elitism=a.elitism,
                              selection="tournament", tournament_k=2, crossover="uniform", mutation="bit_flip")
    model = IslandModel(ga, migrate_every=a.migrate_every, migrate_pct=a.migrate_pct, topology=a.topology)

    def barrier():
        if world > 1:
            dist.barrier()
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    model.connect()  # RCCL p2p connection setup happens outside the timed region
    model.run(a.warmup)
    barrier()
    t0 = time.perf_counter()
    model.run(a.steps)
    model.flush()
    barrier()
    dt = time.perf_counter() - t0

    t = torch.tensor([dt], dtype=torch.float64, device=device if world > 1 and device.type == "cuda" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    best = model.global_reduce_best()
    gens_per_sec = a.steps / dt
    evals = gens_per_sec * a.pop * world
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": evals,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": evals / (REFSEM_EVALS_PER_SEC_PER_GPU * world),
            "baseline": "reference-semantics re-creation on MI355X (bench/refsem.hip), x n_gpus",
            "dtype": "u1-bitpacked",
            "data": "synthetic (random-init population, OneMax objective)",
            "gens_per_sec": gens_per_sec,
            "best_fitness": best,
            "migrations": model.migrations,
            "config": {
                "model": f"OneMax-{a.length}bit",
                "global_batch": a.pop * world,
                "seq_len": a.length,
                "parallelism": f"island{world}",
                "pop_per_gpu": a.pop,
                "selection": "tournament-2",
                "crossover": "uniform",
                "mutation": f"bit-flip 1/{a.length}",
                "elitism": a.elitism,
                "migrate_every": a.migrate_every,
                "migrate_pct": a.migrate_pct,
                "topology": a.topology,
                "device": "cpu" if device.type == "cpu" else torch.cuda.get_device_name(device),
            },
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
