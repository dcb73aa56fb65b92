#!/usr/bin/env python3
"""Many small islands on one device: batched launch vs one stream per island.

    python bench/bench_islands.py [--islands 8] [--pop 4096] [--length 1024] [--gens 500]
                                  [--problem onemax|rastrigin30|tsp128]

LocalIslands runs its islands either as ONE launch per generation (island =
grid y, Island::run_batched) or each island's launch on its own HIP stream
(batched=False).  Migration is off so only the generations are timed.  One
JSON line per mode: generations/s of the whole island set, evals/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libpga_amd as pga  # noqa: E402
from libpga_amd.parallel import LocalIslands  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--islands", type=int, default=8)
    ap.add_argument("--pop", type=int, default=4096)
    ap.add_argument("--length", type=int, default=1024)
    ap.add_argument("--gens", type=int, default=500)
    ap.add_argument("--problem", default="onemax", choices=["onemax", "rastrigin30", "tsp128"])
    a = ap.parse_args()
    if a.problem != "onemax":
        a.length = 30 if a.problem == "rastrigin30" else 128
    for batched in (True, False):
        prob = {"onemax": lambda: pga.models.OneMax(a.length), "rastrigin30": lambda: pga.models.Rastrigin(30),
                "tsp128": lambda: pga.models.TSP.random_euclidean(128, seed=1)}[a.problem]()
        li = LocalIslands(prob, a.islands, a.pop, seed=1, device="cuda:0", migrate_every=0,
                          elitism=1, batched=batched)
        li.run(20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        li.run(a.gens)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"problem": a.problem, "mode": "batched" if batched else "streams", "islands": a.islands,
                          "pop": a.pop,
                          "length": a.length, "gens_per_sec": a.gens / dt, "us_per_gen": dt / a.gens * 1e6,
                          "evals_per_sec": a.gens * a.islands * a.pop / dt,
                          "batched_generations": li.batched_generations}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
