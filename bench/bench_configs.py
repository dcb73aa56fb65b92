#!/usr/bin/env python3
"""Every BASELINE.json config on one device, one JSON line each.

    python bench/bench_configs.py [--only NAME ...] [--out FILE]

Configs (BASELINE.md "Targets" table):
  onemax64_cpu      OneMax 64-bit, pop=1024, CPU reference backend
  onemax1024        OneMax 1024-bit, pop=1M, one GPU (the headline island)
  rastrigin30       Rastrigin-30D float, pop=1M (blend + gaussian)
  rastrigin30_rot   Rastrigin-30D rotated, pop=1M (fitness through MFMA tiles)
  tsp256_ox / _pmx  TSP-256 permutation, pop=256K, OX / PMX crossover (symmetric f32 distance matrix)
  tsp256_asym_*     the same with an asymmetric f32 matrix (L2-gathered)
  tsp256_euc_*      the same instance as city coordinates (TSPEuclidean)
  tsp256_int_*      an integer EUC_2D matrix (u16 copy in LDS)
  e1_sum100_refops  reference example E1 (S=40000, L=100) with the reference's
                    operators — the head-to-head against build/bench/refsem
  e2_knap_refops    reference example E2 (S=100, L=6), launch-bound (hipGraph)
  onemax64_gpu      OneMax 64-bit, pop=1024 on the GPU (launch-bound)
  onemax1024_jit    the headline island with a hipRTC-compiled objective
  rastrigin30_jit   Rastrigin-30D written as HIP source, fused into the REAL kernel
  knapsack1024      0/1 knapsack, 1024 items, pop=1M (matrix-core evaluation)
The 8-GPU island configs are bench.py under torchrun (the driver runs those).
Each line: gens/s, evals/s, ms/gen, best fitness, effective HBM GB/s (the
bytes one generation must move at minimum: read 2 parent rows + write 1
child row + scores, divided by the time).
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


def make(name: str):
    M = pga.models
    if name == "onemax64_cpu":
        return M.OneMax(64), 1024, "cpu", {}, 2000
    if name == "onemax1024":
        return M.OneMax(1024), 1 << 20, None, dict(elitism=1), 300
    if name == "rastrigin30":
        return M.Rastrigin(30), 1 << 20, None, dict(elitism=1), 200
    if name == "rastrigin30_rot":
        return M.Rastrigin(30, rotate=True, seed=1), 1 << 20, None, dict(elitism=1), 200
    if name == "e1_sum100_refops":
        # reference example E1 with the reference's own operators (binary tournament,
        # uniform crossover, 1% single-gene reset): same algorithm as build/bench/refsem
        return M.SumGenes(100), 40000, None, {}, 500
    if name == "onemax1024_jit":
        # the headline config with the objective written as HIP source (hipRTC)
        src = """__device__ float ones(const unsigned int* w, unsigned int n, const float* d) {
            float s = 0.f; for (unsigned i = 0; i < (n + 31) / 32; ++i) s += __popc(w[i]); return s; }"""
        return M.JitObjective("binary", 1024, src, name="ones"), 1 << 20, None, dict(elitism=1), 300
    if name == "rastrigin30_jit":
        # the rastrigin30 config with the objective as user source (fused, LDS rows)
        src = """__device__ float rast(const float* x, unsigned int n, const float* d) {
            float s = 10.f * n;
            for (unsigned int i = 0; i < n; ++i) s += x[i] * x[i] - 10.f * __cosf(6.28318530718f * x[i]);
            return -s; }"""
        return M.JitObjective("real", 30, src, name="rast", bounds=(-5.12, 5.12)), 1 << 20, None, dict(elitism=1), 200
    if name == "e2_knap_refops":
        # reference example E2 (S=100, L=6): launch-bound, the hipGraph replay case
        return M.ReferenceKnapsack(), 100, None, {}, 5000
    if name == "onemax64_gpu":
        return M.OneMax(64), 1024, None, {}, 5000
    if name in ("tsp256_euc_ox", "tsp256_euc_pmx"):
        # the same 256-city instance as tsp256_*, given as coordinates: the
        # fused kernel stages them in LDS instead of gathering matrix entries from L2
        g = torch.Generator().manual_seed(7)
        xy = torch.rand(256, 2, generator=g)
        xo = "ox" if name.endswith("ox") else "pmx"
        return M.TSPEuclidean(xy), 1 << 18, None, dict(elitism=1, crossover=xo), 50
    if name in ("tsp256_int_ox", "tsp256_int_pmx"):
        # the same geometry as an integer matrix (TSPLIB EUC_2D rounding): the
        # fused kernel evaluates tours from a u16 copy of the matrix in LDS
        xo = "ox" if name.endswith("ox") else "pmx"
        return M.TSP.random_integer_euclidean(256, seed=7), 1 << 18, None, dict(elitism=1, crossover=xo), 50
    if name in ("tsp256_ox", "tsp256_pmx"):
        g = torch.Generator().manual_seed(7)
        xy = torch.rand(256, 2, generator=g)
        # the exact pairwise distances (no matmul expansion: through it cdist
        # returns a matrix that is not symmetric bit for bit and has a
        # non-zero diagonal, up to 5e-4); a symmetric float matrix is staged
        # in LDS as its f32 triangle (perm.hip TBL 3), an asymmetric one is
        # gathered from L2 (tsp256_asym_* below)
        d = torch.cdist(xy, xy, compute_mode="donot_use_mm_for_euclid_dist")
        xo = "ox" if name.endswith("ox") else "pmx"
        return M.TSP(d), 1 << 18, None, dict(elitism=1, crossover=xo), 50
    if name in ("tsp256_asym_ox", "tsp256_asym_pmx"):
        # an asymmetric float matrix (each direction of an edge scaled apart):
        # the f32 L2 gather path of the kernel
        g = torch.Generator().manual_seed(7)
        xy = torch.rand(256, 2, generator=g)
        d = torch.cdist(xy, xy, compute_mode="donot_use_mm_for_euclid_dist")
        d = d * (1 + 0.1 * torch.rand(256, 256, generator=g))
        xo = "ox" if name.endswith("ox") else "pmx"
        return M.TSP(d), 1 << 18, None, dict(elitism=1, crossover=xo), 50
    if name == "maxcut512_qubo":
        # Max-Cut of a random 512-vertex graph as a QUBO on the int8 matrix cores
        return M.MaxCut.random_graph(512, degree=16, seed=1), 1 << 20, None, dict(elitism=1), 50
    if name == "qubo1024":
        # dense 1024-variable QUBO (1M int8 MACs per individual)
        return M.QUBO.random(1024, seed=1, lo=-128, hi=127), 1 << 18, None, dict(elitism=1), 20
    if name == "knapsack1024":
        # 0/1 knapsack, 1024 items (integer values / weights 1..99): the
        # integer-exact instance runs its evaluation on the int8 matrix cores
        return M.Knapsack01.random(1024, seed=1), 1 << 20, None, dict(elitism=1), 200
    if name == "onemax1024_rank":
        return M.OneMax(1024), 1 << 20, None, dict(elitism=1, selection="rank", rank_pressure=1.5), 100
    if name == "onemax1024_roulette_2pt":
        # BASELINE north-star operator set: roulette selection, two-point crossover, bit-flip, elitism
        return M.OneMax(1024), 1 << 20, None, dict(elitism=1, selection="roulette", crossover="two_point"), 100
    raise KeyError(name)


NAMES = ["onemax64_cpu", "onemax1024", "rastrigin30", "rastrigin30_rot", "tsp256_ox", "tsp256_pmx", "tsp256_int_ox",
         "tsp256_int_pmx", "tsp256_asym_ox", "tsp256_asym_pmx", "e1_sum100_refops",
         "tsp256_euc_ox", "tsp256_euc_pmx", "e2_knap_refops", "onemax64_gpu", "onemax1024_jit", "rastrigin30_jit", "maxcut512_qubo",
         "qubo1024", "onemax1024_rank", "knapsack1024", "onemax1024_roulette_2pt"]


def qubo_padded(L: int) -> int:
    lp = 64
    while lp < L:
        lp *= 2
    return lp


def run_one(name: str, steps_scale: float) -> dict:
    problem, S, dev, kw, steps = make(name)
    steps = max(5, int(steps * steps_scale))
    if dev is None:
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        if dev == "cpu":
            S, steps = min(S, 4096), min(steps, 20)
    ga = pga.GeneticAlgorithm(problem, S, seed=1, device=dev, **kw)
    ga.run(max(2, steps // 10))
    ga.synchronize()
    t0 = time.perf_counter()
    ga.run(steps)
    ga.synchronize()
    dt = time.perf_counter() - t0
    row_bytes = int(ga.island.row_words) * 4
    gens = steps / dt
    min_bytes = S * (3 * row_bytes + 8)
    return {"config": name, "device": dev if dev == "cpu" else torch.cuda.get_device_name(), "pop": S,
            "length": problem.length, "encoding": problem.encoding, "gens_per_sec": gens, "evals_per_sec": gens * S,
            "ms_per_gen": dt / steps * 1e3, "best": ga.best_score(), "steps": steps,
            "effective_GBps": min_bytes * gens / 1e9,
            **({"int8_TOPS": 2.0 * qubo_padded(problem.length) ** 2 * S * gens / 1e12}
               if problem.objective == pga._ext.C.OBJ_QUBO else {})}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--scale", type=float, default=1.0, help="multiply the step counts")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = []
    for n in (a.only or NAMES):
        r = run_one(n, a.scale)
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
