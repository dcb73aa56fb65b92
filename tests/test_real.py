"""REAL encoding: CPU reference vs torch oracle (CPU) and gfx950 kernels vs
CPU reference / torch oracle (GPU, incl. the MFMA rotated objectives)."""
import pytest
import torch

import libpga_amd as pga

M = pga.models

PROBLEMS = {
    "sphere": lambda: M.Sphere(30),
    "rastrigin": lambda: M.Rastrigin(30),
    "rastrigin_rot": lambda: M.Rastrigin(30, rotate=True, shift=True, seed=3),
    "rosenbrock": lambda: M.Rosenbrock(17),
    "rosenbrock_rot": lambda: M.Rosenbrock(64, rotate=True, seed=1),
    "ackley": lambda: M.Ackley(20),
    "griewank": lambda: M.Griewank(9),
    "schwefel": lambda: M.Schwefel(12, rotate=True),
    "sum": lambda: M.SumGenes(100),
    "knap": lambda: M.ReferenceKnapsack(),
    "tsp_rk": lambda: M.RandomKeyTSP.planted(40),
    "sphere_d3": lambda: M.Sphere(3, rotate=True),
    "sphere_d128": lambda: M.Sphere(128, rotate=True),
    # wave-local MFMA rotation in the pipelined kernel: 16 (GS 4) and 32 (GS 8) padded dims
    "rastrigin_rot16": lambda: M.Rastrigin(16, rotate=True, shift=True, seed=5),
    "rastrigin_rot11": lambda: M.Rastrigin(11, rotate=True, seed=6),
    "ackley_rot20": lambda: M.Ackley(20, rotate=True, shift=True, seed=7),
    "rosenbrock_rot24": lambda: M.Rosenbrock(24, rotate=True, seed=8),
    "griewank_rot32": lambda: M.Griewank(32, rotate=True, seed=9),
    # long genomes (> 256 genes: the chunk-segment kernel, one wave per individual)
    "rastrigin_1024": lambda: M.Rastrigin(1024),
    "sum_1024": lambda: M.SumGenes(1024),
    "rosenbrock_1000": lambda: M.Rosenbrock(1000),
    "ackley_777_shift": lambda: M.Ackley(777, shift=True, seed=2),
    "sphere_4096": lambda: M.Sphere(4096),
}


def close(a, b, rel=2e-4, abs_=2e-3):
    return torch.allclose(a, b, rtol=rel, atol=abs_)


@pytest.mark.parametrize("name", list(PROBLEMS))
def test_cpu_scores_match_oracle(name):
    p = PROBLEMS[name]()
    ga = pga.GeneticAlgorithm(p, 200, seed=5, device="cpu", elitism=2)
    assert close(p.reference_fitness(ga.genomes()), ga.scores)
    ga.run(5)
    assert close(p.reference_fitness(ga.genomes()), ga.scores)
    g = ga.genomes()
    tol = 1e-5 * max(abs(p.lo), abs(p.hi), 1.0)
    assert float(g.min()) >= p.lo - tol and float(g.max()) <= p.hi + tol


@pytest.mark.parametrize("xo", ["uniform", "blend", "arithmetic", "one_point", "two_point"])
@pytest.mark.parametrize("mut", ["gaussian", "uniform", "reset_one"])
def test_cpu_operators(xo, mut):
    p = M.Sphere(24)
    ga = pga.GeneticAlgorithm(p, 300, seed=1, device="cpu", crossover=xo, mutation=mut, elitism=1)
    s0 = ga.best_score()
    ga.run(25)
    assert ga.best_score() >= s0
    assert close(p.reference_fitness(ga.genomes()), ga.scores)


def test_reference_knapsack_optimum():
    """Reference E2 expects 285 = items 2 and 3 (test2/test.cu)."""
    p = M.ReferenceKnapsack()
    ga = pga.GeneticAlgorithm(p, 100, seed=2, device="cpu")
    ga.run(5)
    s, g = ga.best()
    assert s == 285.0
    assert p.counts(g.unsqueeze(0))[0].tolist() == [0, 0, 1, 1, 0, 0]


@pytest.mark.parametrize("xo", ["uniform", "two_point", "arithmetic"])
@pytest.mark.parametrize("mut", ["gaussian", "reset_one"])
def test_cpu_long_genome_operators(xo, mut):
    """L = 1030 (> 256 genes): every operator over a chunk-segment layout."""
    p = M.Rosenbrock(1030)
    ga = pga.GeneticAlgorithm(p, 64, seed=4, device="cpu", crossover=xo, mutation=mut, elitism=1)
    s0 = ga.best_score()
    ga.run(3)
    assert ga.best_score() >= s0
    assert close(p.reference_fitness(ga.genomes()), ga.scores, rel=1e-4, abs_=1.0)


def test_sum_genes_improves():
    ga = pga.GeneticAlgorithm(M.SumGenes(100), 4000, seed=2, device="cpu")
    s0 = ga.best_score()
    ga.run(30)
    assert ga.best_score() > s0 + 10


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(PROBLEMS))
def test_gpu_matches_cpu(name):
    p = PROBLEMS[name]()
    g = pga.GeneticAlgorithm(p, 1000, seed=9, device="cuda:0", elitism=1)
    c = pga.GeneticAlgorithm(p, 1000, seed=9, device="cpu", elitism=1)
    torch.cuda.synchronize()
    assert torch.equal(g.rows.cpu(), c.rows), "init rows differ"
    assert close(g.scores.cpu(), c.scores)
    assert close(p.reference_fitness(g.genomes().cpu()), g.scores.cpu())
    # one generation from the SAME population: selection identical unless two
    # scores are within an ulp; compare children gene-wise with tolerance
    g.run(1)
    c.run(1)
    torch.cuda.synchronize()
    gg, cg = g.genomes().cpu(), c.genomes()
    same_rows = torch.isclose(gg, cg, rtol=1e-4, atol=1e-4).all(-1).float().mean().item()
    assert same_rows > 0.99
    assert close(p.reference_fitness(gg), g.scores.cpu())


@pytest.mark.gpu
def test_gpu_rastrigin30_rotated_mfma_1m():
    """BASELINE config 3 shape: Rastrigin-30D rotated, pop = 1M, MFMA scores."""
    p = M.Rastrigin(30, rotate=True, shift=True, seed=4)
    ga = pga.GeneticAlgorithm(p, 1 << 20, seed=1, device="cuda:0", elitism=1)
    b0 = ga.best_score()
    ga.run(20)
    torch.cuda.synchronize()
    idx = torch.randint(0, 1 << 20, (4096,), device="cuda:0")
    ref = p.reference_fitness(ga.genomes()[idx])
    assert close(ref, ga.scores[idx], rel=1e-4, abs_=5e-3)
    assert ga.best_score() > b0


@pytest.mark.gpu
@pytest.mark.parametrize("xo", ["uniform", "one_point", "blend"])
@pytest.mark.parametrize("mut", ["gaussian", "uniform", "reset_one"])
def test_gpu_long_genome_bitexact_rows(xo, mut):
    """Sphere-1000 / sum-1024: the long-genome kernel's children equal the
    CPU backend's bit for bit over several generations (gaussian mutation:
    to libm tolerance), scores to float rounding."""
    for p in (M.Sphere(1000), M.SumGenes(1024)):
        kw = dict(seed=13, elitism=1, crossover=xo, mutation=mut)
        g = pga.GeneticAlgorithm(p, 512, device="cuda:0", **kw)
        c = pga.GeneticAlgorithm(p, 512, device="cpu", **kw)
        g.run(3)
        c.run(3)
        torch.cuda.synchronize()
        if mut == "gaussian":  # Box-Muller: device and host libm differ by ulps
            same = torch.isclose(g.genomes().cpu(), c.genomes(), rtol=1e-4, atol=1e-4).all(-1).float().mean()
            assert same.item() > 0.99
            assert close(p.reference_fitness(g.genomes().cpu()), g.scores.cpu())
        else:  # children bit for bit; scores to rounding (the device contracts a*b+c into fma)
            assert torch.equal(g.rows.cpu(), c.rows)
            assert close(g.scores.cpu(), c.scores, rel=1e-5, abs_=1e-2)
