"""QUBO / Max-Cut on the int8 matrix cores (csrc/kernels/qubo.hip).

CPU: the CPU backend's integer x^T Q x against a plain-PyTorch oracle, and
search quality on small instances with known optima.  GPU: the MFMA kernel
against the CPU backend bit for bit (every padded length 64..1024, odd
lengths, asymmetric Q, population tails), and whole runs.
Reference: no quadratic objective exists in the reference (its only
objectives are the example device functions, test*/test.cu); parity unpinned."""
import itertools

import pytest
import torch

import libpga_amd as pga
from libpga_amd import models as M


def brute_force(problem):
    L = problem.length
    xs = torch.tensor(list(itertools.product([0, 1], repeat=L)), dtype=torch.uint8)
    return problem.reference_fitness(xs).max().item()


def test_cpu_scores_match_oracle():
    p = M.QUBO.random(70, seed=1)
    ga = pga.GeneticAlgorithm(p, 300, seed=2, device="cpu")
    assert torch.equal(ga.scores, p.reference_fitness(ga.genomes()))
    ga.run(3)
    assert torch.equal(ga.scores, p.reference_fitness(ga.genomes()))


def test_cpu_qubo_finds_optimum_small():
    p = M.QUBO.random(12, seed=5)
    opt = brute_force(p)
    ga = pga.GeneticAlgorithm(p, 512, seed=3, device="cpu", elitism=2)
    ga.run(60)
    assert ga.best_score() == opt


def test_maxcut_bipartite_is_fully_cut():
    # complete bipartite K_{6,6}: the max cut separates the sides, 36 edges
    n = 12
    side = torch.arange(n) < 6
    W = (side[:, None] != side[None, :]).to(torch.int64)
    p = M.MaxCut(W)
    ga = pga.GeneticAlgorithm(p, 1024, seed=4, device="cpu", elitism=1)
    ga.run(40)
    assert ga.best_score() == 36.0
    _, g = ga.best()
    assert p.cut_value(g[None]).item() == 36
    assert torch.equal(p.cut_value(ga.genomes()).float(), ga.scores)


def test_qubo_validation():
    with pytest.raises(ValueError):
        M.QUBO(torch.full((4, 4), 200))
    with pytest.raises(ValueError):
        M.QUBO(torch.full((4, 4), 0.5))


@pytest.mark.gpu
@pytest.mark.parametrize("L", [5, 64, 100, 128, 200, 256, 300, 512, 777, 1024])
def test_gpu_qubo_bitexact(L):
    p = M.QUBO.random(L, seed=L, lo=-128, hi=127)  # full int8 range, asymmetric
    S = 1000 if L <= 512 else 300
    g = pga.GeneticAlgorithm(p, S, seed=7, device="cuda:0", elitism=1)
    c = pga.GeneticAlgorithm(p, S, seed=7, device="cpu", elitism=1)
    torch.cuda.synchronize()
    assert torch.equal(g.scores.cpu(), c.scores)
    assert torch.equal(g.scores.cpu(), p.reference_fitness(g.genomes().cpu()))
    g.run(2)
    c.run(2)
    torch.cuda.synchronize()
    assert torch.equal(g.rows.cpu(), c.rows)
    assert torch.equal(g.scores.cpu(), c.scores)
    assert g.best_score() == c.best_score()


@pytest.mark.gpu
def test_gpu_maxcut_run():
    p = M.MaxCut.random_graph(512, degree=12, seed=3)
    ga = pga.GeneticAlgorithm(p, 1 << 16, seed=1, device="cuda:0", elitism=1)
    s0 = ga.best_score()
    ga.run(30)
    torch.cuda.synchronize()
    assert ga.best_score() > s0
    _, g = ga.best()
    assert p.cut_value(g[None].cpu()).item() == ga.best_score()
