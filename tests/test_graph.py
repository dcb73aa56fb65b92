"""hipGraph replay (Island::run with graph_generations > 0) must be
bit-identical to plain launches, across encodings, elitism and roulette."""
import pytest
import torch

import libpga_amd as pga

M = pga.models

CASES = {
    "onemax_e1": (lambda: M.OneMax(300), 5000, dict(elitism=1)),
    "onemax_e4_roulette": (lambda: M.OneMax(200), 3000, dict(elitism=4, selection="roulette")),
    "trap_k3": (lambda: M.Trap(120, 4), 2000, dict(elitism=2, selection="tournament", tournament_k=3)),
    "rastrigin_rot": (lambda: M.Rastrigin(20, rotate=True, seed=2), 4000, dict(elitism=1)),
    "sum_refops": (lambda: M.SumGenes(100), 40000, {}),
    "tsp_ox": (lambda: M.TSP(torch.rand(40, 40, generator=torch.Generator().manual_seed(1))), 2000, dict(elitism=1)),
    # a source objective fused into the generation kernel: the variant loaded by
    # the first plain generations is replayed inside the graph
    "onemax_jit_fused": (lambda: M.JitObjective("binary", 256, """
__device__ float ones(const unsigned int* w, unsigned int nbits, const float* data) {
  float s = 0.f;
  for (unsigned int i = 0; i < (nbits + 31) / 32; ++i) s += (float)__popc(w[i]);
  return s;
}""", name="ones"), 5000, dict(elitism=1)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_graph_replay_bit_identical(name):
    mk, S, kw = CASES[name]
    p = mk()
    a = pga.GeneticAlgorithm(p, S, seed=3, device="cuda:0", **kw)
    b = pga.GeneticAlgorithm(p, S, seed=3, device="cuda:0", **kw)
    a.island.graph_generations = 0
    b.island.graph_generations = 8
    for n in (3, 21, 40, 1, 17):  # odd lengths: recapture + plain tails
        a.run(n)
        b.run(n)
    torch.cuda.synchronize()
    assert b.island.graph_replays > 0
    assert a.generation == b.generation == 82
    assert torch.equal(a.rows, b.rows)
    assert torch.equal(a.scores, b.scores)
    assert a.best_score() == b.best_score()


def test_graph_setting_cpu_noop():
    ga = pga.GeneticAlgorithm(M.OneMax(64), 128, seed=1, device="cpu")
    ga.island.graph_generations = 7  # rounded to even, unused on the CPU backend
    assert ga.island.graph_generations == 8
    ga.run(20)
    assert ga.island.graph_replays == 0
