"""PERMUTATION encoding (TSP): validity, oracle agreement, operators, and
gfx950 vs CPU bit-exactness."""
import pytest
import torch

import libpga_amd as pga

M = pga.models


def is_perm(g):
    n = g.shape[1]
    return bool((g.sort(-1).values == torch.arange(n, device=g.device)).all())


@pytest.mark.parametrize("xo", ["ox", "pmx", "none"])
@pytest.mark.parametrize("mut", ["swap", "inversion"])
@pytest.mark.parametrize("n", [5, 8, 50, 257])
def test_cpu_valid_and_scores(xo, mut, n):
    p = M.TSP.random_euclidean(n, seed=n)
    ga = pga.GeneticAlgorithm(p, 96, seed=4, device="cpu", crossover=xo, mutation=mut, mutation_rate=0.5,
                              crossover_prob=0.9, elitism=1)
    assert is_perm(ga.genomes())
    ga.run(4)
    g = ga.genomes()
    assert is_perm(g)
    assert torch.allclose(p.reference_fitness(g), ga.scores, rtol=1e-5, atol=1e-2)


def test_crossover_known_answers():
    """The library's OX1 and PMX (the CPU backend's operator, which the GPU
    kernels match bit for bit in test_gpu_bitexact) on the textbook parents
    A = 1..9, B = 9 3 7 8 2 6 5 1 4 with A's segment 4 5 6 7 (cuts [3, 7)),
    written 0-based.  OX1 (Davis): 3 8 2 4 5 6 7 1 9.  PMX (Goldberg and
    Lingle): 9 3 2 4 5 6 7 1 8."""
    from libpga_amd import _C
    A = [0, 1, 2, 3, 4, 5, 6, 7, 8]
    B = [8, 2, 6, 7, 1, 5, 4, 0, 3]
    XO_PMX, XO_OX = 5, 6
    assert _C.perm_crossover(XO_OX, A, B, 3, 7) == [2, 7, 1, 3, 4, 5, 6, 0, 8]
    assert _C.perm_crossover(XO_PMX, A, B, 3, 7) == [8, 2, 1, 3, 4, 5, 6, 0, 7]
    # degenerate segments: an empty one gives B, the full one A
    for op in (XO_OX, XO_PMX):
        assert _C.perm_crossover(op, A, B, 4, 4) == B
        assert _C.perm_crossover(op, A, B, 0, 9) == A

def test_tsp_circle_converges():
    p = M.TSPEuclidean.circle(24)
    ga = pga.GeneticAlgorithm(p, 2048, seed=1, device="cpu", elitism=1)
    ga.run(150)
    opt = float(p.tour_length(torch.arange(24).unsqueeze(0))[0])
    assert -ga.best_score() < 1.05 * opt


@pytest.mark.gpu
@pytest.mark.parametrize("xo", ["ox", "pmx"])
@pytest.mark.parametrize("n,S", [(9, 333), (64, 1000), (256, 2048), (1000, 64)])
@pytest.mark.parametrize("prob", ["matrix", "euc", "open"])
@pytest.mark.parametrize("elitism", [1, 2])  # 1: device argmax elite; 2: elite index list
def test_gpu_bitexact(xo, n, S, prob, elitism):
    p = {"matrix": lambda: M.TSP.random_euclidean(n, seed=2), "euc": lambda: M.TSPEuclidean.random(n, seed=2),
         "open": lambda: M.TSP.random_euclidean(n, seed=2, open_path=True)}[prob]()
    kw = dict(seed=5, crossover=xo, mutation="inversion", mutation_rate=0.4, elitism=elitism)
    g = pga.GeneticAlgorithm(p, S, device="cuda:0", **kw)
    c = pga.GeneticAlgorithm(p, S, device="cpu", **kw)
    for _ in range(3):
        torch.cuda.synchronize()
        assert torch.equal(g.rows.cpu(), c.rows)
        assert torch.equal(g.scores.cpu(), c.scores)
        g.run(1)
        c.run(1)
    assert is_perm(g.genomes().cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("xo", ["ox", "pmx"])
@pytest.mark.parametrize("n", [64, 256])
@pytest.mark.parametrize("shape", ["asymmetric", "nonzero_diagonal"])
def test_gpu_bitexact_general_matrix(xo, n, shape):
    """Distance matrices that are not symmetric, or have a non-zero diagonal
    (the closing edge and clamped ids read it): bit-exact vs the CPU."""
    g0 = torch.Generator().manual_seed(n)
    d = torch.rand(n, n, generator=g0) * 10
    if shape == "nonzero_diagonal":
        d = (d + d.T) / 2
    else:
        d.fill_diagonal_(0)
    p = M.TSP(d)
    kw = dict(seed=8, crossover=xo, mutation="swap", mutation_rate=0.4, elitism=1)
    g = pga.GeneticAlgorithm(p, 1024, device="cuda:0", **kw)
    c = pga.GeneticAlgorithm(p, 1024, device="cpu", **kw)
    g.run(3)
    c.run(3)
    torch.cuda.synchronize()
    assert torch.equal(g.rows.cpu(), c.rows)
    assert torch.equal(g.scores.cpu(), c.scores)


@pytest.mark.gpu
@pytest.mark.parametrize("xo", ["ox", "pmx"])
@pytest.mark.parametrize("inst", ["int_euc256", "e3_100", "int_euc100_open", "f32_sym256", "f32_sym100_open"])
def test_gpu_lds_matrix_bitexact(xo, inst, monkeypatch):
    """Matrices evaluate from a copy in LDS: integer ones as u16 (symmetric:
    strict triangle + diagonal in 16-wave blocks; asymmetric: the full
    matrix), other symmetric ones as the f32 triangle + diagonal (131.6 KB at
    256 cities): rows and scores equal the CPU backend and the f32 L2 path
    bit for bit."""
    p = {"int_euc256": lambda: M.TSP.random_integer_euclidean(256, seed=2),
         "e3_100": lambda: M.TSP.reference_e3(100, seed=1),
         "int_euc100_open": lambda: M.TSP.random_integer_euclidean(100, seed=5, open_path=True),
         "f32_sym256": lambda: M.TSP.random_euclidean(256, seed=2),
         "f32_sym100_open": lambda: M.TSP.random_euclidean(100, seed=5, open_path=True)}[inst]()
    if inst.startswith("f32"):
        assert torch.equal(p.dist, p.dist.T) and not torch.equal(p.dist, p.dist.round())
    kw = dict(seed=8, crossover=xo, mutation="inversion", mutation_rate=0.4, elitism=1)
    g = pga.GeneticAlgorithm(p, 5000, device="cuda:0", **kw)
    c = pga.GeneticAlgorithm(p, 5000, device="cpu", **kw)
    monkeypatch.setenv("PGA_TSP_NO_LDS", "1")
    f = pga.GeneticAlgorithm(p, 5000, device="cuda:0", **kw)
    for _ in range(3):
        g.run(1)
        c.run(1)
        f.run(1)
    torch.cuda.synchronize()
    assert torch.equal(g.rows.cpu(), c.rows) and torch.equal(g.scores.cpu(), c.scores)
    assert torch.equal(g.rows, f.rows) and torch.equal(g.scores, f.scores)
    assert is_perm(g.genomes().cpu())


def test_reference_e3_instance():
    p = M.TSP.reference_e3(100, seed=3)
    d = p.dist
    assert p.open_path and d.shape == (100, 100)
    assert bool((d == d.round()).all()) and float(d.min()) >= 10 and float(d.max()) <= 1009
    assert float(p.tour_length(torch.arange(100).unsqueeze(0))[0]) == 990.0


@pytest.mark.gpu
def test_gpu_tsp256_pop256k():
    """BASELINE config 5 shape on one GPU: TSP-256, pop = 256K, OX."""
    p = M.TSPEuclidean.random(256, seed=9)
    ga = pga.GeneticAlgorithm(p, 256 * 1024, seed=1, device="cuda:0", elitism=1)
    b0 = ga.best_score()
    ga.run(10)
    torch.cuda.synchronize()
    idx = torch.randint(0, 256 * 1024, (2048,), device="cuda:0")
    g = ga.genomes()[idx]
    assert is_perm(g)
    assert torch.allclose(p.reference_fitness(g), ga.scores[idx], rtol=1e-4, atol=0.5)
    assert ga.best_score() > b0


@pytest.mark.gpu
@pytest.mark.parametrize("sel", ["rank", "roulette"])
def test_gpu_bitexact_selections(sel):
    p = M.TSP.random_euclidean(64, seed=3)
    kw = dict(seed=6, crossover="pmx", mutation="swap", mutation_rate=0.3, elitism=1, selection=sel)
    g = pga.GeneticAlgorithm(p, 1500, device="cuda:0", **kw)
    c = pga.GeneticAlgorithm(p, 1500, device="cpu", **kw)
    g.run(3)
    c.run(3)
    torch.cuda.synchronize()
    assert torch.equal(g.rows.cpu(), c.rows)
    assert torch.equal(g.scores.cpu(), c.scores)


@pytest.mark.parametrize("xo", ["ox", "pmx"])
def test_cpu_long_genome(xo):
    """Tours beyond the 4096 genes of the 4-per-block kernels (the GPU runs
    them one individual per 64-lane block)."""
    p = M.TSPEuclidean.random(6000, seed=3)
    ga = pga.GeneticAlgorithm(p, 24, seed=2, device="cpu", crossover=xo, mutation="inversion", elitism=1)
    ga.run(2)
    assert is_perm(ga.genomes())
    assert torch.allclose(p.reference_fitness(ga.genomes()), ga.scores, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("xo", ["ox", "pmx"])
@pytest.mark.parametrize("n,prob", [(4104, "euc"), (10000, "euc"), (8192, "matrix")])
def test_gpu_long_genome_bitexact(xo, n, prob):
    p = M.TSPEuclidean.random(n, seed=7) if prob == "euc" else M.TSP.random_euclidean(n, seed=7)
    kw = dict(seed=3, crossover=xo, mutation="inversion", mutation_rate=0.5, elitism=1)
    g = pga.GeneticAlgorithm(p, 300, device="cuda:0", **kw)
    c = pga.GeneticAlgorithm(p, 300, device="cpu", **kw)
    for _ in range(2):
        g.run(1)
        c.run(1)
    torch.cuda.synchronize()
    assert torch.equal(g.rows.cpu(), c.rows)
    assert torch.equal(g.scores.cpu(), c.scores)
    assert is_perm(g.genomes().cpu())


@pytest.mark.gpu
def test_gpu_long_genome_too_long():
    p = M.TSPEuclidean.random(12000, seed=1)
    with pytest.raises(Exception, match="too long"):
        pga.GeneticAlgorithm(p, 16, device="cuda:0")


def test_cpu_rank_selection_tsp():
    p = M.TSP.random_euclidean(32, seed=4)
    ga = pga.GeneticAlgorithm(p, 512, seed=1, device="cpu", selection="rank", rank_pressure=1.8, elitism=1)
    s0 = ga.best_score()
    ga.run(30)
    assert ga.best_score() > s0
    assert is_perm(ga.genomes())


def _forged_rows(ga, n):
    """k rows of a TSP island: valid tours, then three forgeries (every gene
    city 0; a duplicated city; a city beyond the tour)."""
    k = 8
    rows = ga.rows[:k].clone()
    g16 = rows.view(torch.int16)
    g16[0, :n] = 0
    g16[1, :n] = torch.arange(n, dtype=torch.int16)
    g16[1, n // 2] = 1
    g16[2, :n] = torch.arange(n, dtype=torch.int16)
    g16[2, n - 1] = n + 3
    return rows.reshape(-1), torch.full((k,), 1e9)


@pytest.mark.parametrize("n", [9, 64, 257])
def test_evaluate_rows_sanitizes_forged_cpu(n):
    """Island.evaluate_rows (the migrants' re-scoring) turns a row that is
    not a permutation into the identity tour, scored as one; valid rows keep
    their genes and get their true score."""
    p = M.TSP.random_euclidean(n, seed=1)
    ga = pga.GeneticAlgorithm(p, 64, seed=3, device="cpu")
    rows, sc = _forged_rows(ga, n)
    orig = ga.rows[:8].clone()
    ga.island.evaluate_rows(rows, sc)
    genes = p.decode(rows.view(8, -1))
    ident = torch.arange(n)
    for i in range(3):
        assert torch.equal(genes[i], ident)
    assert torch.equal(rows.view(8, -1)[3:], orig[3:])
    assert torch.allclose(sc, p.reference_fitness(genes), rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [9, 64, 257, 1000])
def test_evaluate_rows_sanitizes_forged_gpu(n):
    """The same on gfx950 (perm.hip MODE_EVAL), bit-exact with the CPU backend."""
    p = M.TSP.random_euclidean(n, seed=1)
    c = pga.GeneticAlgorithm(p, 64, seed=3, device="cpu")
    g = pga.GeneticAlgorithm(p, 64, seed=3, device="cuda:0")
    rc, sc = _forged_rows(c, n)
    rg, sg = rc.clone().cuda(), sc.clone().cuda()
    c.island.evaluate_rows(rc, sc)
    g.island.evaluate_rows(rg, sg)
    torch.cuda.synchronize()
    assert torch.equal(rg.cpu(), rc) and torch.equal(sg.cpu(), sc)
    assert torch.equal(p.decode(rc.view(8, -1))[0], torch.arange(n))
