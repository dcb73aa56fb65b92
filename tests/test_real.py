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


# transcendental objectives: the device's v_cos_f32 / libm differ from the
# host's by ulps, so scores agree to rounding; every other objective is exact
TRANSCENDENTAL = {"rastrigin", "rastrigin_rot", "ackley", "griewank", "schwefel", "rastrigin_rot16", "rastrigin_rot11",
                  "ackley_rot20", "griewank_rot32", "rastrigin_1024", "ackley_777_shift", "tsp_rk"}


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
    g.run(1)
    c.run(1)
    torch.cuda.synchronize()
    if name in TRANSCENDENTAL:
        # selection is identical unless two contestants' scores lie within an ulp
        same_rows = (g.rows.cpu() == c.rows).all(-1).float().mean().item()
        assert same_rows > 0.995
        assert close(g.scores.cpu(), c.scores) or same_rows < 1.0
    else:
        assert torch.equal(g.rows.cpu(), c.rows)
        assert torch.equal(g.scores.cpu(), c.scores)
    assert close(p.reference_fitness(g.genomes().cpu()), g.scores.cpu())


# polynomial objectives through the transposed kernel (real_gen_tp): rows AND
# scores equal the CPU backend's bit for bit, generation after generation
EXACT = {
    "sphere30": lambda: M.Sphere(30),          # GS 8, the Rastrigin-30D geometry
    "sphere30_rot": lambda: M.Sphere(30, rotate=True, shift=True, seed=2),  # wave-local MFMA rotation
    "rosen13_rot": lambda: M.Rosenbrock(13, rotate=True, seed=3),          # GS 4 rotation
    "rosen30": lambda: M.Rosenbrock(30),       # neighbour gene across lanes
    "sum30": lambda: M.SumGenes(30),
    "sphere100": lambda: M.Sphere(100),        # GS 32
    "sphere256": lambda: M.Sphere(256),        # GS 64, every lane a chunk
    "sphere3": lambda: M.Sphere(3),            # GS 1
    "knap": lambda: M.ReferenceKnapsack(),     # GS 2, reference E2
}


@pytest.fixture(autouse=True)
def _transposed_kernel_at_every_size(monkeypatch):
    # the engine routes small REAL populations to the generic kernel
    # (real_tp_min_population); the bit-exact tests below cover the transposed
    # kernel at small sizes too
    monkeypatch.setenv("PGA_TP_MIN_S", "0")


def _exact_pair(p, S, gens, **kw):
    g = pga.GeneticAlgorithm(p, S, device="cuda:0", **kw)
    c = pga.GeneticAlgorithm(p, S, device="cpu", **kw)
    for k in range(gens):
        g.run(1)
        c.run(1)
        torch.cuda.synchronize()
        assert torch.equal(g.rows.cpu(), c.rows), f"rows differ after generation {k + 1}"
        assert torch.equal(g.scores.cpu(), c.scores), f"scores differ after generation {k + 1}"
    assert close(p.reference_fitness(g.genomes().cpu()), g.scores.cpu())
    return g, c


@pytest.mark.gpu
@pytest.mark.parametrize("xo", ["uniform", "blend", "arithmetic", "one_point", "two_point", "none"])
@pytest.mark.parametrize("mut", ["gaussian", "uniform", "reset_one", "none"])
def test_gpu_tp_bitexact_operators(xo, mut):
    """Sphere-30 (the BASELINE config 3 geometry): every crossover x mutation,
    3 generations, children and scores bit for bit vs the CPU backend."""
    _exact_pair(M.Sphere(30), 3000, 3, seed=21, elitism=1, crossover=xo, mutation=mut)


@pytest.mark.gpu
@pytest.mark.parametrize("L", [33, 100, 128])
@pytest.mark.parametrize("mut", ["reset_one", "gaussian"])
def test_gpu_tp_uniform_crossover_block_in_record(L, mut):
    """UNIFORM crossover on 33..128 genes: a child without mutations carries
    its crossover block in the record (one Philox per child), a mutated one
    draws it per lane; both bit for bit vs the CPU backend (reference E1's
    operators at L = 100)."""
    _exact_pair(M.SumGenes(L), 3000, 3, seed=8, elitism=1, crossover="uniform", mutation=mut)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(EXACT))
def test_gpu_tp_bitexact_geometries(name):
    p = EXACT[name]()
    for mut in ("gaussian", "reset_one"):
        _exact_pair(p, 2500, 3, seed=5, elitism=3, crossover="blend", mutation=mut)


# rotated objectives with transcendental terms through the transposed kernel:
# the rotation is the CPU's fma chain bit for bit, the cos / exp terms agree to
# float rounding, so the rows stay the CPU's except where two contestants'
# scores lie within that rounding
ROTATED = {
    "rastrigin30_rot": lambda: M.Rastrigin(30, rotate=True, shift=True, seed=4),  # BASELINE config 3
    "griewank16_rot": lambda: M.Griewank(16, rotate=True, seed=9),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(ROTATED))
def test_gpu_tp_rotated_mfma_close(name):
    p = ROTATED[name]()
    g = pga.GeneticAlgorithm(p, 2500, seed=5, device="cuda:0", elitism=3, crossover="blend")
    c = pga.GeneticAlgorithm(p, 2500, seed=5, device="cpu", elitism=3, crossover="blend")
    for k in range(3):
        g.run(1)
        c.run(1)
        torch.cuda.synchronize()
        same = (g.rows.cpu() == c.rows).all(-1)
        assert same.float().mean().item() > 0.99, f"rows diverged after generation {k + 1}"
        assert close(g.scores.cpu()[same], c.scores[same], rel=1e-5, abs_=1e-4)
    assert close(p.reference_fitness(g.genomes().cpu()), g.scores.cpu(), rel=1e-4, abs_=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("sel", ["random", "rank", "tournament3", "roulette"])
def test_gpu_real_selections_bitexact(sel):
    """rank / random through the transposed kernel, tournament-3 through the
    generic one; roulette on integer scores (exact prefix sums)."""
    kw = dict(seed=8, elitism=1, crossover="two_point", mutation="gaussian")
    if sel == "tournament3":
        kw.update(selection="tournament", tournament_k=3)
    else:
        kw.update(selection=sel)
    p = M.ReferenceKnapsack() if sel == "roulette" else M.Rosenbrock(30)
    _exact_pair(p, 3000, 3, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("rate", [0.2, 0.06])
def test_gpu_real_dense_and_many_flips_bitexact(rate):
    """rate 0.2 (L p = 6): the dense per-chunk sampler; rate 0.06 (L p = 1.8
    > 1.5 too) and, below, 1.4/30: sparse with K > 3 continuing in the group."""
    _exact_pair(M.Sphere(30), 3000, 3, seed=3, elitism=1, crossover="blend", mutation="gaussian", mutation_rate=rate)
    _exact_pair(M.Sphere(30), 3000, 3, seed=4, elitism=1, crossover="uniform", mutation="uniform",
                mutation_rate=1.4 / 30)


@pytest.mark.gpu
def test_gpu_rastrigin30_tp_1m():
    """BASELINE config 3 (plain): pop 1M through real_gen_tp; rows from a
    shared population equal the CPU's, scores match the torch fp32 oracle."""
    p = M.Rastrigin(30)
    ga = pga.GeneticAlgorithm(p, 1 << 20, seed=1, device="cuda:0", elitism=1)
    b0 = ga.best_score()
    ga.run(20)
    torch.cuda.synchronize()
    idx = torch.randint(0, 1 << 20, (8192,), device="cuda:0")
    assert close(p.reference_fitness(ga.genomes()[idx]), ga.scores[idx], rel=1e-4, abs_=5e-3)
    assert ga.best_score() > b0
    s = ga.stats()
    assert s["min"] <= s["mean"] <= s["max"] == ga.best_score()


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
    """Sphere-1000 / sum-1024: the long-genome kernel's children and scores
    equal the CPU backend's bit for bit over several generations."""
    for p in (M.Sphere(1000), M.SumGenes(1024)):
        kw = dict(seed=13, elitism=1, crossover=xo, mutation=mut)
        g = pga.GeneticAlgorithm(p, 512, device="cuda:0", **kw)
        c = pga.GeneticAlgorithm(p, 512, device="cpu", **kw)
        g.run(3)
        c.run(3)
        torch.cuda.synchronize()
        # children bit for bit (gaussian too: real_ops.hpp gauss_z), scores too
        assert torch.equal(g.rows.cpu(), c.rows)
        assert torch.equal(g.scores.cpu(), c.scores)


def test_gauss_z_deterministic_normal():
    """The REAL gaussian mutation's Box-Muller (integer range reduction +
    fma polynomials, identical on host and device): close to the float64
    transform of the same words and N(0, 1) in distribution."""
    from libpga_amd._ext import C
    g = torch.Generator().manual_seed(0)
    w = torch.randint(0, 1 << 32, (200000, 2), generator=g, dtype=torch.int64)
    z = C.gauss_z_batch(w).double()
    u1 = ((w[:, 0] >> 8) + 1).double() / 16777216.0
    u2 = ((w[:, 1] >> 8) + 1).double() / 16777216.0
    ref = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * torch.pi * u2)
    assert float((z - ref).abs().max()) < 2e-5
    assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1.0) < 0.01
    k = float(((z - z.mean()) ** 4).mean() / z.var() ** 2)
    assert abs(k - 3.0) < 0.05  # kurtosis of a normal
    assert C.gauss_z(0xFFFFFFFF, 0) == 0.0 or abs(C.gauss_z(0xFFFFFFFF, 0)) < 1e-6  # u1 = 1: radius 0


def test_cpu_sparse_mutation_rate():
    """Sparse per-gene uniform mutation: mutated genes per child ~ Binomial(L, p)."""
    p = M.Sphere(30)
    ga = pga.GeneticAlgorithm(p, 4000, seed=11, device="cpu", crossover="none", mutation="uniform",
                              selection="random", mutation_rate=1.0 / 30)
    before = ga.genomes().clone()
    ga.run(1)
    after = ga.genomes()
    # with crossover none and random selection every child is a copy of some
    # parent plus its mutations: count genes that match no parent gene value
    vals = set(before.flatten().tolist())
    changed = sum(1 for x in after.flatten().tolist() if x not in vals)
    mean = changed / 4000
    assert 0.9 < mean < 1.1  # E[K] = L p = 1


@pytest.mark.gpu
def test_gpu_rank_order_large_population_bitexact():
    """Linear ranking on f32 scores at S = 300,007: the native radix sort runs
    4 passes of 8-bit digits over 74 tiles (a (digit, tile) table of 18,944
    entries: the two-level scan) and a partial last tile; the rank order, hence
    every child, equals the CPU backend's stable sort."""
    _exact_pair(M.Rosenbrock(30), 300_007, 2, seed=8, elitism=1, selection="rank", crossover="two_point",
                mutation="gaussian")


@pytest.mark.gpu
def test_gpu_small_population_generic_route_bitexact(monkeypatch):
    """The default route of a small REAL population (generic kernel) gives the
    CPU backend's children too."""
    monkeypatch.delenv("PGA_TP_MIN_S", raising=False)
    _exact_pair(M.Sphere(30), 3000, 3, seed=31, elitism=1, crossover="blend", mutation="gaussian")
    _exact_pair(M.SumGenes(100), 3000, 2, seed=32, crossover="uniform", mutation="reset_one")


# tiny populations (every child in one block): GA.run(n) is ONE launch of n
# generations (real.hip real_multi_kernel); rows and scores equal the CPU
# backend's after each multi-generation run
TINY = {
    "knap100": (lambda: M.ReferenceKnapsack(), 100),  # reference E2, GS 2
    "sphere3": (lambda: M.Sphere(3), 256),            # GS 1, the block's 256 groups
    "sum30": (lambda: M.SumGenes(30), 32),            # GS 8
    "rosen30": (lambda: M.Rosenbrock(30), 17),        # neighbour gene across lanes
    "sphere100": (lambda: M.Sphere(100), 8),          # GS 32
    "sphere256": (lambda: M.Sphere(256), 4),          # GS 64
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(TINY))
@pytest.mark.parametrize("kw", [dict(elitism=1), dict(elitism=0, tournament_k=3, mutation="reset_one"),
                                dict(elitism=1, selection="random", crossover="blend")])
def test_gpu_tiny_multi_generation_bitexact(name, kw, monkeypatch):
    monkeypatch.delenv("PGA_TP_MIN_S", raising=False)  # tiny populations: no quantized keys
    mk, S = TINY[name]
    p = mk()
    g = pga.GeneticAlgorithm(p, S, seed=5, device="cuda:0", **kw)
    c = pga.GeneticAlgorithm(p, S, seed=5, device="cpu", **kw)
    for n in (2, 7, 3):
        g.run(n)
        c.run(n)
        torch.cuda.synchronize()
        assert torch.equal(g.rows.cpu(), c.rows), f"rows differ after run({n})"
        assert torch.equal(g.scores.cpu(), c.scores), f"scores differ after run({n})"
    assert g.best_score() == c.best_score() and g.best_index() == c.best_index()
