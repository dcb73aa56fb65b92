"""BINARY encoding on the CPU reference backend (runs without a GPU)."""
import math

import pytest
import torch

import libpga_amd as pga
from libpga_amd import _C


def make(problem, S=256, seed=3, **kw):
    return pga.GeneticAlgorithm(problem, S, seed=seed, device="cpu", **kw)


@pytest.mark.parametrize("L", [1, 31, 64, 100, 128, 129, 1000, 1024, 9000])
def test_init_scores_match_oracle(L):
    ga = make(pga.models.OneMax(L), S=97)
    g = ga.genomes()
    assert g.shape == (97, L)
    assert torch.equal(ga.problem.reference_fitness(g), ga.scores)
    # padding bits are zero
    rw = ga.rows.shape[1]
    assert rw % 4 == 0
    full = pga.ops.decode(ga.rows, "binary", rw * 32)
    assert int(full[:, L:].sum()) == 0
    # roughly half the bits set
    assert abs(g.float().mean().item() - 0.5) < 0.1 + 2.0 / math.sqrt(97 * L)


def test_codec_roundtrip():
    g = torch.randint(0, 2, (13, 77), dtype=torch.uint8)
    rows = pga.ops.encode(g, "binary", 77, 4)
    assert torch.equal(pga.ops.decode(rows, "binary", 77), g)


@pytest.mark.parametrize("prob", ["onemax", "trap", "leading", "knapsack"])
@pytest.mark.parametrize("xo", ["uniform", "one_point", "two_point"])
def test_generation_scores_match_oracle(prob, xo):
    p = {
        "onemax": pga.models.OneMax(300),
        "trap": pga.models.Trap(256, 4),
        "leading": pga.models.LeadingOnes(200),
        "knapsack": pga.models.Knapsack01.random(150, seed=1),
    }[prob]
    ga = make(p, S=128, crossover=xo, elitism=1)
    ga.run(7)
    assert ga.generation == 7
    assert torch.allclose(p.reference_fitness(ga.genomes()), ga.scores, rtol=0, atol=1e-3)


def test_onemax_converges():
    ga = make(pga.models.OneMax(64), S=1024, elitism=1)
    s0 = ga.best_score()
    ga.run(60)
    assert ga.best_score() == 64.0 > s0


def test_elitism_monotone():
    ga = make(pga.models.Trap(128, 4), S=128, elitism=1)
    prev = ga.best_score()
    for _ in range(20):
        ga.run(1)
        cur = ga.best_score()
        assert cur >= prev
        prev = cur


def test_elitism_k_preserves_top():
    ga = make(pga.models.OneMax(200), S=300, elitism=5)
    top_scores, top_genomes = ga.top(5)
    ga.run(1)
    new = ga.genomes()[:5]
    # the elite set (children 0..E-1 in selection order, not necessarily best-first)
    key = lambda rows: sorted(tuple(r.tolist()) for r in rows)  # noqa: E731
    assert key(new) == key(top_genomes)
    assert sorted(ga.scores[:5].tolist()) == sorted(top_scores.tolist())


def test_determinism_and_seed():
    a = make(pga.models.OneMax(500), seed=11)
    b = make(pga.models.OneMax(500), seed=11)
    c = make(pga.models.OneMax(500), seed=12)
    for x in (a, b, c):
        x.run(5)
    assert torch.equal(a.rows, b.rows)
    assert not torch.equal(a.rows, c.rows)


def test_staged_equals_fused():
    """crossover_stage + mutate_stage + swap + evaluate == one fused generation
    (reference pga_run stage order, src/pga.cu:381-390)."""
    a = make(pga.models.OneMax(777), seed=5)
    b = make(pga.models.OneMax(777), seed=5)
    a.run(1)
    isl = b.island
    isl.crossover_stage()
    isl.mutate_stage()
    isl.swap()
    isl.evaluate()
    assert torch.equal(a.rows, b.rows)
    assert torch.equal(a.scores, b.scores)


@pytest.mark.parametrize("p", [0.01, 1.0 / 512])  # dense (per-chunk geometric) and sparse (Binomial) samplers
def test_mutation_rate_statistics(p):
    """Bit-flip at rate p: with crossover=none and random selection, a child
    differs from its parent in Binomial(L, p) bits."""
    L, S = 512, 4096
    ga = make(pga.models.OneMax(L), S=S, selection="random", crossover="none", mutation_rate=p)
    parents = ga.genomes().clone()
    ga.run(1)
    kids = ga.genomes()
    # parent A of child i is selection word 0: ST_SEL (8) block 0, register .x
    seed = 3
    idx = torch.tensor([(_C.philox(0 | (8 << 24), i, 0, 0, seed, 0)[0] * S) >> 32 for i in range(S)])
    nflip = (kids != parents[idx]).sum(-1).float()
    mean = nflip.mean().item()
    assert abs(mean - L * p) < 4 * math.sqrt(L * p * (1 - p) / S)
    var = nflip.var().item()
    assert abs(var - L * p * (1 - p)) < 0.25 * L * p


def test_topk_and_stats():
    ga = make(pga.models.OneMax(100), S=500)
    sc = ga.scores.clone()
    idx = ga.island.topk(17, True).long()
    ref = sorted(range(500), key=lambda i: (-sc[i].item(), i))[:17]
    assert idx.tolist() == ref
    low = ga.island.topk(9, False).long()
    ref = sorted(range(500), key=lambda i: (sc[i].item(), i))[:9]
    assert low.tolist() == ref
    st = ga.stats()
    assert st["max"] == sc.max().item() and st["min"] == sc.min().item()
    assert abs(st["mean"] - sc.mean().item()) < 1e-3


def test_roulette_runs_and_improves():
    ga = make(pga.models.OneMax(64), S=512, selection="roulette")
    m0 = ga.stats()["mean"]
    ga.run(30)
    assert ga.stats()["mean"] > m0 + 3


def test_tournament_k():
    ga = make(pga.models.OneMax(64), S=512, tournament_k=5)
    m0 = ga.stats()["mean"]
    ga.run(5)
    assert ga.stats()["mean"] > m0 + 5


def test_torch_objective():
    fn = lambda g: (g[:, ::2].float().sum(-1) - g[:, 1::2].float().sum(-1))  # noqa: E731
    p = pga.models.BinaryTorchObjective(64, fn, optimum=32)
    ga = make(p, S=512, elitism=1)
    ga.run(40)
    assert torch.equal(fn(ga.genomes()).float(), ga.scores)
    assert ga.best_score() >= 28


def test_checkpoint_resume_exact(tmp_path):
    a = make(pga.models.OneMax(300), seed=9)
    a.run(4)
    a.save(str(tmp_path / "c.ckpt"))
    a.run(6)
    b = make(pga.models.OneMax(300), seed=0)
    b.load(str(tmp_path / "c.ckpt"))
    assert b.generation == 4
    b.run(6)
    assert torch.equal(a.rows, b.rows) and torch.equal(a.scores, b.scores)


def test_philox_known_answer():
    # Random123 known-answer vector for philox4x32-10 (counter=0, key=0)
    assert _C.philox(0, 0, 0, 0, 0, 0) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    assert _C.philox(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF) == (
        0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)
    assert _C.philox(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344, 0xA4093822, 0x299F31D0) == (
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)


def _value_problem(L=24):
    """Individual value = its bits as an integer (exact in f32 for L <= 24)."""
    w = (2.0 ** torch.arange(L)).float()
    return pga.models.BinaryTorchObjective(L, lambda g: g.float() @ w)


def _set_population(ga, genomes):
    ga.island.rows(0).copy_(ga.problem.encode(genomes, int(ga.island.row_words)))
    ga._custom_eval()


def test_tournament_selection_pressure():
    """Tournament-k with distinct scores: a copied parent's rank u = r/S has
    E[u] = k/(k+1) (P(u <= x) = x^k); binary tournament -> 2/3."""
    S, L = 4096, 24
    for k in (2, 4):
        ga = make(_value_problem(L), S=S, tournament_k=k, crossover="none", mutation="none")
        vals = torch.randperm(S)
        bits = ((vals[:, None] >> torch.arange(L)) & 1).to(torch.uint8)
        _set_population(ga, bits)
        ga.run(1)
        u = ga.scores.double() / (S - 1)
        exp, sd = k / (k + 1), math.sqrt(k / ((k + 2) * (k + 1) ** 2))
        assert abs(u.mean().item() - exp) < 5 * sd / math.sqrt(S), (k, u.mean().item())


def test_uniform_crossover_bit_balance():
    """Uniform crossover of an all-zeros and an all-ones parent gives each bit
    from either parent with probability 1/2, independently."""
    S, L = 4096, 256
    ga = make(pga.models.OneMax(L), S=S, selection="random", crossover="uniform", mutation="none")
    bits = torch.zeros(S, L, dtype=torch.uint8)
    bits[S // 2:] = 1
    ga.island.rows(0).copy_(ga.problem.encode(bits, int(ga.island.row_words)))
    ga.evaluate()
    ga.run(1)
    ones = ga.scores
    mixed = (ones > 0) & (ones < L)  # children of one zeros- and one ones-parent (whp)
    frac = mixed.float().mean().item()
    assert abs(frac - 0.5) < 0.05  # P(parents differ) = 1/2
    m = ones[mixed].double()
    assert abs(m.mean().item() - L / 2) < 5 * math.sqrt(L / 4 / m.numel())
    assert abs(m.var().item() - L / 4) < 0.15 * L / 4
    g = ga.genomes()[mixed].double()
    per_bit = g.mean(0)  # every position balanced
    assert (per_bit - 0.5).abs().max().item() < 6 * math.sqrt(0.25 / g.shape[0])


@pytest.mark.parametrize("sp", [1.0, 1.5, 2.0])
def test_rank_selection_pressure(sp):
    """Linear ranking with distinct scores: a copied parent's rank r has
    P(r) = (2-sp)/S + (sp-1)(2r+1)/S^2 exactly (core.hpp rank_pick)."""
    S, L = 4096, 24
    ga = make(_value_problem(L), S=S, selection="rank", rank_pressure=sp, crossover="none", mutation="none")
    vals = torch.randperm(S)
    bits = ((vals[:, None] >> torch.arange(L)) & 1).to(torch.uint8)
    _set_population(ga, bits)
    ga.run(1)
    r = torch.arange(S, dtype=torch.float64)
    pmf = (2 - sp) / S + (sp - 1) * (2 * r + 1) / S ** 2
    assert abs(pmf.sum().item() - 1) < 1e-12
    mean = (pmf * r).sum().item()
    sd = math.sqrt((pmf * (r - mean) ** 2).sum().item())
    got = ga.scores.double()
    assert abs(got.mean().item() - mean) < 5 * sd / math.sqrt(S), (sp, got.mean().item(), mean)
    # the best individual is copied sp times on average
    top = (got == S - 1).double().sum().item()
    assert abs(top - sp) < 6 * math.sqrt(sp) + 1


def test_rank_selection_converges_and_is_deterministic():
    runs = []
    for _ in range(2):
        ga = make(pga.models.OneMax(64), S=512, selection="rank", rank_pressure=2.0, elitism=1)
        ga.run(60)
        runs.append(ga.scores.clone())
    assert torch.equal(runs[0], runs[1])
    assert runs[0].max().item() == 64.0
    with pytest.raises(Exception):
        make(pga.models.OneMax(64), S=64, selection="rank", rank_pressure=2.5)


def test_worker_pool_exceptions():
    """A throwing slot of the CPU worker pool (csrc/cpu/parallel.cpp) surfaces
    as one exception on the caller after every slot finished, on the caller's
    slot and on a worker's alike, and the pool keeps working afterwards."""
    from libpga_amd import _C
    n = 4096
    assert _C._pool_sum(n, n) == n * (n - 1) // 2
    for bad in (0, n - 1, n // 2):
        with pytest.raises(RuntimeError, match="slot failed"):
            _C._pool_sum(n, bad)
        assert _C._pool_sum(n, n) == n * (n - 1) // 2


def test_torch_objective_history():
    """History rows of a torch-objective run are the statistics of the scores
    that objective produced (rows appended after its evaluation), one per
    generation, equal to stats() taken after every step."""
    fn = lambda g: (g[:, ::2].float().sum(-1) - g[:, 1::2].float().sum(-1))  # noqa: E731
    ga = make(pga.models.BinaryTorchObjective(64, fn, optimum=32), S=256, elitism=1)
    ga.record_history()
    want = []
    for _ in range(5):
        ga.step()
        s = ga.stats()
        want.append([s["min"], s["max"], s["mean"]])
    h = ga.history()
    assert h.shape == (5, 4)
    assert torch.allclose(h[:, :3], torch.tensor(want), rtol=1e-6, atol=1e-5)
    assert torch.all(h[:, 3] == 256)
