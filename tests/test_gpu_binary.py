"""gfx950 BINARY kernels vs the CPU reference backend (bit-exact) and the
plain-PyTorch fp32 fitness oracle."""
import pytest
import torch

import libpga_amd as pga

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def pair(problem, S, seed=21, **kw):
    g = pga.GeneticAlgorithm(problem, S, seed=seed, device=DEV, **kw)
    c = pga.GeneticAlgorithm(problem, S, seed=seed, device="cpu", **kw)
    return g, c


def same(g, c):
    torch.cuda.synchronize()
    assert torch.equal(g.rows.cpu(), c.rows), "rows differ"
    assert torch.equal(g.scores.cpu(), c.scores), "scores differ"


def test_extension_is_native():
    import libpga_amd._C as C

    assert C.__file__.endswith("_C.so")
    ga = pga.GeneticAlgorithm(pga.models.OneMax(64), 64, device=DEV)
    assert ga.island.on_gpu


@pytest.mark.parametrize("L", [1, 64, 100, 128, 1000, 1024, 4096, 9000])
@pytest.mark.parametrize("S", [1, 77, 4096])
def test_init_bitexact(L, S):
    g, c = pair(pga.models.OneMax(L), S)
    same(g, c)


@pytest.mark.parametrize("L", [64, 1024, 3000, 9000])
@pytest.mark.parametrize("xo", ["uniform", "one_point", "two_point", "none"])
@pytest.mark.parametrize("elitism", [0, 1, 3])
def test_generations_bitexact(L, xo, elitism):
    g, c = pair(pga.models.OneMax(L), 1000, crossover=xo, elitism=elitism, crossover_prob=0.8)
    g.run(3)
    c.run(3)
    same(g, c)
    assert g.best_score() == c.best_score()


@pytest.mark.parametrize("prob", ["trap", "leading", "knapsack"])
def test_objectives_bitexact(prob):
    p = {
        "trap": pga.models.Trap(512, 8),
        "leading": pga.models.LeadingOnes(300),
        "knapsack": pga.models.Knapsack01.random(700, seed=2),
    }[prob]
    g, c = pair(p, 513, elitism=1, tournament_k=3)
    g.run(4)
    c.run(4)
    same(g, c)
    ref = p.reference_fitness(g.genomes().cpu())
    assert torch.allclose(ref, g.scores.cpu(), rtol=0, atol=1e-2)


@pytest.mark.parametrize("L,scale,digits", [(1024, 1, 1), (700, 1, 1), (300, 1, 1), (2000, 1, 1), (3000, 1, 1),
                                             (1024, 250, 2), (1024, "big", 3), (1024, -1, 1), (1024, 0.5, 0),
                                             (200, 1, 0)])
def test_knapsack_matrix_cores_bitexact(L, scale, digits):
    """Knapsack evaluated on the int8 matrix cores in the hot kernel (tournament
    2): bit-exact against the CPU's float sums for integer instances (1-3
    balanced base-256 digits, negative values), and the scalar evaluation for
    non-integer instances or genomes of fewer than 4 lanes (digits 0)."""
    base = pga.models.Knapsack01.random(L, seed=3)
    v, w = base.values.clone(), base.weights.clone()
    if scale == -1:
        v = v - 50  # negative values
    elif scale == "big":
        v[:3] = torch.tensor([5e6, 3e6, 1e6])  # 3 digits, sums still below 2^24
    else:
        v = v * scale
    p = pga.models.Knapsack01(v, w, base.capacity)
    g, c = pair(p, 2500, elitism=1)
    for _ in range(3):
        g.run(1)
        c.run(1)
        same(g, c)
    assert g.island.knapsack_digits == digits
    ref = p.reference_fitness(g.genomes().cpu())
    assert torch.allclose(ref, g.scores.cpu(), rtol=1e-6, atol=1e-2)


@pytest.mark.parametrize("S,L,sel,elitism", [(1048576, 1024, "tournament", 1), (1048576, 1024, "rank", 3),
                                              (1600000, 1024, "tournament", 3), (1600000, 1024, "rank", 1),
                                              (1047576, 1024, "rank", 1),
                                              (1048576, 1024, "roulette", 1), (700001, 300, "roulette", 2),
                                              (1900000, 256, "tournament", 1), (300000, 64, "roulette", 1),
                                              (200000, 1024, "tournament", 2)])
def test_headline_geometry_bitexact(S, L, sel, elitism):
    """The hot kernel at the headline geometry, rows and scores against the
    CPU backend over 2 generations: one 16-wave block per CU with ~16 batches
    pulled per block (1M), 24 batches per block (1.6M), a block share above
    one round's parent capacity (1.9M x 256 bits: two tournament / breed
    rounds per block), and the 4-wave occupancy grid (200K).  Roulette runs
    OneMax-64 so that the f32 prefix sums stay exact (< 2^24)."""
    kw = dict(rank_pressure=1.7) if sel == "rank" else {}
    g, c = pair(pga.models.OneMax(L), S, seed=5, selection=sel, elitism=elitism, **kw)
    for _ in range(2):
        g.run(1)
        c.run(1)
        same(g, c)
    assert g.best_score() == c.best_score()


@pytest.mark.parametrize("mut", [("bit_flip", 0.0), ("bit_flip", 0.05), ("bit_flip", 1.0), ("reset_one", 0.3)])
def test_mutation_modes_bitexact(mut):
    name, rate = mut
    g, c = pair(pga.models.OneMax(300), 400, mutation=name, mutation_rate=rate)
    g.run(2)
    c.run(2)
    same(g, c)


@pytest.mark.parametrize("L,S,rate", [(1000, 100000, 0.0015), (64, 20000, 1.5 / 64), (8192, 3000, None), (200, 5000, None)])
def test_sparse_mutation_bitexact(L, S, rate):
    """Sparse bit-flip sampler (L*p <= 1.5): the transposed kernel's record
    positions, its sequential fallback and the K > 8 group continuation (about
    3 children per generation at S=100000, L*p=1.5) against the CPU."""
    kw = {} if rate is None else {"mutation_rate": rate}
    g, c = pair(pga.models.OneMax(L), S, elitism=1, **kw)
    g.run(2)
    c.run(2)
    same(g, c)


def test_staged_equals_fused_gpu():
    a = pga.GeneticAlgorithm(pga.models.OneMax(1024), 2048, seed=4, device=DEV)
    b = pga.GeneticAlgorithm(pga.models.OneMax(1024), 2048, seed=4, device=DEV)
    a.run(1)
    isl = b.island
    isl.crossover_stage()
    isl.mutate_stage()
    isl.swap()
    isl.evaluate()
    torch.cuda.synchronize()
    assert torch.equal(a.rows, b.rows) and torch.equal(a.scores, b.scores)


@pytest.mark.parametrize("S,k", [(1000, 1), (1000, 10), (100000, 1000), (1 << 20, 10486)])
def test_topk_matches_cpu(S, k):
    ga = pga.GeneticAlgorithm(pga.models.OneMax(64), S, seed=1, device=DEV)
    sc = ga.scores.cpu()
    for largest in (True, False):
        idx = ga.island.topk(k, largest).cpu().long()
        key = -sc if largest else sc
        order = torch.from_numpy(__import__("numpy").lexsort((torch.arange(S).numpy(), key.numpy())))
        assert torch.equal(idx, order[:k])


def test_stats_and_best():
    ga = pga.GeneticAlgorithm(pga.models.OneMax(1024), 100000, seed=2, device=DEV)
    sc = ga.scores.cpu()
    st = ga.stats()
    assert st["max"] == sc.max().item() and st["min"] == sc.min().item()
    assert abs(st["mean"] - sc.double().mean().item()) < 1e-2
    s, i = ga.island.best()
    assert s == sc.max().item() and i == int((sc == sc.max()).nonzero()[0])


def test_roulette_gpu_improves():
    ga = pga.GeneticAlgorithm(pga.models.OneMax(256), 65536, seed=2, device=DEV, selection="roulette")
    m0 = ga.stats()["mean"]
    ga.run(20)
    assert ga.stats()["mean"] > m0 + 5


def test_gather_scatter_gpu():
    ga = pga.GeneticAlgorithm(pga.models.OneMax(1024), 5000, seed=2, device=DEV)
    isl = ga.island
    idx = torch.tensor([5, 17, 4999, 0], dtype=torch.int32, device=DEV)
    rows = torch.empty(4 * isl.row_words, dtype=torch.int32, device=DEV)
    sc = torch.empty(4, dtype=torch.float32, device=DEV)
    isl.gather(idx, rows, sc)
    assert torch.equal(rows.view(4, -1), ga.rows[idx.long()])
    assert torch.equal(sc, ga.scores[idx.long()])
    dst = torch.tensor([1, 2, 3, 4], dtype=torch.int32, device=DEV)
    isl.scatter(dst, rows, sc)
    assert torch.equal(ga.rows[1:5], rows.view(4, -1))


def test_headline_config_converges():
    """1M x 1024-bit OneMax: fused kernel scores == popcount oracle."""
    ga = pga.GeneticAlgorithm(pga.models.OneMax(1024), 1 << 20, seed=3, device=DEV, elitism=1)
    b0 = ga.best_score()
    ga.run(50)
    torch.cuda.synchronize()
    ref = ga.problem.reference_fitness(ga.genomes())
    assert torch.equal(ref, ga.scores)
    assert ga.best_score() > b0 + 20


@pytest.mark.gpu
@pytest.mark.parametrize("problem", ["onemax", "knapsack_like"])
@pytest.mark.parametrize("sorted_", [True, False])
def test_gpu_topk_matches_cpu(problem, sorted_):
    """Device top-k (u16-key path for integer objectives, f32 path otherwise),
    sorted and selection order, equals the CPU backend's."""
    S = 200_000
    p = pga.models.OneMax(300) if problem == "onemax" else pga.models.Rastrigin(12)
    g = pga.GeneticAlgorithm(p, S, seed=5, device="cuda:0", elitism=1)
    c = pga.GeneticAlgorithm(p, S, seed=5, device="cpu", elitism=1)
    g.run(3)
    c.run(3)
    torch.cuda.synchronize()
    if problem == "onemax":
        assert torch.equal(g.scores.cpu(), c.scores)
    else:  # REAL rows can differ by ulps: use the GPU scores on both sides
        c.island.scores(0).copy_(g.scores.cpu())
    for k in (1, 7, 2000, 10486):
        for largest in (True, False):
            a = g.island.topk(k, largest, sorted_).cpu()
            b = c.island.topk(k, largest, sorted_)
            assert torch.equal(a, b), (k, largest, sorted_)


@pytest.mark.parametrize("sp", [1.25, 2.0])
def test_rank_selection_bitexact(sp):
    """Device rank order (native stable LSD radix sort of score keys) + integer
    rank sampling reproduce the CPU backend bit for bit, ties included."""
    g, c = pair(pga.models.OneMax(300), 5000, selection="rank", rank_pressure=sp, elitism=2)
    g.run(4)
    c.run(4)
    same(g, c)


@pytest.mark.parametrize("prob", ["onemax1024", "onemax100", "knapsack_real"])
@pytest.mark.parametrize("elitism", [1, 3])
@pytest.mark.parametrize("sel", ["rank", "roulette"])
def test_rank_roulette_fast_kernel_bitexact(prob, elitism, sel):
    """Linear ranking (two rank picks, two rank-order loads per child) and
    roulette (guide table: one guide + one cumfit load per pick) in the fast kernel's
    first phase: u16-key objectives at full and partial lane groups, and an
    f32-score objective (non-integer knapsack), bit-exact vs the CPU backend."""
    g0 = torch.Generator().manual_seed(3)
    problem = {"onemax1024": lambda: pga.models.OneMax(1024), "onemax100": lambda: pga.models.OneMax(100),
               "knapsack_real": lambda: pga.models.Knapsack01(torch.rand(256, generator=g0) * 10,
                                                            torch.rand(256, generator=g0) * 10, 300.0)}[prob]()
    kw = dict(rank_pressure=1.7) if sel == "rank" else {}
    g, c = pair(problem, 3000, selection=sel, elitism=elitism, **kw)
    if sel == "roulette" and prob == "knapsack_real":
        # non-integer scores: the device prefix sums (parallel scan) round
        # differently from the CPU's sequential ones, so picks near a bucket
        # edge may differ; the GPU run is checked against the torch oracle
        g.run(3)
        torch.cuda.synchronize()
        ref = problem.reference_fitness(g.genomes().cpu())
        assert torch.allclose(ref, g.scores.cpu(), rtol=1e-5, atol=1e-3)
        return
    for _ in range(3):
        g.run(1)
        c.run(1)
        same(g, c)


@pytest.mark.gpu
@pytest.mark.parametrize("heavy", [0, 1 << 20])
def test_roulette_guide_table_heavy_tail(heavy):
    """Roulette picks through the guide table equal the CPU's binary search
    on integer-valued scores (exact prefix sums), also when one individual
    holds half the weight (its bucket span goes through the long-span list)
    and when most weights are zero (long runs of equal cumfit)."""
    S = 65536
    g, c = pair(pga.models.OneMax(64), S, seed=9, selection="roulette", elitism=1)
    gen = torch.Generator().manual_seed(5)
    sc = torch.randint(0, 16, (S,), generator=gen).float()
    sc[torch.rand(S, generator=gen) < 0.6] = 0.0  # 60% zero weight (min 0)
    sc[1234] = float(heavy) if heavy else sc[1234]
    for ga in (g, c):
        ga.scores.copy_(sc.to(ga.scores.device))
        ga.island.rebest()
    g.run(1)
    c.run(1)
    same(g, c)


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1 << 20, (1 << 22) + 12345])
def test_gpu_topk_selection_order_many_blocks(S):
    """u16-key top-k in selection order (the migration path: histogram + one
    fused look-back select launch) over up to 1024 blocks, repeated so the
    histogram / ticket reset between calls is exercised: the indices with a
    key beyond the threshold in population order, then the first ties."""
    ga = pga.GeneticAlgorithm(pga.models.OneMax(64), S, seed=11, device=DEV)
    sc = ga.scores.cpu()
    for k in (10486, 1, S // 3, 10486):
        for largest in (True, False):
            got = ga.island.topk(k, largest, False).cpu().long()
            key = sc if largest else -sc
            T = key.sort(descending=True).values[k - 1]
            gt = (key > T).nonzero().flatten()
            eq = (key == T).nonzero().flatten()[: k - gt.numel()]
            assert torch.equal(got, torch.cat([gt, eq])), (k, largest)


@pytest.mark.parametrize("S", [5000, 300000])
def test_topk_keys_above_range(S):
    """Scores outside the objective's range (a checkpoint's or an unvalidated
    migrant's) reach the u16-key top-k: every pass clamps the key to the
    histogram's top bin, so the selection stays exactly k distinct indices."""
    L = 64
    ga = pga.GeneticAlgorithm(pga.models.OneMax(L), S, seed=5, device=DEV)
    isl = ga.island
    forged = torch.tensor([3, 17, S // 2, S - 1], dtype=torch.int32, device=DEV)
    rows = torch.empty((forged.numel(), isl.row_words), dtype=torch.int32, device=DEV)
    sc = torch.empty(forged.numel(), dtype=torch.float32, device=DEV)
    isl.gather(forged, rows, sc)
    isl.scatter(forged, rows, torch.tensor([5000.0, 70.0, 1e9, float("nan")], device=DEV))
    torch.cuda.synchronize()
    for k in (1, 3, 10, 257):
        top = isl.topk(k, True).cpu().tolist()
        assert len(top) == k and len(set(top)) == k and all(0 <= i < S for i in top)
        if k >= 3:  # the three finite forged scores clamp to the top bin (no true score reaches L here)
            assert {3, 17, S // 2} <= set(top)
        low = isl.topk(k, False).cpu().tolist()
        assert len(low) == k and len(set(low)) == k and all(0 <= i < S for i in low)


@pytest.mark.parametrize("S,k", [(5000, 50), (1 << 20, 10486)])
def test_fused_migration_matches_unfused(S, k):
    """Island.emigrate / immigrate (selection kernel with the row gather /
    scatter fused in) == topk + gather / topk + scatter, bit for bit, and the
    victims' tournament keys follow their new scores."""
    kw = dict(seed=9, device=DEV, elitism=1)
    a = pga.GeneticAlgorithm(pga.models.OneMax(1024), S, **kw)
    b = pga.GeneticAlgorithm(pga.models.OneMax(1024), S, **kw)
    a.run(3)
    b.run(3)
    ia, ib = a.island, b.island
    ia.migration_policy = pga._ext.C.MIG_TOPK
    rw = int(ia.row_words)
    ra, sa = torch.empty(k * rw, dtype=torch.int32, device=DEV), torch.empty(k, device=DEV)
    rb, sb = torch.empty_like(ra), torch.empty_like(sa)
    ia.emigrate(k, ra, sa)
    ib.gather(ib.topk(k, True, False), rb, sb)
    torch.cuda.synchronize()
    assert torch.equal(ra, rb) and torch.equal(sa, sb)
    # immigrants: another island's best rows replace the worst
    c = pga.GeneticAlgorithm(pga.models.OneMax(1024), S, seed=10, device=DEV, elitism=1)
    c.run(5)
    rc, sc = torch.empty_like(ra), torch.empty_like(sa)
    c.island.emigrate(k, rc, sc)
    ia.immigrate(k, rc, sc)
    ib.scatter(ib.topk(k, False, False), rc, sc)
    torch.cuda.synchronize()
    assert torch.equal(a.rows, b.rows) and torch.equal(a.scores, b.scores)
    assert a.best_score() == b.best_score()
    a.run(2)
    b.run(2)  # identical keys => identical tournaments
    torch.cuda.synchronize()
    assert torch.equal(a.rows, b.rows) and torch.equal(a.scores, b.scores)


def stripe_reference(scores, rows, k):
    """Plain-torch MIG_STRIPE: per stripe [i*S//k, (i+1)*S//k) the best
    (ties: lowest index) and the worst (ties: lowest index)."""
    S = scores.numel()
    best, worst = [], []
    for i in range(k):
        lo, hi = i * S // k, (i + 1) * S // k
        s = scores[lo:hi].double()
        best.append(lo + int(torch.nonzero(s == s.max())[0]))
        worst.append(lo + int(torch.nonzero(s == s.min())[0]))
    return best, worst


@pytest.mark.parametrize("S,k", [(5000, 50), (100003, 997)])
@pytest.mark.parametrize("prob", ["onemax", "knapsack"])
def test_stripe_migration_gpu(S, k, prob):
    """Stripe policy (opt-in; exact top-k is the default): GPU == CPU
    backend bit for bit, == the torch reference, and the immigrate kernel's
    fused best partials and statistics describe the new population exactly."""
    p = pga.models.OneMax(1024) if prob == "onemax" else pga.models.Knapsack01.random(700, seed=4)
    g, c = pair(p, S, elitism=1)
    g.run(3)
    c.run(3)
    same(g, c)
    gi, ci = g.island, c.island
    assert gi.migration_policy == pga._ext.C.MIG_TOPK  # the default
    gi.migration_policy = ci.migration_policy = pga._ext.C.MIG_STRIPE
    rw = int(gi.row_words)
    out_g = torch.empty(k * rw, dtype=torch.int32, device=DEV), torch.empty(k, device=DEV)
    out_c = torch.empty(k * rw, dtype=torch.int32), torch.empty(k)
    gi.emigrate(k, *out_g)
    ci.emigrate(k, *out_c)
    torch.cuda.synchronize()
    assert torch.equal(out_g[0].cpu(), out_c[0]) and torch.equal(out_g[1].cpu(), out_c[1])
    best, worst = stripe_reference(c.scores, c.rows, k)
    assert torch.equal(out_c[1], c.scores[best])
    assert torch.equal(out_c[0].view(k, rw), c.rows[best])
    # immigrants: another island's emigrants replace each stripe's worst
    d = pga.GeneticAlgorithm(p, S, seed=77, device="cpu", elitism=1)
    d.run(4)
    inc = torch.empty(k * rw, dtype=torch.int32), torch.empty(k)
    d.island.emigrate(k, *inc)
    expect_rows, expect_scores = c.rows.clone(), c.scores.clone()
    expect_rows[worst] = inc[0].view(k, rw)
    expect_scores[worst] = inc[1]
    gi.immigrate(k, inc[0].to(DEV), inc[1].to(DEV))
    ci.immigrate(k, *inc)
    torch.cuda.synchronize()
    assert torch.equal(c.rows, expect_rows) and torch.equal(c.scores, expect_scores)
    same(g, c)
    assert g.best_score() == c.best_score() == float(expect_scores.max())
    assert g.island.best()[1] == int(torch.nonzero(expect_scores == expect_scores.max())[0])
    st = g.stats()
    assert st["min"] == float(expect_scores.min()) and st["max"] == float(expect_scores.max())
    assert st["mean"] == pytest.approx(float(expect_scores.double().mean()), rel=1e-5)
    g.run(2)
    c.run(2)  # keys of the replaced individuals follow their scores
    same(g, c)


@pytest.mark.gpu
def test_rank_selection_u16_keys_partial_tile_bitexact():
    """OneMax rank selection sorts the u16 tournament keys (2 passes, 6 + 5
    bits for L = 1024) over a population that is not a multiple of the
    4096-key tile: children equal the CPU backend's."""
    p = pga.models.OneMax(1024)
    kw = dict(seed=13, elitism=1, selection="rank")
    g = pga.GeneticAlgorithm(p, 70_001, device="cuda:0", **kw)
    c = pga.GeneticAlgorithm(p, 70_001, device="cpu", **kw)
    for _ in range(3):
        g.run(1)
        c.run(1)
        torch.cuda.synchronize()
        assert torch.equal(g.rows.cpu(), c.rows)
        assert torch.equal(g.scores.cpu(), c.scores)


@pytest.mark.gpu
@pytest.mark.parametrize("L,S", [(300, 9000), (2000, 5000), (1500, 20_000)])
def test_rank_selection_single_pass_widths(L, S):
    """The single-pass rank order (digit = the whole u16 key, 9..11 bits;
    L = 2000 needs more than 64 KiB of dynamic LDS in the 16-wave scatter)
    against the CPU backend over partial tiles."""
    p = pga.models.OneMax(L)
    kw = dict(seed=3, elitism=1, selection="rank", rank_pressure=1.8)
    g = pga.GeneticAlgorithm(p, S, device="cuda:0", **kw)
    c = pga.GeneticAlgorithm(p, S, device="cpu", **kw)
    for _ in range(3):
        g.run(1)
        c.run(1)
        torch.cuda.synchronize()
        assert torch.equal(g.rows.cpu(), c.rows)
        assert torch.equal(g.scores.cpu(), c.scores)


@pytest.mark.parametrize("S", [4099, 1 << 20, (1 << 22) + 12345])
@pytest.mark.parametrize("dist", ["ties", "spread"])
def test_gpu_topk32_selection_order(S, dist):
    """f32-score top-k in selection order (3 radix digits + one ticketed
    select, topk32_*): the indices with a score beyond the threshold in
    population order, then the first ties; heavy ties, +-inf and a negative
    zero included; repeated so the histogram / state / ticket reset between
    calls is exercised."""
    ga = pga.GeneticAlgorithm(pga.models.Rastrigin(8), S, seed=11, device=DEV)
    g = torch.Generator().manual_seed(S)
    if dist == "ties":  # a converged population: few distinct values sharing their high bits
        sc = -(100.0 + torch.randint(0, 7, (S,), generator=g).float() * 2 ** -10)
    else:
        sc = torch.randn(S, generator=g) * 1e3
    sc[5], sc[S // 2], sc[7] = float("inf"), float("-inf"), -0.0
    ga.scores.copy_(sc.to(DEV))
    ga.island.rebest()
    key_src = sc.double()
    for k in (10486 % S, 1, S // 3, 10486 % S, S):
        k = max(1, k)
        for largest in (True, False):
            got = ga.island.topk(k, largest, False).cpu().long()
            key = key_src if largest else -key_src
            T = key.sort(descending=True).values[k - 1]
            gt = (key > T).nonzero().flatten()
            eq = (key == T).nonzero().flatten()[: k - gt.numel()]
            assert torch.equal(got, torch.cat([gt, eq])), (k, largest)


@pytest.mark.parametrize("S,k", [(5000, 50), (1 << 20, 10486)])
@pytest.mark.parametrize("prob", ["rastrigin", "tsp"])
def test_fused_migration_matches_unfused_f32(S, k, prob):
    """f32-score islands (REAL, PERMUTATION): Island.emigrate / immigrate
    (the radix select with the row gather / scatter and the new best partials
    fused in) == topk + gather / topk + scatter + best pass, bit for bit."""
    mk = {"rastrigin": lambda: pga.models.Rastrigin(30),
          "tsp": lambda: pga.models.TSP.random_euclidean(64, seed=2)}[prob]
    S = S if prob == "rastrigin" else min(S, 1 << 18)
    kw = dict(seed=9, device=DEV, elitism=1)
    a, b = pga.GeneticAlgorithm(mk(), S, **kw), pga.GeneticAlgorithm(mk(), S, **kw)
    a.run(3)
    b.run(3)
    ia, ib = a.island, b.island
    ia.migration_policy = pga._ext.C.MIG_TOPK
    rw = int(ia.row_words)
    ra, sa = torch.empty(k * rw, dtype=torch.int32, device=DEV), torch.empty(k, device=DEV)
    rb, sb = torch.empty_like(ra), torch.empty_like(sa)
    ia.emigrate(k, ra, sa)
    ib.gather(ib.topk(k, True, False), rb, sb)
    torch.cuda.synchronize()
    assert torch.equal(ra, rb) and torch.equal(sa, sb)
    c = pga.GeneticAlgorithm(mk(), S, seed=10, device=DEV, elitism=1)
    c.run(5)
    rc, sc = torch.empty_like(ra), torch.empty_like(sa)
    c.island.emigrate(k, rc, sc)
    ia.immigrate(k, rc, sc)
    ib.scatter(ib.topk(k, False, False), rc, sc)
    torch.cuda.synchronize()
    assert torch.equal(a.rows, b.rows) and torch.equal(a.scores, b.scores)
    assert a.best_score() == b.best_score() and a.best_index() == b.best_index()
    a.run(2)
    b.run(2)
    torch.cuda.synchronize()
    assert torch.equal(a.rows, b.rows) and torch.equal(a.scores, b.scores)


@pytest.mark.parametrize("S,L,mut", [(1 << 20, 1024, "bit_flip"), (300_000, 512, "bit_flip"), (400_000, 100, "reset_one")])
def test_persistent_multi_generation_bitexact(S, L, mut):
    """Island.run(n) at the headline geometry takes ONE persistent launch of n
    generations (binary_gen_tp_multi: device-wide barrier between them):
    rows, scores and the best equal n plain launches (PGA_TP_MULTI=0 path
    inside one process is not switchable, so: the CPU backend) bit for bit,
    also at partial lane groups (L = 100) and with the fused key histogram
    the island model turns on (its top-k then matches the CPU's)."""
    g, c = pair(pga.models.OneMax(L), S, seed=13, elitism=1, mutation=mut)
    g.island.persistent = True  # (off by default: measured slower)
    g.island.fused_histogram = True
    g.run(5)
    c.run(5)
    same(g, c)
    assert g.best_score() == c.best_score() and g.generation == c.generation == 5
    assert g.island.fused_histogram_ready
    for largest in (True, False):
        assert torch.equal(g.island.topk(777, largest, False).cpu(), c.island.topk(777, largest, False))
    g.run(1)  # a single generation: the plain launch after the persistent one
    c.run(1)
    g.run(3)
    c.run(3)
    same(g, c)
