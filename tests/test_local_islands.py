"""Single-device island model (LocalIslands): migration semantics on the CPU
backend, stream-concurrent evolution bit-identical to serial on the GPU."""
import pytest
import torch

import libpga_amd as pga
from libpga_amd.parallel import LocalIslands


def stripe_best(scores, k):
    S = scores.numel()
    out = []
    for i in range(k):
        lo, hi = i * S // k, (i + 1) * S // k
        s = scores[lo:hi]
        out.append(lo + int(torch.nonzero(s == s.max())[0]))
    return torch.tensor(out)


@pytest.mark.parametrize("policy", ["stripe", "topk"])
def test_local_islands_ring_migration_cpu(policy):
    li = LocalIslands(pga.models.OneMax(100), 4, 200, seed=3, device="cpu", migrate_every=5, migrate_pct=0.05,
                      policy=policy)
    li.run(4)
    tops = []
    for ga in li.islands:
        idx = ga.island.topk(li.k, True).long() if policy == "topk" else stripe_best(ga.scores, li.k)
        tops.append(ga.rows.clone()[idx])
    li.migrate()
    assert li.migrations == 1
    for i, ga in enumerate(li.islands):
        src = tops[(i - 1) % 4]
        have = {tuple(r.tolist()) for r in ga.rows}
        assert all(tuple(r.tolist()) in have for r in src)
    li.run(31)  # generations 5, 10, ..., 35 migrate
    s, isl, g = li.best()
    assert s == float(g.sum()) and li.migrations == 8 and li.generation == 35


def test_local_islands_random_topology_cpu():
    li = LocalIslands(pga.models.OneMax(64), 3, 100, seed=1, device="cpu", migrate_every=3, topology="random")
    li.run(12)
    assert li.migrations == 4


@pytest.mark.gpu
def test_local_islands_streams_match_serial_gpu():
    kw = dict(seed=7, device="cuda:0", migrate_every=4, migrate_pct=0.02)
    a = LocalIslands(pga.models.OneMax(256), 6, 3000, **kw)
    b = LocalIslands(pga.models.OneMax(256), 6, 3000, **kw)
    b.streams = None  # serial on the default stream
    a.run(21)
    b.run(21)
    torch.cuda.synchronize()
    for x, y in zip(a.islands, b.islands):
        assert torch.equal(x.rows, y.rows) and torch.equal(x.scores, y.scores)
    assert a.migrations == b.migrations == 5


@pytest.mark.gpu
@pytest.mark.parametrize("L,kw", [(256, {}), (1024, dict(selection="rank")), (700, dict(crossover="two_point"))])
def test_local_islands_batched_launch_matches_streams_gpu(L, kw):
    # one launch per generation for all islands (Island::run_batched, island =
    # grid y) evolves every island exactly as its own launch on its own stream
    common = dict(seed=11, device="cuda:0", migrate_every=5, migrate_pct=0.02, elitism=1, **kw)
    a = LocalIslands(pga.models.OneMax(L), 8, 4096, **common)
    b = LocalIslands(pga.models.OneMax(L), 8, 4096, batched=False, **common)
    a.run(23)
    b.run(23)
    torch.cuda.synchronize()
    assert a.batched_generations == 23 and b.batched_generations == 0
    for x, y in zip(a.islands, b.islands):
        assert torch.equal(x.rows, y.rows) and torch.equal(x.scores, y.scores)
        assert x.best_score() == y.best_score()
    assert a.migrations == b.migrations == 4


@pytest.mark.gpu
@pytest.mark.parametrize("prob,kw", [("sphere30", {}), ("rosen30", dict(selection="rank")), ("sphere100", {})])
def test_local_islands_real_batched_matches_streams_gpu(prob, kw):
    # REAL islands in ONE launch per generation (real_gen_tp_batch, island =
    # grid y) evolve exactly as on their own streams (the generic kernel at
    # this island size): polynomial objectives are exact on both
    p = {"sphere30": lambda: pga.models.Sphere(30), "rosen30": lambda: pga.models.Rosenbrock(30),
         "sphere100": lambda: pga.models.Sphere(100)}[prob]
    common = dict(seed=5, device="cuda:0", migrate_every=5, migrate_pct=0.02, elitism=1, **kw)
    a = LocalIslands(p(), 8, 4096, **common)
    b = LocalIslands(p(), 8, 4096, batched=False, **common)
    a.run(12)
    b.run(12)
    torch.cuda.synchronize()
    assert a.batched_generations == 12 and b.batched_generations == 0
    for x, y in zip(a.islands, b.islands):
        assert torch.equal(x.rows, y.rows) and torch.equal(x.scores, y.scores)
        assert x.best_score() == y.best_score()


@pytest.mark.gpu
@pytest.mark.parametrize("prob,xo", [("matrix", "ox"), ("euc", "pmx"), ("open", "ox")])
def test_local_islands_perm_batched_matches_streams_gpu(prob, xo):
    # TSP islands in ONE launch per generation (perm_gen_fast_batch)
    p = {"matrix": lambda: pga.models.TSP.random_euclidean(100, seed=3),
         "euc": lambda: pga.models.TSPEuclidean.random(64, seed=4),
         "open": lambda: pga.models.TSP.reference_e3(100, seed=2)}[prob]
    common = dict(seed=7, device="cuda:0", migrate_every=4, migrate_pct=0.02, elitism=1, crossover=xo)
    a = LocalIslands(p(), 6, 2048, **common)
    b = LocalIslands(p(), 6, 2048, batched=False, **common)
    a.run(9)
    b.run(9)
    torch.cuda.synchronize()
    assert a.batched_generations == 9 and b.batched_generations == 0
    for x, y in zip(a.islands, b.islands):
        assert torch.equal(x.rows, y.rows) and torch.equal(x.scores, y.scores)


@pytest.mark.gpu
@pytest.mark.parametrize("prob", ["small", "rotated"])
def test_local_islands_batched_falls_back_gpu(prob):
    # a REAL batch below the two-phase kernel's population, or a rotated
    # objective, runs its islands on their streams
    if prob == "small":
        li = LocalIslands(pga.models.Rastrigin(8), 3, 2048, seed=1, device="cuda:0", migrate_every=0)
    else:
        li = LocalIslands(pga.models.Rastrigin(16, rotate=True, seed=1), 4, 8192, seed=1, device="cuda:0",
                          migrate_every=0)
    li.run(3)
    torch.cuda.synchronize()
    assert li.batched_generations == 0
