"""Fused key histogram of the headline kernel (GenArgs::key_hist): the exact
top-k / bottom-k selections that read it (migration, elitism > 1, unsorted
top-k) return exactly what the histogram-pass path and the CPU backend return.

Reference semantics: pga_migrate / pga_migrate_between move the "top pct%"
(include/pga.h:108-115), stubbed in the reference (src/pga.cu:368-374)."""
import numpy as np
import pytest
import torch

import libpga_amd as pga

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ga(S, L=1024, seed=5, fused=True, **kw):
    ga = pga.GeneticAlgorithm(pga.models.OneMax(L), S, seed=seed, device=DEV, **kw)
    ga.island.fused_histogram = fused
    return ga


def _order(sc, largest):
    key = -sc if largest else sc
    return torch.from_numpy(np.lexsort((np.arange(sc.numel()), key.numpy())))


@pytest.mark.parametrize("S", [1 << 20, 300007])
def test_fused_histogram_topk_selection_order(S):
    ga = _ga(S)
    assert not ga.island.fused_histogram_ready  # the initial population has none
    ga.run(3)
    assert ga.island.fused_histogram_ready
    sc = ga.scores.cpu()
    k = 10486
    for largest in (True, False):
        idx = ga.island.topk(k, largest, False).cpu().long()
        assert ga.island.fused_histogram_ready  # a selection reads it, leaves it valid
        # selection order: every key beyond the threshold by index, then the ties by index
        ref = _order(sc, largest)[:k]
        assert torch.equal(torch.sort(idx).values, torch.sort(ref).values)
        thr = sc[ref[-1]]
        beyond = (sc > thr) if largest else (sc < thr)
        nb = int(beyond.sum())
        assert torch.equal(idx[:nb], torch.nonzero(beyond).flatten())
    # twice in a row on the same population: the status words are re-zeroed
    a = ga.island.topk(777, True, False).cpu()
    b = ga.island.topk(777, True, False).cpu()
    assert torch.equal(a, b)


def test_fused_histogram_migration_epoch_identical():
    """emigrate -> re-score -> immigrate (IslandModel's epoch) with and without
    the fused histogram: same emigrants, same population afterwards."""
    S, k = 1 << 20, 10486
    gs = [_ga(S, seed=9, fused=f) for f in (True, False)]
    outs = []
    for ga in gs:
        ga.run(4)
        isl = ga.island
        rw = int(isl.row_words)
        rows = torch.empty(k * rw, dtype=torch.int32, device=DEV)
        sc = torch.empty(k, dtype=torch.float32, device=DEV)
        isl.emigrate(k, rows, sc)
        ga.run(1)
        isl.evaluate_rows(rows, sc)
        isl.immigrate(k, rows, sc)
        assert not isl.fused_histogram_ready  # the victims' keys changed
        ga.run(2)
        torch.cuda.synchronize()
        outs.append((rows.cpu(), sc.cpu(), ga.rows.cpu(), ga.scores.cpu()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_fused_histogram_elitism_matches_cpu():
    """elitism > 1 turns the fused histogram on (top-k every generation);
    rows and scores stay bit-identical with the CPU backend."""
    S = 50000
    g = pga.GeneticAlgorithm(pga.models.OneMax(1024), S, seed=3, device=DEV, elitism=5)
    c = pga.GeneticAlgorithm(pga.models.OneMax(1024), S, seed=3, device="cpu", elitism=5)
    assert g.island.fused_histogram
    g.run(6)
    c.run(6)
    torch.cuda.synchronize()
    assert g.island.fused_histogram_ready
    assert torch.equal(g.rows.cpu(), c.rows) and torch.equal(g.scores.cpu(), c.scores)


def test_fused_histogram_local_islands_migration():
    """LocalIslands with exact top-k migration on streams: fused on == off."""
    res = []
    for fused in (True, False):
        li = pga.parallel.LocalIslands(pga.models.OneMax(256), 3, 40000, seed=4, device=DEV, migrate_every=2,
                                       migrate_pct=0.02, batched=False)
        for ga in li.islands:
            ga.island.fused_histogram = fused
        li.run(7)
        torch.cuda.synchronize()
        res.append([ga.rows.cpu() for ga in li.islands])
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("L,gens", [(1024, 3), (64, 150)])
def test_immigrate_best_partials_exact(L, gens):
    """The bottom-k selection writes the population's new per-block packed
    bests itself (no pass over the scores): best() is the max score at its
    lowest index, also in a converged population where the victims are ties
    of the best score (L = 64 after 150 generations)."""
    S, k = 65536, 1311
    ga = _ga(S, L=L, seed=12)
    ga.run(gens)
    isl = ga.island
    rw = int(isl.row_words)
    rows = torch.empty(k * rw, dtype=torch.int32, device=DEV)
    sc = torch.empty(k, dtype=torch.float32, device=DEV)
    isl.emigrate(k, rows, sc)
    ga.run(1)
    isl.evaluate_rows(rows, sc)
    isl.immigrate(k, rows, sc)
    torch.cuda.synchronize()
    s = ga.scores.cpu()
    best, idx = isl.best()
    assert best == s.max().item()
    assert idx == int(torch.nonzero(s == s.max())[0])
    assert torch.equal(ga.problem.reference_fitness(ga.genomes().cpu()), s)
