"""Fused per-generation statistics (device.hpp ScoreStats): the generation
kernels store {min, sum} per block beside their packed best, so
GeneticAlgorithm.stats() / history() need no pass over the scores.  Checked
against plain torch over the score array, on every kernel family."""
import pytest
import torch

import libpga_amd as pga

M = pga.models


def torch_stats(scores):
    s = scores.double().cpu()
    return float(s.min()), float(s.max()), float(s.mean())


def check(ga, rtol=1e-5):
    st = ga.stats()
    mn, mx, mean = torch_stats(ga.scores)
    assert st["min"] == pytest.approx(mn, rel=0, abs=0)
    assert st["max"] == pytest.approx(mx, rel=0, abs=0)
    assert st["mean"] == pytest.approx(mean, rel=rtol, abs=1e-6)


def test_history_cpu():
    ga = pga.GeneticAlgorithm(M.OneMax(100), 300, seed=2, device="cpu", elitism=1)
    ga.record_history()
    rows = []
    for _ in range(5):
        ga.run(1)
        rows.append(torch_stats(ga.scores))
    h = ga.history()
    assert h.shape == (5, 4)
    for r, (mn, mx, mean) in zip(h.tolist(), rows):
        assert r[0] == mn and r[1] == mx and r[2] == pytest.approx(mean, rel=1e-6) and r[3] == 300
    ga.record_history(False)
    ga.run(2)
    assert ga.history().shape == (5, 4)  # stopped recording


def test_run_target_native_cpu():
    ga = pga.GeneticAlgorithm(M.OneMax(64), 512, seed=3, device="cpu", elitism=1)
    g = ga.run(400, target=64.0, check_every=4)
    assert 0 < g < 400 and g % 4 == 0 and ga.best_score() == 64.0


GPU_CASES = {
    "onemax_tp": lambda: (M.OneMax(1024), dict(elitism=1)),
    "onemax_generic": lambda: (M.OneMax(1024), dict(elitism=1, tournament_k=3)),
    "knapsack_mfma": lambda: (M.Knapsack01.random(1024, seed=1), dict(elitism=1)),
    "rastrigin": lambda: (M.Rastrigin(30), dict(elitism=1)),
    "rastrigin_rot": lambda: (M.Rastrigin(30, rotate=True, seed=1), dict(elitism=1)),
    "real_long": lambda: (M.Rastrigin(1000), dict(elitism=1)),
    "tsp": lambda: (M.TSP.random_euclidean(64, seed=1), dict(elitism=1)),
    "tsp_long": lambda: (M.TSPEuclidean.random(5000, seed=1), dict(elitism=1)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(GPU_CASES))
def test_fused_stats_gpu(case):
    problem, kw = GPU_CASES[case]()
    S = 200 if case == "tsp_long" else 20000
    ga = pga.GeneticAlgorithm(problem, S, seed=4, device="cuda:0", **kw)
    check(ga)  # from the INIT kernel's partials
    ga.record_history()
    rows = []
    for _ in range(3):
        ga.run(1)
        torch.cuda.synchronize()
        check(ga)
        rows.append(torch_stats(ga.scores))
    h = ga.history()
    assert h.shape == (3, 4)
    for r, (mn, mx, mean) in zip(h.tolist(), rows):
        assert r[0] == mn and r[1] == mx and r[2] == pytest.approx(mean, rel=1e-5, abs=1e-6)


@pytest.mark.gpu
def test_stats_after_external_rescore_gpu():
    """After migration the fused partials are stale: stats falls back to the
    pass over the scores and stays exact."""
    ga = pga.GeneticAlgorithm(M.OneMax(256), 4096, seed=5, device="cuda:0", elitism=1)
    ga.run(2)
    isl = ga.island
    rows = torch.zeros((8, isl.row_words), dtype=torch.int32, device="cuda:0") - 1  # all-ones genomes
    sc = torch.full((8,), 256.0, device="cuda:0")
    isl.immigrate(8, rows, sc)
    torch.cuda.synchronize()
    check(ga)
    assert ga.stats()["max"] == 256.0


@pytest.mark.gpu
def test_run_target_native_gpu():
    ga = pga.GeneticAlgorithm(M.OneMax(128), 1 << 16, seed=3, device="cuda:0", elitism=1)
    g = ga.run(2000, target=128.0, check_every=8)
    assert 0 < g < 2000 and g % 8 == 0 and ga.best_score() == 128.0
