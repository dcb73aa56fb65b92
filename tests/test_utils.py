"""Utilities: tracing no-ops, timers, evaluate_rows (migrant re-scoring),
single-island checkpoint round trip."""
import torch

import libpga_amd as pga
from libpga_amd.utils import GpuTimer, trace_mark, trace_range, tracing_enabled


def test_trace_and_timer_cpu():
    assert tracing_enabled() is False  # PGA_TRACE unset in the test env
    with trace_range("outer"):
        trace_mark("m")
        with GpuTimer(torch.device("cpu")) as t:
            sum(range(1000))
    assert t.ms >= 0.0


def test_evaluate_rows_rescoring_cpu():
    ga = pga.GeneticAlgorithm(pga.models.OneMax(200), 64, seed=3, device="cpu")
    rows = ga.rows[:8].clone()
    forged = torch.full((8,), 1e9)
    assert ga.island.evaluate_rows(rows, forged)
    assert torch.equal(forged, ga.scores[:8])


def test_evaluate_rows_perm_clamps_forged_genes():
    n = 16
    d = torch.rand(n, n)
    ga = pga.GeneticAlgorithm(pga.models.TSP(d), 32, seed=1, device="cpu")
    rows = ga.rows[:2].clone()
    rows.view(torch.int16)[0, :n] = 0x7FFF  # out-of-range city ids must not read out of bounds
    sc = torch.zeros(2)
    ga.island.evaluate_rows(rows, sc)
    assert torch.isfinite(sc).all()
    assert sc[1] == ga.scores[1]


def test_checkpoint_roundtrip_exact(tmp_path):
    kw = dict(seed=11, device="cpu", elitism=2)
    a = pga.GeneticAlgorithm(pga.models.OneMax(130), 100, **kw)
    a.run(3)
    a.save(str(tmp_path / "a.ckpt"))
    a.run(5)
    b = pga.GeneticAlgorithm(pga.models.OneMax(130), 100, initialize=False, **kw)
    b.load(str(tmp_path / "a.ckpt"))
    b.run(5)
    assert torch.equal(a.rows, b.rows) and torch.equal(a.scores, b.scores)
