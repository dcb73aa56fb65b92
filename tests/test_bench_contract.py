"""bench.py driver contract on the CPU (gloo): one JSON line from rank 0 with
the whole-job value, launched exactly as the driver launches N > 1."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(*extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2",
           *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "transport", "rccl_ranks", "migrations_timed",
              "migrations_expected", "degraded", "failures"):
        assert k in out
    # migration health: every exchange of the timed window happened
    assert out["degraded"] is False and out["failures"] == 0
    assert out["migrations_timed"] == out["migrations_expected"] >= 1
    assert out["transport"] == "torch" and out["rccl_ranks"] == 0  # gloo: no RCCL involved
    return out


def test_expected_migrations():
    sys.path.insert(0, ROOT)
    import bench

    # IslandModel.run starts an exchange at every generation g > 0 with g % every == 0
    assert bench.expected_migrations(0, 10, 10) == 0
    assert bench.expected_migrations(2, 12, 10) == 1
    assert bench.expected_migrations(10, 20, 10) == 2
    assert bench.expected_migrations(5, 500, 10) == 50
    assert bench.expected_migrations(5, 500, 0) == 0


def test_bench_tsp256_two_ranks_gloo():
    """BASELINE config 5 through the driver's launcher (reduced population)."""
    out = _run("--steps", "12", "--warmup", "2", "--problem", "tsp256", "--crossover", "pmx", "--pop", "1024")
    assert out["config"]["model"] == "TSP-256" and out["config"]["crossover"] == "pmx"
    assert out["config"]["global_batch"] == 2048 and out["dtype"] == "u16-permutation"
    assert out["vs_baseline"] is None  # no reference-semantics run for TSP
    assert abs(out["value"] - out["gens_per_sec"] * 1024 * 2) < 1e-6 * out["value"]


def test_bench_two_ranks_gloo():
    out = _run("--steps", "12", "--warmup", "2", "--pop", "4096", "--length", "128")
    assert out["n_gpus"] == 2 and out["steps"] == 12 and out["warmup"] == 2 and out["scaling"] == "weak"
    # whole-job aggregate: evals/s over both islands
    assert abs(out["value"] - out["gens_per_sec"] * 4096 * 2) < 1e-6 * out["value"]
    assert abs(out["ms_per_step"] - 1e3 / out["gens_per_sec"]) < 1e-6 * out["ms_per_step"]
    assert out["config"]["global_batch"] == 8192 and out["config"]["parallelism"] == "island2"
    assert out["migrations"] >= 1
