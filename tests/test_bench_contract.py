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


def test_bench_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2",
           "--steps", "12", "--warmup", "2", "--pop", "4096", "--length", "128"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["n_gpus"] == 2 and out["steps"] == 12 and out["warmup"] == 2 and out["scaling"] == "weak"
    # whole-job aggregate: evals/s over both islands
    assert abs(out["value"] - out["gens_per_sec"] * 4096 * 2) < 1e-6 * out["value"]
    assert abs(out["ms_per_step"] - 1e3 / out["gens_per_sec"]) < 1e-6 * out["ms_per_step"]
    assert out["config"]["global_batch"] == 8192 and out["config"]["parallelism"] == "island2"
    assert out["migrations"] >= 1
