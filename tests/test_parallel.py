"""Island model across processes (torch.distributed, gloo on CPU; the same
code path uses RCCL on GPUs)."""
import os
import types
import socket
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(world, mode, tmp_path):
    port = free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), str(world), str(port),
                               mode, str(tmp_path)]) for r in range(world)]
    for p in procs:
        assert p.wait(timeout=300) == 0


def test_migration_faults_and_resume(tmp_path):
    spawn(2, "faults", tmp_path)
    for r in range(2):
        x = torch.load(tmp_path / f"fault_{r}.pt", weights_only=True)
        assert x["forged_ok"], "forged migrant scores leaked into the population"
        assert x["dropped"] == 1
        assert x["gen"] == 12
        assert x["resume_equal"], "island-model checkpoint did not resume bit-exactly"
        assert x["migrations"] >= 3  # forged (accepted after re-scoring) + later epochs; the dropped one not counted


def launch(world, topology, tmp_path):
    port = free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), str(world), str(port),
                               topology, str(tmp_path)]) for r in range(world)]
    for p in procs:
        assert p.wait(timeout=300) == 0
    mig = [torch.load(tmp_path / f"mig_{r}.pt", weights_only=True) for r in range(world)]
    res = [torch.load(tmp_path / f"res_{r}.pt", weights_only=True) for r in range(world)]
    return mig, res


@pytest.mark.parametrize("world,topology", [(2, "ring"), (3, "ring"), (3, "random"), (4, "all_to_all")])
def test_island_model_multiprocess(world, topology, tmp_path):
    mig, res = launch(world, topology, tmp_path)
    if topology == "ring":
        # rank r received exactly rank r-1's emigrants (rows present after migration)
        for r in range(world):
            src = mig[(r - 1) % world]
            after = {tuple(x.tolist()) for x in mig[r]["rows_after"]}
            assert all(tuple(x.tolist()) in after for x in src["emigrants"])
            assert float(mig[r]["scores_after"].max()) >= src["send_best"]
    gmax = max(x["best"] for x in res)
    for x in res:
        assert x["gen"] == 45
        assert x["migrations"] >= 8
        assert x["global"] == gmax and x["gmax"] == gmax
        assert x["genome_sum"] == gmax  # OneMax: broadcast genome matches the global best score
        assert x["best"] > x["b0"]


def _is_perm(x: torch.Tensor) -> torch.Tensor:
    return (x.sort(dim=1).values == torch.arange(x.shape[1])).all(dim=1)


@pytest.mark.parametrize("name,world,topology", [("tsp", 2, "ring"), ("tsp", 3, "all_to_all"),
                                                 ("rastrigin", 2, "ring"), ("rastrigin", 3, "all_to_all"),
                                                 ("tsp_forged", 2, "ring")])
def test_island_model_problems_multiprocess(name, world, topology, tmp_path):
    """Cross-process migration of permutation (u16) and f32 rows, ring and
    all-to-all (gloo, the same IslandModel code path as RCCL)."""
    port = free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), str(world), str(port),
                               "problem", name, topology, str(tmp_path)]) for r in range(world)]
    for p in procs:
        assert p.wait(timeout=300) == 0
    res = [torch.load(tmp_path / f"prob_{r}.pt", weights_only=True) for r in range(world)]
    L = res[0]["after"].shape[1]
    for r, x in enumerate(res):
        assert not x["degraded"] and x["gen"] == 35 and x["migrations"] == 7
        for key in ("after", "final"):
            ref = x["ref_" + key]
            got = x["scores_after" if key == "after" else "final_scores"]
            # every stored score is the local objective's (ulp-level: the
            # native sum order differs from torch's)
            assert torch.allclose(got, ref, rtol=1e-5, atol=1e-4), (key, (got - ref).abs().max())
            if name != "rastrigin":
                assert bool(_is_perm(x[key]).all()), f"rank {r}: a non-permutation row entered ({key})"
        rows_after = {tuple(v.tolist()) for v in x["after"]}
        if name == "tsp_forged":
            # the three forged rows became the identity tour, scored as one
            # (no 1e9 claim survives); the other migrants arrived intact
            ident = tuple(range(L))
            assert ident in rows_after
            assert float(x["scores_after"].max()) < 0
            src = res[(r - 1) % world]["emigrants"]
            assert sum(tuple(v.tolist()) in rows_after for v in src) >= src.shape[0] - 3
        elif topology == "ring":
            src = res[(r - 1) % world]["emigrants"]
            assert all(tuple(v.tolist()) in rows_after for v in src)
        else:  # all_to_all: each peer's slice of its top-k arrived
            per = x["k"] // (world - 1)
            for p in range(world):
                if p != r:
                    got = sum(tuple(v.tolist()) in rows_after for v in res[p]["emigrants"])
                    assert got >= per, (r, p, got, per)


class _Done:
    def wait(self, *a):
        return True


def _loopback_model(side: bool):
    """A 2-island ring whose 'network' is a device copy send -> recv on the
    posting stream: exercises the stream ordering of the overlapped migration
    on one GPU (RCCL allows one rank per device)."""
    import libpga_amd as pga
    from libpga_amd.parallel import IslandModel

    ga = pga.GeneticAlgorithm(pga.models.OneMax(512), 50_000, seed=3, device="cuda:0", elitism=1)
    m = IslandModel(ga, migrate_every=3, migrate_pct=0.02, side_stream=side)
    m.world, m.rank = 2, 0
    return m


@pytest.mark.gpu
def test_overlapped_migration_stream_order_gpu(monkeypatch):
    import torch.distributed as dist

    def fake_batch(ops):
        send = next(o.tensor for o in ops if o.op is dist.isend)
        recv = next(o.tensor for o in ops if o.op is dist.irecv)
        recv.copy_(send)  # on the current (side) stream, like the NCCL stream would after waiting on it
        return [_Done()]

    monkeypatch.setattr(dist, "batch_isend_irecv", fake_batch)
    monkeypatch.setattr(dist, "P2POp", lambda op, t, peer, group=None: types.SimpleNamespace(op=op, tensor=t))
    a, b = _loopback_model(True), _loopback_model(False)
    assert a._side is not None
    a.run(31)
    b.run(31)
    a.flush()  # (lag 2 on GPU islands: the epoch that left at 30 lands here)
    b.flush()
    torch.cuda.synchronize()
    assert a.migrations == b.migrations == 10
    assert torch.equal(a.ga.rows, b.ga.rows) and torch.equal(a.ga.scores, b.ga.scores)


@pytest.mark.gpu
def test_rccl_self_exchange_matches_loopback_gpu():
    """The real RCCL migration path (backend nccl, world 1, ncclSend/ncclRecv
    to self) gives the same island as a device-copy exchange, bit for bit."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_self_worker.py"), str(free_port())], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    # the engine's RCCL communicator, torch P2P ops on the compute stream and on the side stream
    assert r.stdout.count("rccl self-exchange ok") == 3


@pytest.mark.gpu
def test_rccl_withheld_send_degrades_gpu():
    """RCCL failure path of the python island model: a receive whose send is
    withheld trips the 2 s host deadline, the group is aborted, and the
    island finishes its generations degraded (exit 0, no hang)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_self_worker.py"), str(free_port()), "withhold"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl withheld send ok" in r.stdout


@pytest.mark.gpu
def test_rccl_engine_withheld_send_degrades_gpu():
    """The same failure through the engine's own RCCL communicator
    (comm_bind.cpp): its withheld 3rd exchange expires the deadline, the
    communicator is aborted, the island runs on degraded."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_self_worker.py"), str(free_port()), "withhold",
                        "engine"], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl withheld send ok engine" in r.stdout


def _bench_rccl_self(*extra):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--rccl-self", "--steps", "30",
                        "--warmup", "5", *extra], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    import json

    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["transport"] == "engine" and out["rccl_ranks"] == 1 and out["self_exchange"]
    assert out["migrations_timed"] == out["migrations_expected"] == 3
    assert out["degraded"] is False and out["failures"] == 0
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("problem", ["onemax", "tsp256", "rastrigin30"])
def test_bench_rccl_self_engine_gpu(problem):
    """The driver's bench path with real RCCL migration on one GPU (the
    island exchanges with itself over the engine communicator): every
    BASELINE multi-GPU config migrates through the engine transport, and the
    JSON line accounts for every exchange of the timed window."""
    _bench_rccl_self("--problem", problem, "--pop", "65536")
