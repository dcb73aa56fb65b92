"""Worker for test_parallel.py::test_rccl_self_exchange_matches_loopback_gpu
(mode "match") and ::test_rccl_withheld_send_degrades_gpu (mode "withhold").

One process, torch.distributed backend "nccl" (= RCCL) with world size 1 on
the box's one GPU.  The island model is told it has a peer, but both peers
are rank 0, so every migration epoch runs the real overlapped RCCL path
(fused top-k + pack, batch_isend_irecv = grouped ncclSend/ncclRecv,
stream wait, bottom-k + scatter) with the migrants going back to the
sending island.  The result must be bit-identical to the same run whose
"network" is a device copy on the posting stream.  Mode "match" runs this
twice: with emigrant selection + packing on the compute stream (the default)
and on the side stream (side_stream=True).
"""
import os
import sys
import types

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Done:
    def wait(self, *a):
        return True


def model(pga, IslandModel, **kw):
    ga = pga.GeneticAlgorithm(pga.models.OneMax(512), 50_000, seed=3, device="cuda:0", elitism=1)
    m = IslandModel(ga, migrate_every=3, migrate_pct=0.02, **kw)
    m.world, m.rank = 2, 0
    m._peers = lambda: (0, 0)
    return m


def main(port: int) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import libpga_amd as pga
    from libpga_amd.parallel import IslandModel

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    for transport, side in (("engine", False), ("torch", False), ("torch", True)):
        match(pga, IslandModel, side, transport)
    dist.destroy_process_group()


def match(pga, IslandModel, side: bool, transport: str) -> None:
    a = model(pga, IslandModel, side_stream=side, transport=transport)
    assert a._use_engine == (transport == "engine")
    a.run(31)
    a.flush()  # (lag 2 on GPU islands: the epoch that left at 30 lands here)
    torch.cuda.synchronize()

    real_batch, real_p2p = dist.batch_isend_irecv, dist.P2POp

    def fake_batch(ops):
        send = next(o.tensor for o in ops if o.op is dist.isend)
        recv = next(o.tensor for o in ops if o.op is dist.irecv)
        recv.copy_(send)
        return [_Done()]

    dist.batch_isend_irecv = fake_batch
    dist.P2POp = lambda op, t, peer, group=None: types.SimpleNamespace(op=op, tensor=t)
    try:
        b = model(pga, IslandModel, side_stream=side, transport="torch")
        b.run(31)
        b.flush()
        torch.cuda.synchronize()
    finally:
        dist.batch_isend_irecv, dist.P2POp = real_batch, real_p2p

    assert a.migrations == b.migrations == 10, (a.migrations, b.migrations)
    assert not a.degraded and a.failures == 0
    assert torch.equal(a.ga.rows, b.ga.rows), "RCCL self-exchange diverged from the loopback exchange"
    assert torch.equal(a.ga.scores, b.ga.scores)
    print("rccl self-exchange ok", transport, "side stream" if side else "compute stream", a.migrations, a.bytes_sent)


def withhold(port: int) -> None:
    """Migration epochs over real RCCL, then one whose send is withheld: the
    receive can never complete, the 2 s host deadline expires, the group is
    aborted, and the island keeps evolving (degraded) without ever ordering
    its compute stream after the dead transfer."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import libpga_amd as pga
    from libpga_amd.parallel import IslandModel

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    engine = len(sys.argv) > 3 and sys.argv[3] == "engine"
    # lag 1: each epoch completes one generation after it leaves (the counts below)
    m = model(pga, IslandModel, timeout_s=2.0, transport="engine" if engine else "torch", lag=1)
    if engine:  # the engine communicator's own fault injection: the 3rd exchange's sends withheld
        m._engine().set_fault(3, 3)
    m.run(7)  # epochs at generations 3 and 6 complete
    assert m.migrations == 2 and not m.degraded
    if not engine:
        m._withhold_send = True
    t0 = time.monotonic()
    m.run(10)  # epoch at generation 9 times out; generations 9..16 still run
    best = m.ga.best_score()
    dt = time.monotonic() - t0
    assert m.degraded and m.failures == 1 and m.migrations == 2, (m.degraded, m.failures, m.migrations)
    assert m.ga.generation == 17 and best > 0
    assert dt < 30, dt
    print("rccl withheld send ok", "engine" if engine else "torch", round(dt, 2))
    sys.stdout.flush()
    os._exit(0)  # the aborted group is not torn down again


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "withhold":
        withhold(int(sys.argv[1]))
    else:
        main(int(sys.argv[1]))
