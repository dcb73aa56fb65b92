"""Worker for test_parallel.py::test_rccl_self_exchange_matches_loopback_gpu.

One process, torch.distributed backend "nccl" (= RCCL) with world size 1 on
the box's one GPU.  The island model is told it has a peer, but both peers
are rank 0, so every migration epoch runs the real overlapped RCCL path
(side-stream top-k + pack, batch_isend_irecv = grouped ncclSend/ncclRecv,
stream wait, bottom-k + scatter) with the migrants going back to the
sending island.  The result must be bit-identical to the same run whose
"network" is a device copy on the posting stream.
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


def model(pga, IslandModel):
    ga = pga.GeneticAlgorithm(pga.models.OneMax(512), 50_000, seed=3, device="cuda:0", elitism=1)
    m = IslandModel(ga, migrate_every=3, migrate_pct=0.02)
    m.world, m.rank = 2, 0
    m._peers = lambda: (0, 0)
    return m


def main(port: int) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import libpga_amd as pga
    from libpga_amd.parallel import IslandModel

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    a = model(pga, IslandModel)
    a.run(31)
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
        b = model(pga, IslandModel)
        b.run(31)
        torch.cuda.synchronize()
    finally:
        dist.batch_isend_irecv, dist.P2POp = real_batch, real_p2p

    assert a.migrations == b.migrations == 10, (a.migrations, b.migrations)
    assert not a.degraded and a.failures == 0
    assert torch.equal(a.ga.rows, b.ga.rows), "RCCL self-exchange diverged from the loopback exchange"
    assert torch.equal(a.ga.scores, b.ga.scores)
    dist.destroy_process_group()
    print("rccl self-exchange ok", a.migrations, a.bytes_sent)


if __name__ == "__main__":
    main(int(sys.argv[1]))
