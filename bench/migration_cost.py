#!/usr/bin/env python3
"""Per-epoch cost of the island-migration device work on one GPU (everything
IslandModel does except the RCCL transfer itself): top-k emigrants, pack,
bottom-k victims, scatter, best/key refresh (Island.emigrate / immigrate).  Prints one JSON line."""
import json
import types
import os
import sys


def emit(res):
    """One JSON line on stdout, and to $PGA_OUT when set (RCCL may print its
    version banner on stdout, so the file is the clean record)."""
    line = json.dumps(res)
    print(line, flush=True)
    if os.environ.get("PGA_OUT"):
        with open(os.environ["PGA_OUT"], "w") as f:
            f.write(line + "\n")

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libpga_amd as pga  # noqa: E402


def problem(name):
    """PGA_MIG_PROBLEM: onemax (default), rastrigin30, tsp256 (bench.py's configs)."""
    if name == "rastrigin30":
        return pga.models.Rastrigin(30), 1 << 20
    if name == "tsp256":
        g = torch.Generator().manual_seed(7)
        xy = torch.rand(256, 2, generator=g)
        return pga.models.TSP(torch.cdist(xy, xy, compute_mode="donot_use_mm_for_euclid_dist")), 1 << 18
    return pga.models.OneMax(1024), 1 << 20


def main():
    prob, S = problem(os.environ.get("PGA_MIG_PROBLEM", "onemax"))
    S = int(sys.argv[1]) if len(sys.argv) > 1 else S
    pct = float(sys.argv[2]) if len(sys.argv) > 2 else 0.01
    ga = pga.GeneticAlgorithm(prob, S, seed=1, device="cuda:0", elitism=1)
    ga.run(20)
    isl = ga.island
    k = int(round(pct * S))
    rw = int(isl.row_words)
    rows = torch.empty(k * rw, dtype=torch.int32, device="cuda:0")
    sc = torch.empty(k, dtype=torch.float32, device="cuda:0")

    def epoch():  # exactly IslandModel's device work (fused selections)
        isl.emigrate(k, rows, sc)
        isl.evaluate_rows(rows, sc)
        isl.immigrate(k, rows, sc)

    for _ in range(5):
        epoch()
    torch.cuda.synchronize()
    res = {}
    def epoch_gen():  # IslandModel's order: emigrate, one generation, re-score, immigrate
        isl.emigrate(k, rows, sc)
        isl.run(1)
        isl.evaluate_rows(rows, sc)
        isl.immigrate(k, rows, sc)

    def with_fused(on, fn):
        def f():
            isl.fused_histogram = on
            fn()
        return f

    for name, fn in (("topk_sorted", lambda: isl.topk(k, True)), ("topk", lambda: isl.topk(k, True, False)),
                     ("epoch", epoch), ("generation", lambda: isl.run(1)),
                     ("epoch_gen_nofused", with_fused(False, epoch_gen)), ("epoch_gen_fused", with_fused(True, epoch_gen)),
                     ("generation_fused", with_fused(True, lambda: isl.run(1)))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        a.record()
        for _ in range(n):
            fn()
        b.record()
        b.synchronize()
        res[name + "_us"] = a.elapsed_time(b) / n * 1e3
        isl.fused_histogram = False
    # the epoch's device work beyond the generation it overlaps (what the
    # island model adds every migrate_every generations)
    res["epoch_device_nofused_us"] = res["epoch_gen_nofused_us"] - res["generation_us"]
    res["epoch_device_fused_us"] = res["epoch_gen_fused_us"] - res["generation_fused_us"]
    res.update(pop=S, k=k, problem=os.environ.get("PGA_MIG_PROBLEM", "onemax"))
    emit(res)


if __name__ == "__main__" and not os.environ.get("PGA_LOOPBACK") and not os.environ.get("PGA_RCCL_SELF"):
    main()


def loopback_overhead(S=1 << 20, every=10, gens=200):
    """Generations/s of a 2-island ring whose transfer is a device copy
    (one GPU): the island-model overhead the driver's N>1 runs pay, minus xGMI."""
    import torch.distributed as dist
    from libpga_amd.parallel import IslandModel

    class Done:
        def wait(self, *a):
            return True

    def fake_batch(ops):
        ops[1].tensor.copy_(ops[0].tensor)
        return [Done()]

    dist.batch_isend_irecv = fake_batch
    dist.P2POp = lambda op, t, peer, group=None: types.SimpleNamespace(op=op, tensor=t)
    out = {}
    for side in (False, True):
        ga = pga.GeneticAlgorithm(pga.models.OneMax(1024), S, seed=1, device="cuda:0", elitism=1)
        m = IslandModel(ga, migrate_every=every, migrate_pct=0.01, side_stream=side)
        m.world, m.rank = 2, 0
        m.run(20)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        m.run(gens)
        m.flush()
        b.record()
        b.synchronize()
        out["us_per_gen_" + ("overlap" if side else "serial")] = a.elapsed_time(b) / gens * 1e3
    emit(out)


if __name__ == "__main__" and os.environ.get("PGA_LOOPBACK"):
    loopback_overhead()


def rccl_self_overhead(S=1 << 20, every=10, gens=500):
    """us/gen of the headline island with and without migration, where the
    migration runs the REAL RCCL path (backend nccl, world 1, grouped
    ncclSend/ncclRecv to self) on one GPU: everything the driver's N>1 runs
    pay per GPU except the xGMI wire time."""
    import torch.distributed as dist
    from libpga_amd.parallel import IslandModel

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    out = {}
    # (name, every, side stream, overlap, fused histogram, transport)
    arms = (("none", 0, False, True, False, "torch"), ("rccl_self", every, False, True, True, "engine"),
            ("rccl_self_torch", every, False, True, True, "torch"),
            ("rccl_self_torch_side", every, True, True, True, "torch"),
            ("rccl_self_serial", every, False, False, True, "engine"),
            ("rccl_self_nofused", every, False, True, False, "engine"))
    for name, ev, side, overlap, fused, transport in arms:
        ga = pga.GeneticAlgorithm(pga.models.OneMax(1024), S, seed=1, device="cuda:0", elitism=1)
        m = IslandModel(ga, migrate_every=ev, migrate_pct=0.01, side_stream=side, overlap=overlap,
                        transport=transport)
        m.world, m.rank = 2, 0
        ga.island.fused_histogram = fused  # what IslandModel sets for world > 1 (constructed here at world 1)
        m._peers = lambda: (0, 0)
        m.connect() if ev else None
        m.run(50)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        m.run(gens)
        m.flush()
        b.record()
        b.synchronize()
        out["us_per_gen_" + name] = a.elapsed_time(b) / gens * 1e3
        out["migrations_" + name] = m.migrations
    for v in ("rccl_self", "rccl_self_torch", "rccl_self_torch_side", "rccl_self_serial", "rccl_self_nofused"):
        out["overhead_pct_" + v] = 100.0 * (out["us_per_gen_" + v] / out["us_per_gen_none"] - 1.0)
    out.update(pop=S, every=every)
    emit(out)
    dist.destroy_process_group()


if __name__ == "__main__" and os.environ.get("PGA_RCCL_SELF"):
    rccl_self_overhead()
