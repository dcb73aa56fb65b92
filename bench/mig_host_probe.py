#!/usr/bin/env python3
"""Host-side timing of one RCCL self-exchange migration epoch (world 1,
PGA_RCCL_SELF setup as bench/migration_cost.py), per transport of
IslandModel: "torch" (emigrate, batch_isend_irecv, wait, re-score, immigrate
as separate host calls) and "engine" (the engine's RCCL communicator,
comm_bind.cpp: one call packs + posts, one completes).  Prints one JSON line
with the host microseconds of each call and their sum per epoch."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libpga_amd as pga  # noqa: E402
from libpga_amd.parallel import IslandModel  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29518")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))


def probe(transport):
    ga = pga.GeneticAlgorithm(pga.models.OneMax(1024), 1 << 20, seed=1, device="cuda:0", elitism=1)
    m = IslandModel(ga, migrate_every=10, migrate_pct=0.01, transport=transport)
    m.world, m.rank = 2, 0
    m._peers = lambda: (0, 0)
    ga.island.fused_histogram = True
    m.connect()
    m.run(50)
    torch.cuda.synchronize()
    tm = {"post": [], "gen": [], "finish": [], "idle_before_post": []}
    isl = ga.island
    for ep in range(20):
        for _ in range(9):
            isl.run(1)
        ev = torch.cuda.Event()
        ev.record()
        t = time.perf_counter()
        m.start_migration()  # emigrate + post (torch: isl.emigrate + batch_isend_irecv)
        t1 = time.perf_counter()
        tm["idle_before_post"].append(bool(ev.query()))
        isl.run(1)
        t2 = time.perf_counter()
        m.finish_migration()  # wait + re-score + immigrate
        t3 = time.perf_counter()
        tm["post"].append(t1 - t)
        tm["gen"].append(t2 - t1)
        tm["finish"].append(t3 - t2)
    torch.cuda.synchronize()
    assert m.migrations >= 20 and not m.degraded
    out = {k: (sum(v) / len(v) * 1e6 if k != "idle_before_post" else sum(v)) for k, v in tm.items()}
    out["epoch_host_us"] = out["post"] + out["finish"]
    return out


res = {t: probe(t) for t in ("torch", "engine")}
print(json.dumps({"host_us": res}))
dist.destroy_process_group()
