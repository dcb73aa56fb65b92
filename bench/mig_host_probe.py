#!/usr/bin/env python3
"""Host-side timing of one RCCL self-exchange epoch (world 1, PGA_RCCL_SELF
setup as bench/migration_cost.py): how long each host call of
IslandModel.run's epoch takes, and whether the GPU queue was drained."""
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
ga = pga.GeneticAlgorithm(pga.models.OneMax(1024), 1 << 20, seed=1, device="cuda:0", elitism=1)
m = IslandModel(ga, migrate_every=10, migrate_pct=0.01)
m.world, m.rank = 2, 0
m._peers = lambda: (0, 0)
m.connect()
m.run(50)
torch.cuda.synchronize()
tm = {"emigrate": [], "batch": [], "gen": [], "finish": [], "idle_before_emigrate": []}
isl = ga.island
for ep in range(20):
    for _ in range(9):
        isl.run(1)
    ev = torch.cuda.Event()
    ev.record()
    t = time.perf_counter()
    srows, sscores = m._views(m.send)
    isl.emigrate(m.k, srows, sscores)
    t1 = time.perf_counter()
    tm["idle_before_emigrate"].append(bool(ev.query()))
    ops = [dist.P2POp(dist.isend, m.send, 0), dist.P2POp(dist.irecv, m.recv, 0)]
    works = dist.batch_isend_irecv(ops)
    t2 = time.perf_counter()
    isl.run(1)
    t3 = time.perf_counter()
    for wk in works:
        wk.wait()
    rows, scores = m._views(m.recv)
    isl.evaluate_rows(rows, scores)
    isl.immigrate(m.k, rows, scores)
    t4 = time.perf_counter()
    tm["emigrate"].append(t1 - t)
    tm["batch"].append(t2 - t1)
    tm["gen"].append(t3 - t2)
    tm["finish"].append(t4 - t3)
torch.cuda.synchronize()
out = {k: (sum(v) / len(v) * 1e6 if k != "idle_before_emigrate" else sum(v)) for k, v in tm.items()}
print(json.dumps({"host_us": out}))
dist.destroy_process_group()
