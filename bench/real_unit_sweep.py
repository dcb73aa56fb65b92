"""REAL small-population sweep of the two-phase grid's breed unit (PGA_TP_UMAX,
read once per process: run one process per value).  One JSON line per size."""
import os, sys, time, json, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import libpga_amd as pga
M = pga.models
for name, prob, kw in [("sum100_refops", lambda: M.SumGenes(100), {}), ("rast30", lambda: M.Rastrigin(30), dict(elitism=1))]:
    for S in (40000, 100000):
        ga = pga.GeneticAlgorithm(prob(), S, seed=1, device="cuda:0", **kw)
        ga.run(20); torch.cuda.synchronize()
        n = 300
        t0 = time.perf_counter(); ga.run(n); torch.cuda.synchronize()
        print(json.dumps({"cfg": name, "S": S, "umax": os.environ.get("PGA_TP_UMAX", "64"),
                          "us": (time.perf_counter() - t0) / n * 1e6}), flush=True)
