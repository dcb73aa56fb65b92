import os, sys, time, json, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import libpga_amd as pga
M = pga.models
for name, prob, kw in [("sum100_refops", lambda: M.SumGenes(100), {}), ("rast30", lambda: M.Rastrigin(30), dict(elitism=1))]:
    for S in (10000, 40000, 100000, 250000, 1 << 20):
        ga = pga.GeneticAlgorithm(prob(), S, seed=1, device="cuda:0", **kw)
        ga.run(20); torch.cuda.synchronize()
        n = 200 if S < 200000 else 60
        t0 = time.perf_counter(); ga.run(n); torch.cuda.synchronize()
        print(json.dumps({"cfg": name, "S": S, "generic": os.environ.get("PGA_FORCE_GENERIC", "0"), "us": (time.perf_counter() - t0) / n * 1e6}), flush=True)
