"""Per-generation fixed cost of the REAL two-phase kernel (PGA_TP_MIN_S=0
forces it at every size): SumGenes-100 at small sizes with operator parts
switched off, to split the ~13 us intercept of the size sweep."""
import os, sys, time, json, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import libpga_amd as pga
M = pga.models
arms = {"refops": {}, "no_mut": dict(mutation="none"), "no_xo": dict(crossover="none"),
        "none": dict(mutation="none", crossover="none"), "elite1": dict(elitism=1), "random_sel": dict(selection="random")}
for S in (512, 4096, 40000):
    for arm, kw in arms.items():
        ga = pga.GeneticAlgorithm(M.SumGenes(100), S, seed=1, device="cuda:0", **kw)
        ga.run(20); torch.cuda.synchronize()
        n = 300
        t0 = time.perf_counter(); ga.run(n); torch.cuda.synchronize()
        print(json.dumps({"S": S, "arm": arm, "min_s": os.environ.get("PGA_TP_MIN_S", "-"),
                          "us": (time.perf_counter() - t0) / n * 1e6}), flush=True)
