import sys, time, torch
sys.path.insert(0, ".")
import libpga_amd as pga
which = sys.argv[1]
if which == "rast1m":
    ga = pga.GeneticAlgorithm(pga.models.Rastrigin(30), 1 << 20, seed=1, device="cuda:0", elitism=1)
elif which == "sum40k":
    ga = pga.GeneticAlgorithm(pga.models.SumGenes(100), 40000, seed=1, device="cuda:0")
print("init", flush=True)
for i in range(5):
    ga.run(1); torch.cuda.synchronize(); print("gen", i, ga.best_score(), flush=True)
