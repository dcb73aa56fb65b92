"""Worker for the multi-process island-model tests (launched by
tests/test_parallel.py with torch.multiprocessing, gloo backend on CPU)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(rank: int, world: int, port: int, topology: str, out_dir: str) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import libpga_amd as pga
    from libpga_amd.parallel import IslandModel, init_distributed

    r, w, dev = init_distributed("gloo")
    assert (r, w) == (rank, world)
    ga = pga.GeneticAlgorithm(pga.models.OneMax(96), 256, seed=77, island=rank, device="cpu", elitism=1)
    model = IslandModel(ga, migrate_every=5, migrate_pct=0.05, topology=topology)
    b0 = ga.best_score()
    # capture this island's emigrants right before the first migration epoch
    ga.run(5)
    send_scores = ga.scores.clone()
    k = model.k
    # the default policy (the reference's "top pct%"): the exact top-k, ties to the lower index
    S = send_scores.numel()
    top_idx = sorted(range(S), key=lambda i: (-float(send_scores[i]), i))[:k]
    emigrants = ga.rows.clone()[torch.tensor(top_idx)]
    model.start_migration()
    model.finish_migration()
    torch.save({"rank": rank, "emigrants": emigrants, "rows_after": ga.rows.clone(), "k": k,
                "scores_after": ga.scores.clone(), "send_best": float(send_scores.max())},
               os.path.join(out_dir, f"mig_{rank}.pt"))
    model.run(40)
    # early stop: every island stops at the same generation once the global best reaches the target
    tgt = model.global_reduce_best()
    ran = model.run(50, target=tgt, check_every=5)
    assert ran == 5, ran
    score, owner, genome = model.global_best()
    gmax = model.global_reduce_best()
    torch.save({"rank": rank, "b0": b0, "best": ga.best_score(), "global": score, "owner": owner,
                "gmax": gmax, "genome_sum": float(genome.sum()), "migrations": model.migrations,
                "gen": ga.generation - 5},
               os.path.join(out_dir, f"res_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def run_faults(rank: int, world: int, port: int, out_dir: str) -> None:
    """Forged migrants are re-scored, dropped batches are skipped, and an
    island-model checkpoint resumes bit-exactly."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import libpga_amd as pga
    from libpga_amd.parallel import IslandModel, init_distributed
    from libpga_amd.utils import load_model, save_model

    init_distributed("gloo")
    L = 64

    def hook(buf, epoch):
        if epoch == 1:  # forge: claim every migrant is perfect and zero its genes
            k = model.k
            buf[: k * model.rw] = 0
            buf[k * model.rw:] = torch.tensor([1e9], dtype=torch.float32).view(torch.int32)
            return True
        return epoch != 2  # drop the second batch

    ga = pga.GeneticAlgorithm(pga.models.OneMax(L), 128, seed=5, island=rank, device="cpu", elitism=1)
    model = IslandModel(ga, migrate_every=4, migrate_pct=0.1, topology="ring", fault_hook=hook)
    model.run(5)  # one migration (forged)
    forged_ok = ga.best_score() <= L and bool((ga.scores == ga.genomes().sum(1).float()).all())
    model.run(4)  # second migration (dropped)
    dropped = model.dropped
    model.fault_hook = None
    model.run(3)
    prefix = os.path.join(out_dir, "ckpt")
    save_model(model, prefix)
    model.run(10)
    final = ga.rows.clone()
    ga2 = pga.GeneticAlgorithm(pga.models.OneMax(L), 128, seed=5, island=rank, device="cpu", elitism=1)
    model2 = IslandModel(ga2, migrate_every=4, migrate_pct=0.1, topology="ring")
    meta = load_model(model2, prefix)
    model2.run(10)
    torch.save({"forged_ok": forged_ok, "dropped": dropped, "resume_equal": bool(torch.equal(final, ga2.rows)),
                "gen": meta["generation"], "migrations": model.migrations, "migrations2": model2.migrations},
               os.path.join(out_dir, f"fault_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _problem(name):
    import libpga_amd as pga

    if name == "tsp":
        return pga.models.TSP.random_euclidean(40, seed=3)
    return pga.models.Rastrigin(12)


def run_problem(rank: int, world: int, port: int, name: str, topology: str, out_dir: str) -> None:
    """TSP (u16 permutation rows) and Rastrigin (f32 rows) islands: the exact
    emigrants arrive, every row stays valid and correctly scored, and the
    islands migrate on schedule.  name "tsp_forged": the received batch of
    the first epoch is forged into non-permutations claiming a perfect score
    (the native re-scoring must turn them into the identity tour)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import libpga_amd as pga
    from libpga_amd.parallel import IslandModel, init_distributed

    init_distributed("gloo")
    forged = name == "tsp_forged"
    prob = _problem("tsp" if forged else name)
    L = prob.length

    def hook(buf, epoch):
        if epoch == 1:
            k, rw = model.k, model.rw
            g16 = buf[: k * rw].view(k, rw).view(torch.int16)
            g16[0, :L] = 0                        # every gene city 0
            g16[1, :L] = torch.arange(L, dtype=torch.int16)
            g16[1, 5] = 7                          # a duplicate city
            g16[2, :L] = torch.arange(L, dtype=torch.int16)
            g16[2, 9] = L + 100                    # a city beyond the tour
            buf[k * rw:] = torch.tensor([1e9], dtype=torch.float32).view(torch.int32)
        return True

    ga = pga.GeneticAlgorithm(prob, 256, seed=11, island=rank, device="cpu", elitism=1)
    model = IslandModel(ga, migrate_every=5, migrate_pct=0.05, topology=topology,
                        fault_hook=hook if forged else None)
    assert model.transport == "torch" and model.rccl_ranks == 0
    ga.run(5)
    sc = ga.scores.clone()
    k = model.k
    top_idx = sorted(range(sc.numel()), key=lambda i: (-float(sc[i]), i))[:k]
    emigrants = ga.genomes().clone()[torch.tensor(top_idx)]
    model.start_migration()
    model.finish_migration()
    after = ga.genomes().clone()
    scores_after = ga.scores.clone()
    model.run(30)
    final = ga.genomes().clone()
    torch.save({"emigrants": emigrants, "after": after, "scores_after": scores_after,
                "ref_after": prob.reference_fitness(after), "final": final, "final_scores": ga.scores.clone(),
                "ref_final": prob.reference_fitness(final), "k": k, "migrations": model.migrations,
                "degraded": model.degraded, "gen": ga.generation},
               os.path.join(out_dir, f"prob_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    if sys.argv[4] == "problem":
        run_problem(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[5], sys.argv[6], sys.argv[7])
    elif sys.argv[4] == "faults":
        run_faults(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[5])
    else:
        run(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5])
