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
    top_idx = ga.island.topk(k, True).long()
    emigrants = ga.rows.clone()[top_idx]
    model.start_migration()
    model.finish_migration()
    torch.save({"rank": rank, "emigrants": emigrants, "rows_after": ga.rows.clone(), "k": k,
                "scores_after": ga.scores.clone(), "send_best": float(send_scores.max())},
               os.path.join(out_dir, f"mig_{rank}.pt"))
    model.run(40)
    score, owner, genome = model.global_best()
    gmax = model.global_reduce_best()
    torch.save({"rank": rank, "b0": b0, "best": ga.best_score(), "global": score, "owner": owner,
                "gmax": gmax, "genome_sum": float(genome.sum()), "migrations": model.migrations,
                "gen": ga.generation},
               os.path.join(out_dir, f"res_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    run(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5])
