"""Two ranks (gloo host all-reduce) on one GPU, block by block, with
per-column cross Grams forced (OCFFM_CCG=2): which block's solve fails."""
import os
import sys

import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "one-class-ffm_amd"))


def worker(rank, port, env):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **env)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    import torch
    import ocffm
    import synth

    def allreduce(arr):
        dist.all_reduce(torch.from_numpy(arr))

    ds = synth.kkbox(seed=5, m=300, n=400, mean=12.0, name="kkbox_dist")
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, rank=rank, nranks=2, allreduce=allreduce)
    ocffm.srand(1)
    g.init()
    f = 5
    for e in range(2):
        for f1 in range(f):
            for f2 in range(f1, f):
                try:
                    g.solve_block(f1, f2)
                except Exception as ex:
                    print(f"rank {rank} epoch {e} block ({f1},{f2}) FAILED: {ex}; cg {list(map(int, g.cg_log()))}",
                          flush=True)
                    os._exit(1)
        print(f"rank {rank} epoch {e} ok cg {list(map(int, g.cg_log()))}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    env = dict(a.split("=") for a in sys.argv[1:])
    mp.spawn(worker, args=(29557, env), nprocs=2, join=True)
