"""Debug: 2 sharded ranks (host all-reduce) vs single rank, block by block."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    import ocffm
    import synth

    def allreduce(arr):
        t = torch.from_numpy(arr)
        dist.all_reduce(t)

    ds = synth.tiny(seed=8)
    a = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
    b = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, rank=rank, nranks=2, allreduce=allreduce)
    for g in (a, b):
        ocffm.srand(1)
        g.init()
    f = 3
    for f1 in range(f):
        for f2 in range(f1, f):
            for half in (0, 1):
                ga, gb = a.grad(f1, f2, half), b.grad(f1, f2, half)
                v = np.random.default_rng(0).standard_normal(ga.size)
                ha, hb = a.hv(f1, f2, half, v), b.hv(f1, f2, half, v)
                if rank == 0:
                    print("grad/hv", f1, f2, half, np.abs(ga - gb).max() / np.abs(ga).max(),
                          np.abs(ha - hb).max() / np.abs(ha).max(), flush=True)
            a.solve_block(f1, f2)
            b.solve_block(f1, f2)
            bi = ocffm.block_index(f1, f2, f)
            if rank == 0:
                for what in "WH":
                    xa, xb = a.get(what, bi), b.get(what, bi)
                    print("state", f1, f2, what, np.abs(xa - xb).max() / np.abs(xa).max(), flush=True)
                print("cg", a.cg_log()[-2:], b.cg_log()[-2:], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(worker, args=(29533,), nprocs=2, join=True)
