"""Debug: state inputs of the gradient, sharded rank vs single rank."""
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
    m = 1000
    u0, u1 = m * rank // 2, m * (rank + 1) // 2
    out = []
    for what in "as":
        xa, xb = a.get(what)[u0:u1], b.get(what)
        out.append((what, xa.size, xb.size, float(np.abs(xa - xb).max())))
    for what in "bt":
        xa, xb = a.get(what), b.get(what)
        out.append((what, xa.size, xb.size, float(np.abs(xa - xb).max())))
    ya = a.get("u")
    yb = b.get("u")
    p0 = int(ds.train.yptr[u0]); p1 = int(ds.train.yptr[u1])
    out.append(("u", ya[p0:p1].size, yb.size, float(np.abs(ya[p0:p1] - yb).max())))
    for bi in range(6):
        for what in "WHPQ":
            xa, xb = a.get(what, bi), b.get(what, bi)
            if what in "PQ" and xa.size != xb.size:
                xa = xa.reshape(-1, 4)[u0:u1].ravel()
            out.append((what + str(bi), xa.size, xb.size, float(np.abs(xa - xb).max()) if xa.size == xb.size else -1))
    print(rank, out, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(worker, args=(29534,), nprocs=2, join=True)
