"""SGD-mode benchmark (north_star extras; not the headline line of bench.py).

python tools/bench_sgd.py [--steps K] [--warmup W] [--k 32] [--nneg 1]
  [--cpu-sample N]

Workload: the kkbox-shape data of bench.py (30,755 users, 100,000 items,
~2.1 M positives), field-aware FM by AdaGrad with HOGWILD writes, `nneg`
on-device negatives per positive.  A step is one epoch; instances = positives
x (1 + nneg).  Prints one JSON line like bench.py: value = instances/s,
roofline of the k_sgd kernel (compulsory bytes: every active slot row
w[j_a][f] read + written and its AdaGrad row read + written, once per
instance) and the CPU baseline = oracle/sgd_oracle.cpp (serial, 1 core) on
the first N positives.  Multi-GPU: torchrun, each rank trains its user shard
and the ranks average W and G with RCCL after every epoch (weak scaling).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import ocffm  # noqa: E402
import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0
ROWS_PER_GPU = 30755


def slot_rows(fields):
    """Active slots (a, f) of one instance with node fields `fields`."""
    cnt = {}
    for f in fields:
        cnt[f] = cnt.get(f, 0) + 1
    return sum(sum(1 for f, c in cnt.items() if c - (1 if f == fa else 0) > 0) for fa in fields)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--nneg", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=100000)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    ds = synth.kkbox(m=ROWS_PER_GPU * world)
    U = ocffm.ImpData.from_rows(ds.train)
    V = ocffm.ImpData.from_rows(ds.item)
    comm = None
    if world > 1:
        obj = [ocffm.comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = obj[0]
    t = ocffm.SgdTrainer(U, V, rank=rank, nranks=world, comm=comm, k=args.k, nneg=args.nneg, neg_power=0.75,
                         device=local)
    info = t.info
    for _ in range(args.warmup):
        t.epoch()
        t.average()

    def barrier():
        t.sync()
        if world > 1:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    losses = []
    for _ in range(args.steps):
        losses.append(t.epoch())
        t.average()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        x = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        dt = float(x.item())
    inst_rank = info["instances"]
    total = inst_rank * world
    if rank != 0:
        dist.destroy_process_group()
        return
    # compulsory bytes per instance (kkbox rows: users 1 id + 2 context nodes,
    # items 3 nodes; every item row has the same field layout)
    uf = [0, 1, 1]
    vf = [2, 3, 4]
    slots = slot_rows(uf + vf)
    kp = info["kp"]
    bytes_inst = slots * kp * 4 * 4  # W and G rows: read + write
    per_epoch_s = dt / args.steps
    achieved = inst_rank * bytes_inst / per_epoch_s / 1e9
    cpu = None
    if world == 1:
        cpu = cpu_baseline(ds, info, args)
    line = {
        "metric": "train instances/sec, kkbox-shape k=32, SGD/AdaGrad FFM + on-device negatives (north_star mode)",
        "value": round(total / per_epoch_s, 1), "unit": "instances/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(per_epoch_s * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "kkbox-shape positives (30,755 users/GPU, 100,000 items), AdaGrad HOGWILD",
                   "k": args.k, "nneg": args.nneg, "instances_per_epoch": total, "positives": info["positives"] * world,
                   "mean_loss_last_epoch": round(losses[-1], 5), "parallelism": f"dp{world} + model averaging"},
        "roofline": {"kernel": "k_sgd", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "alg_bytes_per_instance": bytes_inst, "slots_per_instance": slots},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(ds, info, args):
    """oracle/sgd_oracle.cpp (serial, one core) on the first N positives."""
    try:
        import test_sgd as T
        o = T.OracleSgd(ds, info["n_fields"], info["kp"],
                        {"eta": 0.2, "lambda": 2e-5, "nneg": args.nneg, "neg_power": 0.75, "adagrad": 1, "norm": 1,
                         "seed": 1})
        n = min(args.cpu_sample, o.pu.size)
        o.pu, o.pv = o.pu[:n].copy(), o.pv[:n].copy()
        W = np.zeros(info["n_features"] * info["n_fields"] * info["kp"], np.float32)
        W[:] = 0.01
        G = np.ones_like(W)
        t0 = time.perf_counter()
        o.epoch(W, G, 0, 1000003, 7)
        secs = time.perf_counter() - t0
        inst = n * (1 + args.nneg)
        return {"value": round(inst / secs, 1), "unit": "instances/s", "cores": 1, "kind": "port",
                "sample": f"{inst} instances ({n} positives x (1 + {args.nneg})), {secs:.2f} s"}
    except Exception as e:
        return {"value": None, "unit": "instances/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}


if __name__ == "__main__":
    main()
