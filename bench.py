"""Benchmark: training epochs of the one-class FFM block Newton-CG on MI355X.

Metric (BASELINE.json): train instances/sec, kkbox-shape k=32.  A "step" is
one training epoch (ImpProblem::one_epoch, ffm.cpp:852-870) over the
synthetic kkbox-shaped rows (SURVEY §8d, configs[2]); instances = training
rows.  Inputs are resident in HBM before the timed region.

Multi-GPU (torchrun, one process per GPU): weak scaling — each rank owns a
kkbox-shaped user shard of 30,755 rows (the items are shared), the gradient
and Hessian-vector partial sums are all-reduced with RCCL inside the
library; torch.distributed (gloo) is only the control plane (comm-id
broadcast, barrier, max-over-ranks timing).

The JSON line also carries:
  roofline     — the dominant kernel family: algorithmic bytes per launch
                  / its HIP-event-measured average
                 duration on the solver stream, over a second pass of the
                 same K epochs right after the (uninstrumented) timed region.
  cpu_baseline — the CPU oracle (clean-room OpenMP port of the reference,
                 fp64) timed on this host on a bounded sample, rank 0, N=1.
"""
import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (loads the HIP runtime first: one runtime per process)
import torch.distributed as dist  # noqa: E402

import ocffm  # noqa: E402
import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ROWS_PER_GPU = 30755


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precision", choices=["fp32", "fp64"], default="fp32")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-epochs", type=int, default=4)
    ap.add_argument("--cpu-single-epochs", type=int, default=1, help="one-thread oracle epochs (0: skip)")
    ap.add_argument("--sgd", choices=["auto", "off"], default="auto",
                    help="N=1: also time the SGD/AdaGrad mode (tools/bench_sgd.py) into 'modes'")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    prec = ocffm.FP32 if args.precision == "fp32" else ocffm.FP64

    ds = synth.kkbox(m=ROWS_PER_GPU * world)
    comm = None
    allreduce = None
    rehearsal = world > 1 and os.environ.get("OCFFM_BENCH_REHEARSAL") == "1"
    if rehearsal:
        # N ranks on one GPU (tests of this script's multi-rank flow on a
        # one-GPU box): the library's all-reduces go through gloo on the host
        local = 0

        def allreduce(arr):
            dist.all_reduce(torch.from_numpy(arr))
    elif world > 1:
        obj = [ocffm.comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = obj[0]
    elif os.environ.get("OCFFM_BENCH_COMM1") == "1":
        # N = 1 on the multi-rank code path (a one-rank RCCL communicator):
        # the compute cost of that path without any real exchange
        comm = ocffm.comm_id()
    g = ocffm.problem_from_dataset(ds, precision=prec, with_test=False, device=local, rank=rank, nranks=world,
                                   comm=comm, allreduce=allreduce)
    ocffm.srand(1)
    g.init()

    def barrier():
        g.sync()
        if world > 1:
            dist.barrier()

    # warmup; the first warmup epoch also finds the dominant kernel family
    g.set_profiling(True)
    for _ in range(max(1, args.warmup)):
        g.one_epoch()
    ks = g.kernel_stats()
    dominant = max(((k, v) for k, v in ks.items() if not k.startswith("half(")),
                   key=lambda kv: kv[1]["total_ms"])[0]
    g.reset_stats()
    g.set_profiling(False)

    # timed region: K epochs, no instrumentation (event-carrying dispatches
    # cost ~7 us each and would perturb the wall clock)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.one_epoch()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    cg = g.cg_log()
    alg = g.alg_bytes()
    # kernel-timing pass: the same K epochs again, the dominant family's
    # dispatches carrying start/stop HIP events on the solver stream
    g.reset_stats()
    g.set_profile_filter(dominant)
    g.set_profiling(True)
    for _ in range(args.steps):
        g.one_epoch()
    barrier()
    ks = g.kernel_stats()

    rows_total = ROWS_PER_GPU * world
    value = rows_total * args.steps / dt
    d = ks.get(dominant, dict(launches=0, total_ms=0.0, alg_bytes=0.0))
    avg_ms = d["total_ms"] / max(1, d["launches"])
    bytes_per_launch = d["alg_bytes"] / max(1, d["launches"])
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    roof = {"kernel": dominant, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "avg_launch_us": round(avg_ms * 1e3, 2), "alg_bytes_per_launch": bytes_per_launch,
            "launches": d["launches"],
            "epoch_alg_GBps": round(alg / dt / 1e9, 1),
            "epoch_alg_bytes": alg / max(1, args.steps)}
    # HBM bytes per launch of the same kernel family from the committed
    # rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE, MI355X guide §HBM).
    pmcs = sorted(p for p in glob.glob(os.path.join(REPO, "profiles", "r*_pmc_traffic.json")) if "_sgd_" not in p)
    if pmcs:
        pmc = pmcs[-1]
        roof["traffic_source"] = os.path.relpath(pmc, REPO)
        try:
            t = json.load(open(pmc)).get(dominant)
            roof["traffic"] = None if t is None else round(t["bytes_per_launch"])
        except Exception:
            pass

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        cpu = cpu_baseline(ds, args.cpu_epochs, args.cpu_single_epochs)
    modes = None
    if world == 1 and args.sgd == "auto":
        modes = {"sgd": sgd_mode(ds, args)}

    if rank == 0:
        line = {
            "metric": "train instances/sec, kkbox-shape k=32; 1/2/4/8 MI355X vs CPU OpenMP",
            "value": round(value, 1), "unit": "instances/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32" if prec == ocffm.FP32 else "f64",
            "data": "synthetic",
            "config": {"workload": "kkbox-shape (BASELINE configs[2]): one-class FFM block Newton-CG epoch",
                       "rows_per_gpu": ROWS_PER_GPU, "rows_total": rows_total, "items": int(ds.item.m),
                       "positives": ds.n_positives, "user_fields": 2, "item_fields": 3, "k": 32,
                       "lambda": 4.0, "omega": 0.0078125, "r": -1.0,
                       "parallelism": f"dp{world}" + ("-rccl1" if comm is not None and world == 1 else ""),
                       "cg_iters_per_epoch": round(cg.sum() / max(1, args.steps), 1)},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if modes:
            line["modes"] = modes
        print(json.dumps(line), flush=True)
    g.close()
    if world > 1:
        dist.destroy_process_group()


def sgd_mode(ds, args):
    """The SGD/AdaGrad + on-device-negatives mode on the same kkbox-shape data
    (north_star extra, parity unpinned vs the reference; tools/bench_sgd.py
    has the full line).  Instances = positives x 2 (one negative each)."""
    try:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        import bench_sgd as BS
        U = ocffm.ImpData.from_rows(ds.train)
        V = ocffm.ImpData.from_rows(ds.item)
        t = ocffm.SgdTrainer(U, V, k=32, nneg=1, neg_power=0.75)
        t.epoch()
        t.sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            t.epoch()
        t.sync()
        per = (time.perf_counter() - t0) / args.steps
        info = t.info
        kp = info["kp"]
        bpi = BS.slot_rows([0, 1, 1, 2, 3, 4]) * kp * 4 * 4
        ach = info["instances"] * bpi / per / 1e9
        t.close()
        return {"metric": "train instances/sec (SGD/AdaGrad, HOGWILD, on-device negatives)",
                "value": round(info["instances"] / per, 1), "unit": "instances/s", "ms_per_step": round(per * 1e3, 3),
                "roofline": {"kernel": "k_sgd", "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "alg_bytes_per_instance": bpi},
                "parity": "unpinned vs reference (no counterpart); pinned to oracle/sgd_oracle.cpp"}
    except Exception as e:  # never blocks the headline number
        return {"value": None, "error": str(e)}


def cpu_baseline(ds, epochs, single_epochs=1):
    """The CPU oracle on a bounded sample: `epochs` epochs of the same
    kkbox-shaped problem, fp64, all host threads this process may use."""
    try:
        import oracle_lib as O
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        o = O.Oracle(ds, threads=threads, with_test=False)
        ocffm.srand(1)
        o.init()
        secs = o.time_epochs(epochs, threads)
        out = {"value": round(ds.train.m * epochs / secs, 1), "unit": "instances/s", "cores": threads,
               "kind": "port", "precision": "f64",
               "sample": f"{epochs} epoch(s) of the same kkbox-shape problem ({ds.train.m} rows), {secs:.2f} s"}
        if single_epochs > 0:  # also the one-thread rate (the reference's -c 1)
            s1 = o.time_epochs(single_epochs, 1)
            out["single_thread"] = {"value": round(ds.train.m * single_epochs / s1, 1), "cores": 1,
                                    "sample": f"{single_epochs} epoch(s), {s1:.2f} s"}
        return out
    except Exception as e:  # the baseline never blocks the GPU number
        return {"value": None, "unit": "instances/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}


if __name__ == "__main__":
    main()
