"""Benchmark: training epochs of the one-class FFM block Newton-CG on MI355X.

Metric (BASELINE.json): train instances/sec, kkbox-shape k=32.  A "step" is
one training epoch (ImpProblem::one_epoch, ffm.cpp:852-870) over the
synthetic kkbox-shaped rows (SURVEY §8d, configs[2]); instances = training
rows.  Inputs are resident in HBM before the timed region.

Multi-GPU (one process per GPU): weak scaling — each rank owns a
kkbox-shaped user shard of 30,755 rows (the items are shared), the gradient
and Hessian-vector partial sums are all-reduced with RCCL inside the
library; torch.distributed (gloo) is only the control plane (comm-id
broadcast, barrier, max-over-ranks timing).  Launched either by torchrun
(RANK / WORLD_SIZE in the environment) or as `python bench.py --gpus N`:
without WORLD_SIZE and with N > 1 this process starts N child ranks of
itself (fresh interpreters, nothing here has touched the GPU yet) and exits
with their status; rank 0 prints the line.

The JSON line also carries:
  roofline     — the dominant kernel family (the most kernel time over a
                 second pass of the same K epochs right after the
                 uninstrumented timed region, every dispatch carrying HIP
                 events on the solver stream): algorithmic bytes per launch
                  / its average event-measured duration.
  cpu_baseline — the CPU oracle (clean-room OpenMP port of the reference,
                 fp64) timed on this host on a bounded sample, rank 0, N=1:
                 the same epoch window as the GPU's first timed epochs (the
                 oracle starts from the GPU's tables after the warm-up).
  modes        — (N=1) the same kkbox epochs in fp64 (the reference's own
                 arithmetic, the parity mode); the config-5 shard (BASELINE
                 configs[4] restated, SURVEY §8d: 2 M rows, 39+1 fields,
                 k=64, 20 GB of P caches: past the Infinity Cache); the
                 SGD/AdaGrad mode.  Each with its own roofline: "mfma" with
                 TFLOP/s against the f32 MFMA peak when the dominant family's
                 algorithmic flop/byte exceeds the ridge, else "hbm".
"""
import argparse
import glob
import json
import os
import re
import resource
import socket
import subprocess
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
MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32), dense
RIDGE_FLOP_PER_B = MFMA_F32_PEAK_TFS * 1e12 / (HBM_PEAK_GBS * 1e9)
ROWS_PER_GPU = 30755
CFG5_ROWS = 12_500_000  # BASELINE configs[4]: 100 M rows over 8 GPUs


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
    ap.add_argument("--modes", choices=["auto", "off"], default="auto",
                    help="N=1: also time the fp64 parity mode and the config-5 shard into 'modes'")
    ap.add_argument("--cfg5-steps", type=int, default=2, help="timed epochs of the config-5 mode (<= --steps)")
    ap.add_argument("--cfg5-rows", type=int, default=CFG5_ROWS, help="rows of the config-5 shard")
    ap.add_argument("--cpu-all-child", type=int, default=0, help=argparse.SUPPRESS)
    return ap.parse_args()


def spawn_ranks(n):
    """`bench.py --gpus N` outside torchrun: N fresh child processes of this
    script, one per GPU (LOCAL_RANK = rank), rendezvous on 127.0.0.1.  The
    parent has not touched the GPU; it waits and returns the worst status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OCFFM_BENCH_LAUNCHER="spawn")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        p.wait()
        rc = rc or p.returncode
    return rc


def run_newton(ds, prec, steps, warmup, k=32, self_side=True, world=1, rank=0, local=0, comm=None, allreduce=None,
               pmc_tag="", snapshot=None):
    """W warm-up epochs, K timed epochs (barrier + device sync on both sides,
    max over ranks, no instrumentation), then the same K epochs again with
    every dispatch carrying HIP events: the family with the most kernel
    time over that pass is the dominant one, its average launch the
    roofline's.  snapshot(g): called after the warm-up (CPU baseline)."""
    ts = time.perf_counter()
    g = ocffm.problem_from_dataset(ds, precision=prec, with_test=False, device=local, rank=rank, nranks=world,
                                   comm=comm, allreduce=allreduce, k=k, self_side=self_side)
    t_create = time.perf_counter() - ts
    ts = time.perf_counter()
    ocffm.srand(1)
    g.init()
    g.sync()
    t_init = time.perf_counter() - ts

    def barrier():
        g.sync()
        if world > 1:
            dist.barrier()

    for _ in range(max(1, warmup)):
        g.one_epoch()
    if snapshot is not None:
        snapshot(g)
    cg0 = g.cg_log().size

    # timed region: K epochs, no instrumentation (event-carrying dispatches
    # cost ~7 us each and would perturb the wall clock)
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.one_epoch()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    cg = g.cg_log()[cg0:]
    alg = g.alg_bytes()
    # kernel-timing pass: the same K epochs again, every dispatch carrying
    # start/stop HIP events on the solver stream
    g.reset_stats()
    g.set_profiling(True)
    for _ in range(steps):
        g.one_epoch()
    barrier()
    ks = g.kernel_stats()
    # persistent column-Gram CG launches and the ones whose grid gave up on
    # its barrier and finished per step (ocffm_problem_counter)
    cgp = {"launches": g.counter("cgp_launches"), "recovered": g.counter("cgp_recovered")}
    g.close()

    fams = {kk: v for kk, v in ks.items() if not kk.startswith("half(") and not kk.endswith(".noop")}
    dominant = max(fams.items(), key=lambda kv: kv[1]["total_ms"])[0]
    d = ks[dominant]
    avg_ms = d["total_ms"] / max(1, d["launches"])
    bytes_per_launch = d["alg_bytes"] / max(1, d["launches"])
    flops_per_launch = d.get("alg_flops", 0.0) / max(1, d["launches"])
    if flops_per_launch > RIDGE_FLOP_PER_B * bytes_per_launch:  # an MFMA-bound family (k x k Grams / T at large C)
        ach = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
        roof = {"kernel": dominant, "bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_F32_PEAK_TFS,
                "unit": "TFLOP/s", "frac": round(ach / MFMA_F32_PEAK_TFS, 4), "traffic": None,
                "alg_flops_per_launch": flops_per_launch,
                "achieved_GBps": round(bytes_per_launch / (avg_ms * 1e-3) / 1e9, 1) if avg_ms > 0 else 0.0}
    else:
        ach = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        roof = {"kernel": dominant, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None}
    tot_ms = sum(v["total_ms"] for v in fams.values())
    roof.update({"avg_launch_us": round(avg_ms * 1e3, 2), "alg_bytes_per_launch": bytes_per_launch,
                 "launches": d["launches"], "share_of_kernel_time": round(d["total_ms"] / max(1e-9, tot_ms), 3),
                 "epoch_alg_GBps": round(alg / dt / 1e9, 1), "epoch_alg_bytes": alg / max(1, steps),
                 "families_ms_per_epoch": {kk: round(v["total_ms"] / steps, 3) for kk, v in
                                           sorted(fams.items(), key=lambda kv: -kv[1]["total_ms"])[:6]},
                 # the same six families' own rates: algorithmic GB/s per launch (and
                 # TFLOP/s for the MFMA families) against the same peaks
                 "families_frac": {kk: round(v["alg_bytes"] / max(1e-12, v["total_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                   if v.get("alg_flops", 0.0) <= RIDGE_FLOP_PER_B * v["alg_bytes"] else
                                   round(v["alg_flops"] / max(1e-12, v["total_ms"] * 1e-3) / 1e12 / MFMA_F32_PEAK_TFS, 4)
                                   for kk, v in sorted(fams.items(), key=lambda kv: -kv[1]["total_ms"])[:6]}})
    # HBM bytes per launch of the same kernel family from the committed
    # rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE, MI355X guide §HBM).
    # Those passes are one-GPU runs: on several ranks nobody measured this
    # run's counters, so the line carries null (and says why).
    # (rNN[a-z]_<tag>pmc_traffic.json: the headline's tag is empty)
    name_re = re.compile(r"^r\d+[a-z]?_" + re.escape(pmc_tag) + r"pmc_traffic\.json$")
    pmcs = sorted(p for p in glob.glob(os.path.join(REPO, "profiles", "r*pmc_traffic.json"))
                  if name_re.match(os.path.basename(p)))
    if world > 1:
        roof["traffic_source"] = "none: the committed PMC passes are N=1 runs"
    elif pmcs:
        pmc = pmcs[-1]
        roof["traffic_source"] = os.path.relpath(pmc, REPO)
        try:
            t = json.load(open(pmc)).get(dominant)
            roof["traffic"] = None if t is None else round(t["bytes_per_launch"])
        except Exception:
            pass
    # what ran, observed (not re-derived from the library's gate): the
    # item-owned CG steps' row pass appears in the kernel-timing pass
    io_launches = int(ks.get("hs_cross_io", {}).get("launches", 0))
    return dict(dt=dt, roof=roof, cg_per_epoch=round(cg.sum() / max(1, steps), 1),
                setup_s={"create": round(t_create, 3), "init": round(t_init, 3)}, io_launches=io_launches, cgp=cgp)


T_START = time.perf_counter()


def log(msg):
    """Progress on stderr (a long silent run is taken for a hung one)."""
    print(f"[bench {time.perf_counter() - T_START:6.1f}s] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.cpu_all_child:
        _cpu_all_child(args.cpu_all_child)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and "--gpus" in " ".join(sys.argv):
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        dist.init_process_group("gloo")
    if os.environ.get("OCFFM_BENCH_DRY") == "1":
        # launcher check (CPU tests): every rank reports in, nothing touches the GPU
        t = torch.tensor([1.0])
        if world > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"n_gpus": world, "ranks_seen": int(t.item()),
                              "launcher": os.environ.get("OCFFM_BENCH_LAUNCHER", "torchrun" if world > 1 else "none")}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
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
    snap = {}
    want_cpu = rank == 0 and world == 1 and args.cpu_baseline == "auto"

    def take(g):  # the GPU's tables after the warm-up: the CPU baseline starts there
        fu = int(ds.train.fid.max()) + 1
        fv = int(ds.item.fid.max()) + 1
        snap["tables"] = {(w, b): g.get(w, b) for b in _blocks(fu, fv) for w in "WH"}
        snap["epoch"] = max(1, args.warmup) + 1

    log(f"rank {rank}/{world}: kkbox-shape data ready, headline epochs")
    r = run_newton(ds, prec, args.steps, args.warmup, k=32, world=world, rank=rank, local=local, comm=comm,
                   allreduce=allreduce, pmc_tag="" if prec == ocffm.FP32 else "fp64_",
                   snapshot=take if want_cpu else None)
    rows_total = ROWS_PER_GPU * world
    value = rows_total * args.steps / r["dt"]

    cpu = None
    if want_cpu:
        log("CPU baseline")
        cpu = cpu_baseline(ds, args.cpu_epochs, args.cpu_single_epochs, snap, r["cg_per_epoch"])
    modes = {}
    if world == 1 and args.modes == "auto":
        if prec == ocffm.FP32:
            modes["fp64"] = timed_mode(fp64_mode, ds, args)
        modes["kdd12"] = timed_mode(shape_mode, args, "kdd12")
        modes["outbrain"] = timed_mode(shape_mode, args, "outbrain")
        modes["cfg5"] = timed_mode(cfg5_mode, args)
        if args.sgd == "auto":
            modes["sgd"] = timed_mode(sgd_mode, ds, args)

    if rank == 0:
        line = {
            "metric": "train instances/sec, kkbox-shape k=32; 1/2/4/8 MI355X vs CPU OpenMP",
            "value": round(value, 1), "unit": "instances/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(r["dt"] / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32" if prec == ocffm.FP32 else "f64",
            "data": "synthetic",
            "config": {"workload": "kkbox-shape (BASELINE configs[2]): one-class FFM block Newton-CG epoch",
                       "rows_per_gpu": ROWS_PER_GPU, "rows_total": rows_total, "items": int(ds.item.m),
                       "positives": ds.n_positives, "user_fields": 2, "item_fields": 3, "k": 32,
                       "lambda": 4.0, "omega": 0.0078125, "r": -1.0,
                       "parallelism": f"dp{world}" + ("-rccl1" if comm is not None and world == 1 else ""),
                       "rccl_ranks": world if comm is not None else 0,
                       "launcher": os.environ.get("OCFFM_BENCH_LAUNCHER", "torchrun" if world > 1 else "none"),
                       "allreduce": "gloo-host (rehearsal)" if rehearsal else ("rccl" if comm is not None else "none"),
                       # song-id item halves' CG steps item-owned: observed,
                       # launches of their row pass in the kernel-timing pass
                       "item_owned_cg": r["io_launches"] > 0,
                       "item_owned_cg_launches": r["io_launches"],
                       "persistent_cg": r["cgp"],
                       "cg_iters_per_epoch": r["cg_per_epoch"]},
            "roofline": r["roof"],
            "cpu_baseline": cpu,
        }
        if modes:
            line["modes"] = modes
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _blocks(fu, fv, self_side=True):
    """index_vec (ffm.cpp:53-55) of every block of the model."""
    f = fu + fv
    return [f2 + (f - 1) * f1 - f1 * (f1 - 1) // 2 for f1 in range(f) for f2 in range(f1, f)
            if self_side or (f1 < fu <= f2)]


def timed_mode(fn, *a):
    """A mode's result with its wall time and the process's peak host RSS."""
    log(f"mode {fn.__name__}{'' if len(a) < 2 or not isinstance(a[-1], str) else ' ' + a[-1]}")
    t0 = time.perf_counter()
    out = fn(*a)
    out["wall_s"] = round(time.perf_counter() - t0, 1)
    out["peak_rss_GB"] = round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2)
    return out


def fp64_mode(ds, args):
    """The same kkbox-shape epochs in the reference's own arithmetic (fp64,
    ffm.h:34-35): the parity mode's speed, with its own roofline (s = 8)."""
    try:
        r = run_newton(ds, ocffm.FP64, args.steps, args.warmup, k=32, pmc_tag="fp64_")
        return {"metric": "train instances/sec, kkbox-shape k=32, fp64 (parity mode)",
                "value": round(ROWS_PER_GPU * args.steps / r["dt"], 1), "unit": "instances/s", "dtype": "f64",
                "ms_per_step": round(r["dt"] / args.steps * 1e3, 3), "cg_iters_per_epoch": r["cg_per_epoch"],
                "roofline": r["roof"]}
    except Exception as e:  # never blocks the headline number
        return {"value": None, "error": str(e)}


SHAPES = {  # BASELINE configs at their SURVEY §8d per-GPU sizes (synth.kdd12 / synth.outbrain)
    "kdd12": dict(k=16, workload="BASELINE configs[1] shape (SURVEY §8d): kdd12, 500 k users x 50 k ads, "
                              "user fields UserID + {QueryID, Depth}, ad fields Title, Description, Keyword, "
                              "{AdID, DisplayURL, Advertiser}, k=16, squared loss (the reference has no log-loss)"),
    "outbrain": dict(k=64, workload="BASELINE configs[3] shape (SURVEY §8d): one GPU's 250 k-row shard of the "
                                    "2 M-row 8-GPU run, 10 k ads, 2 + 2 multi-node fields, ~1 positive per row, k=64"),
}


def shape_mode(args, name):
    """One of BASELINE's other configs at its per-GPU size, fp32, with its
    own roofline (the same measurement as the headline line)."""
    try:
        t0 = time.perf_counter()
        ds = getattr(synth, name)()
        gen = time.perf_counter() - t0
        sh = SHAPES[name]
        r = run_newton(ds, ocffm.FP32, args.steps, args.warmup, k=sh["k"], pmc_tag=name + "_")
        return {"metric": f"train instances/sec, {name}-shape k={sh['k']}",
                "value": round(ds.train.m * args.steps / r["dt"], 1), "unit": "instances/s", "dtype": "f32",
                "ms_per_step": round(r["dt"] / args.steps * 1e3, 3),
                "config": {"workload": sh["workload"], "rows_per_gpu": ds.train.m, "items": int(ds.item.m),
                           "positives": ds.n_positives, "user_fields": int(ds.train.fid.max()) + 1,
                           "item_fields": int(ds.item.fid.max()) + 1, "k": sh["k"],
                           "cg_iters_per_epoch": r["cg_per_epoch"], "datagen_s": round(gen, 2),
                           "setup_s": r["setup_s"]},
                "roofline": r["roof"]}
    except Exception as e:  # never blocks the headline number
        return {"value": None, "error": str(e)}


def cfg5_mode(args):
    """BASELINE configs[4] as SURVEY §8d restates it, one GPU's row shard of
    the 100 M-row, 8-GPU run: --ns, 39 user fields of 250,000 features + the
    item id (250,000 items), k = 64, fp32, CFG5_ROWS rows (the 39 P caches
    alone are 20 GB: every pass streams from HBM, past the 256 MB Infinity
    Cache).  Weak scaling at N GPUs = N such shards."""
    try:
        t0 = time.perf_counter()
        rows = args.cfg5_rows
        ds = synth.cfg5(m=rows)
        gen = time.perf_counter() - t0
        steps = max(1, min(args.steps, args.cfg5_steps))
        # two warm-up epochs: epoch 2 is the shard's slowest (most CG steps)
        # and the halves' column-Gram choice follows the previous epoch's counts
        r = run_newton(ds, ocffm.FP32, steps, 2, k=64, self_side=False, pmc_tag="cfg5_")
        return {"metric": "train instances/sec, config-5 shard (39+1 fields, 250k feats/field, k=64, --ns)",
                "value": round(rows * steps / r["dt"], 1), "unit": "instances/s", "dtype": "f32",
                "steps": steps, "warmup": 2, "ms_per_step": round(r["dt"] / steps * 1e3, 3),
                "config": {"workload": "BASELINE configs[4] restated (SURVEY §8d): one GPU's row shard "
                                       "(100 M rows / 8 GPUs)" if rows == CFG5_ROWS else
                                       f"BASELINE configs[4] structure, {rows} rows (not the 8-GPU shard)",
                           "rows_per_gpu": rows, "items": int(ds.item.m), "positives": ds.n_positives,
                           "user_fields": 39, "item_fields": 1, "features_per_field": 250000, "k": 64,
                           "self_side": False, "cg_iters_per_epoch": r["cg_per_epoch"],
                           "p_cache_GB": round(39 * rows * 64 * 4 / 1e9, 1), "datagen_s": round(gen, 1),
                           "setup_s": r["setup_s"]},
                "roofline": r["roof"]}
    except Exception as e:  # never blocks the headline number
        return {"value": None, "error": str(e)}


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


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CPU_ALL_LIMIT_S = 40


def _cpu_all_threads(threads, m):
    """One oracle epoch of the kkbox shape from init on `threads` threads,
    in a child process bounded by CPU_ALL_LIMIT_S seconds."""
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-all-child", str(threads)]
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=CPU_ALL_LIMIT_S)
        secs = float(r.stdout.strip().splitlines()[-1])
        return {"value": round(m / secs, 1), "cores": threads,
                "sample": f"1 epoch from init of the same problem on {threads} threads, {secs:.2f} s"}
    except subprocess.TimeoutExpired:
        return {"value": None, "cores": threads, "upper_bound": round(m / CPU_ALL_LIMIT_S, 1),
                "sample": f"1 epoch from init on {threads} threads did not finish in {CPU_ALL_LIMIT_S} s "
                          f"(with data generation and init, {time.perf_counter() - t0:.0f} s): below "
                          f"{m / CPU_ALL_LIMIT_S:.0f} instances/s"}
    except Exception as e:
        return {"value": None, "cores": threads, "sample": f"failed: {e}"}


def _cpu_all_child(threads):
    import oracle_lib as O
    ds = synth.kkbox(m=ROWS_PER_GPU)
    o = O.Oracle(ds, threads=threads, with_test=False)
    ocffm.srand(1)
    o.init()
    print(o.time_epochs(1, threads), flush=True)


def _physical_cores():
    """(physical id, core id) pairs of /proc/cpuinfo: cores, not SMT threads."""
    try:
        cores, phys = set(), None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                cores.add((phys, line.split(":", 1)[1].strip()))
        return len(cores) or None
    except OSError:
        return None


def cpu_baseline(ds, epochs, single_epochs=1, snap=None, gpu_cg=None, all_epochs=1):
    """The CPU oracle on a bounded sample: `epochs` epochs of the same
    kkbox-shaped problem, fp64, on every host core this process may use.
    With `snap` (the GPU's tables after its warm-up) the oracle starts from
    that state, so its sample is the same epoch window as the GPU's first
    timed epochs (later epochs need fewer CG steps than the first ones)."""
    try:
        import oracle_lib as O
        avail = len(os.sched_getaffinity(0))
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or avail
        o = O.Oracle(ds, threads=threads, with_test=False)
        ocffm.srand(1)
        o.init()
        window = "epochs 1.." + str(epochs) + " from init"
        if snap and "tables" in snap:
            for (w, b), t in snap["tables"].items():
                o.set(w, b, t)
            o.refresh()
            window = f"epochs {snap['epoch']}..{snap['epoch'] + epochs - 1} (from the GPU's tables after its warm-up)"
        o.cg_log_clear()
        secs = o.time_epochs(epochs, threads)
        cg = float(o.cg_log().sum()) / max(1, epochs)
        out = {"value": round(ds.train.m * epochs / secs, 1), "unit": "instances/s", "cores": threads,
               "kind": "port", "precision": "f64",
               "sample": f"{epochs} epoch(s) of the same kkbox-shape problem ({ds.train.m} rows), {window}, "
                         f"{secs:.2f} s",
               "cg_iters_per_epoch": round(cg, 1), "gpu_cg_iters_per_epoch": gpu_cg,
               "host": {"cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count(), "affinity_cpus": avail,
                        "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}}
        if gpu_cg:  # the same rate per CG step (the work an epoch does scales with its CG steps)
            out["value_at_gpu_cg_count"] = round(out["value"] * cg / gpu_cg, 1)
        # SURVEY 8(d)'s -c <all cores>: every CPU this process may run on
        # (the box exposes the whole host; its fair share is OMP_NUM_THREADS).
        # The reference zeroes and sums nr_threads x D x k buffers every CG
        # step (ffm.cpp:557,759,783-794), so its epoch grows with the thread
        # count past a few dozen threads: the point runs in a child process
        # under a time limit, and a timeout is reported as an upper bound.
        out["host"]["physical_cores"] = _physical_cores()
        if avail > threads and all_epochs > 0:
            out["all_threads"] = _cpu_all_threads(avail, ds.train.m)
        if single_epochs > 0:  # also the one-thread rate (the reference's -c 1)
            s1 = o.time_epochs(single_epochs, 1)
            out["single_thread"] = {"value": round(ds.train.m * single_epochs / s1, 1), "cores": 1,
                                    "sample": f"{single_epochs} epoch(s) after the sample above, {s1:.2f} s"}
        return out
    except Exception as e:  # the baseline never blocks the GPU number
        return {"value": None, "unit": "instances/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}


if __name__ == "__main__":
    main()
