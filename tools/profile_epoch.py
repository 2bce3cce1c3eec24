"""Per-kernel-family breakdown of epochs (HIP events on the solver stream).
Usage: python tools/profile_epoch.py [fp32|fp64] [epochs] [kkbox|cfg5|kdd12|outbrain]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))

import ocffm  # noqa: E402
import synth  # noqa: E402


def main():
    prec = ocffm.FP64 if (len(sys.argv) > 1 and sys.argv[1] == "fp64") else ocffm.FP32
    epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    work = sys.argv[3] if len(sys.argv) > 3 else "kkbox"
    if work == "cfg5":
        ds = synth.cfg5(m=int(os.environ.get("CFG5_ROWS", "2000000")))
        g = ocffm.problem_from_dataset(ds, precision=prec, with_test=False, k=64, self_side=False)
    elif work in ("kdd12", "outbrain"):
        ds = getattr(synth, work)()
        g = ocffm.problem_from_dataset(ds, precision=prec, with_test=False)
    else:
        ds = synth.kkbox()
        g = ocffm.problem_from_dataset(ds, precision=prec, with_test=False)
    ocffm.srand(1)
    g.init()
    g.one_epoch()
    g.sync()
    t0 = time.perf_counter()
    g.one_epoch()
    g.sync()
    plain = time.perf_counter() - t0
    g.reset_stats()
    g.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(epochs):
        g.one_epoch()
    g.sync()
    prof = (time.perf_counter() - t0) / epochs
    ks = g.kernel_stats()
    tot = sum(v["total_ms"] for k, v in ks.items() if not k.startswith("half(")) / epochs
    print(f"epoch wall (no events) {plain*1e3:.2f} ms; with events {prof*1e3:.2f} ms; "
          f"sum of kernel time {tot:.2f} ms/epoch; cg iters/epoch {g.cg_log().sum()/epochs:.1f}")
    rows = sorted(ks.items(), key=lambda kv: -kv[1]["total_ms"])
    print(f"{'kernel':20s} {'launch/ep':>9s} {'ms/ep':>8s} {'us/launch':>10s} {'alg GB/s':>9s}")
    for name, v in rows:
        per = v["total_ms"] / max(1, v["launches"])
        bw = v["alg_bytes"] / max(1e-12, v["total_ms"] * 1e-3) / 1e9
        tf = v.get("alg_flops", 0.0) / max(1e-12, v["total_ms"] * 1e-3) / 1e12
        print(f"{name:20s} {v['launches']/epochs:9.1f} {v['total_ms']/epochs:8.3f} {per*1e3:10.1f} {bw:9.1f}"
              + (f" {tf:7.1f} TF/s" if tf else ""))
    out = os.path.join(REPO, "gpurun_out", "profile_epoch.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump({"plain_ms": plain * 1e3, "stats": ks, "epochs": epochs}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
