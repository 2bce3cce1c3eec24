"""Wall time and CG steps of each epoch of one shape (fp32 unless argv[3] is
fp64): python tools/epoch_times.py <kkbox|kdd12|outbrain> <epochs> [fp64]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "one-class-ffm_amd"))
import ocffm  # noqa: E402
import synth  # noqa: E402


def main():
    work = sys.argv[1] if len(sys.argv) > 1 else "kdd12"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    prec = ocffm.FP64 if (len(sys.argv) > 3 and sys.argv[3] == "fp64") else ocffm.FP32
    ds = getattr(synth, work)()
    k = {"kkbox": 32, "kdd12": 16, "outbrain": 64}[work]
    g = ocffm.problem_from_dataset(ds, precision=prec, with_test=False, k=k)
    ocffm.srand(1)
    g.init()
    g.sync()
    c0 = 0
    for e in range(n):
        t0 = time.perf_counter()
        g.one_epoch()
        g.sync()
        dt = time.perf_counter() - t0
        cg = g.cg_log()
        print(f"epoch {e + 1:3d}  {dt * 1e3:8.2f} ms  cg {int(cg[c0:].sum()):5d}", flush=True)
        c0 = cg.size
    g.close()


if __name__ == "__main__":
    main()
