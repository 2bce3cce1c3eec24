"""Host set-up phases of a config-5 shard (or kkbox): data generation, the
ImpData build (split_fields / transY), problem creation (per-field CSR/CSC,
segments, uploads) and init, each timed; OCFFM_TIMING=1 adds the library's
own phase marks on stderr.  Usage: python tools/setup_timing.py [cfg5|kkbox] [rows]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))

import ocffm  # noqa: E402
import synth  # noqa: E402


def main():
    work = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
    t = time.perf_counter()
    if work == "cfg5":
        ds = synth.cfg5(m=int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000)
        kw = dict(k=64, self_side=False)
    else:
        ds = synth.kkbox()
        kw = {}
    t1 = time.perf_counter()
    U = ocffm.ImpData.from_rows(ds.train)
    V = ocffm.ImpData.from_rows(ds.item)
    V.trans_y(U)
    t2 = time.perf_counter()
    p = ds.params
    prm = ocffm.Parameter(omega=p["w"], lambda_=p["l"], r=p["r"], nr_pass=p["t"], k=kw.get("k", p["k"]),
                          precision=ocffm.FP32, self_side=int(kw.get("self_side", True)))
    g = ocffm.ImpProblem(U, None, V, prm)
    t3 = time.perf_counter()
    ocffm.srand(1)
    g.init()
    g.sync()
    t4 = time.perf_counter()
    print(f"{work}: datagen {t1-t:.2f} s, ImpData (split_fields+transY) {t2-t1:.2f} s, "
          f"create {t3-t2:.2f} s, init {t4-t3:.2f} s", flush=True)
    g.close()


if __name__ == "__main__":
    main()
