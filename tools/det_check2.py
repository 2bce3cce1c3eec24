"""Locate the first run-to-run difference: epoch 1 by one_epoch, then block
by block with the state of every block compared after each solve."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
import ocffm  # noqa: E402
import synth  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "blocks"
    ds = synth.cfg5(m=20000, n=3000, d_user=2000, seed=3)
    fu = 39
    bl = [(f1, fu) for f1 in range(fu)]
    idx = lambda f1, f2: f2 + (fu + 1 - 1) * f1 - f1 * (f1 - 1) // 2  # noqa: E731
    runs = []
    for r in range(2):
        g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, with_test=False, k=32, self_side=False)
        ocffm.srand(1)
        g.init()
        g.one_epoch()
        trace = []
        if mode == "blocks":
            for (f1, f2) in bl:
                g.solve_block(f1, f2)
                b = idx(f1, f2)
                trace.append({w: g.get(w, b) for w in "WHPQ"} | {"u": g.get("u"), "cg": g.cg_log().copy()})
        else:
            for e in range(int(mode)):
                g.one_epoch()
                trace.append({"W%d" % b[0]: g.get("W", idx(*b)) for b in bl} | {"cg": g.cg_log().copy()})
        runs.append(trace)
        g.close()
    for t, (a, b) in enumerate(zip(*runs)):
        bad = [k for k in a if not np.array_equal(a[k], b[k])]
        print(t, "differ:" if bad else "same", bad[:8], flush=True)
        if bad and mode == "blocks":
            break


if __name__ == "__main__":
    main()
