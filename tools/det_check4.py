"""Same state, the gradient twice in one run; and across runs the inputs the
block comparison did not cover (item-major y~, biases)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
import ocffm  # noqa: E402
import synth  # noqa: E402


def main():
    f1 = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    nomfma = len(sys.argv) > 2
    if nomfma:
        os.environ["OCFFM_NO_MFMA"] = "1"
    ds = synth.cfg5(m=20000, n=3000, d_user=2000, seed=3)
    fu, k = 39, 32
    st = []
    for r in range(2):
        g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, with_test=False, k=k, self_side=False)
        ocffm.srand(1)
        g.init()
        g.one_epoch()
        for b in range(f1):
            g.solve_block(b, fu)
        inputs = {w: g.get(w) for w in "abuv"}
        Ga = g.grad(f1, fu, 0)
        Gb = g.grad(f1, fu, 0)
        print(f"run {r}: grad twice equal: {np.array_equal(Ga, Gb)}; max diff {np.abs(Ga - Gb).max():.3e}", flush=True)
        st.append((inputs, Ga))
        g.close()
    for w in "abuv":
        print(w, "equal across runs:", np.array_equal(st[0][0][w], st[1][0][w]), flush=True)


if __name__ == "__main__":
    main()
