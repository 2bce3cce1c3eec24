"""Gradient / Hessian-vector of one half, run-to-run, after the same state:
which of the two is order-dependent, and in which feature columns."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
import ocffm  # noqa: E402
import synth  # noqa: E402


def main():
    f1 = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    ds = synth.cfg5(m=20000, n=3000, d_user=2000, seed=3)
    fu, k = 39, 32
    res = []
    for r in range(3):
        g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, with_test=False, k=k, self_side=False)
        ocffm.srand(1)
        g.init()
        g.one_epoch()
        print("epoch-1 cg", g.cg_log().tolist(), flush=True)
        for b in range(f1):
            g.solve_block(b, fu)
        G0 = g.grad(f1, fu, 0).reshape(-1, k)
        v = np.random.default_rng(0).standard_normal(G0.size)
        H0 = g.hv(f1, fu, 0, v).reshape(-1, k)
        G1 = g.grad(f1, fu, 1).reshape(-1, k)
        H1 = g.hv(f1, fu, 1, np.random.default_rng(1).standard_normal(G1.size)).reshape(-1, k)
        res.append((G0, H0, G1, H1))
        g.close()
    xidx = np.asarray(ds.train.idx).reshape(-1, fu)[:, f1]
    cnt = np.bincount(xidx.astype(np.int64), minlength=2000)
    for name, i in (("grad W", 0), ("hv W", 1), ("grad H", 2), ("hv H", 3)):
        for (r0, r) in ((0, 1), (0, 2), (1, 2)):
            a, b = res[r0][i], res[r][i]
            rows = np.where((a != b).any(1))[0]
            print(name, f"run{r0} vs run{r}:", len(rows), "rows differ", rows[:10],
                  "col counts", (cnt[rows[:10]] if i < 2 else ""), flush=True)


if __name__ == "__main__":
    main()
