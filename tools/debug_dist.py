"""Debug: fused single-rank path vs the unfused (all-reduce) path, block by block."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
import numpy as np  # noqa: E402

import ocffm  # noqa: E402
import synth  # noqa: E402

ds = synth.tiny(seed=8)
a = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
b = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, allreduce=lambda arr: None)
for g in (a, b):
    ocffm.srand(1)
    g.init()
f = 3
for f1 in range(f):
    for f2 in range(f1, f):
        for half in (0, 1):
            ga, gb = a.grad(f1, f2, half), b.grad(f1, f2, half)
            print("grad", f1, f2, half, np.abs(ga - gb).max() / np.abs(ga).max())
            v = np.random.default_rng(0).standard_normal(ga.size)
            ha, hb = a.hv(f1, f2, half, v), b.hv(f1, f2, half, v)
            print("hv  ", f1, f2, half, np.abs(ha - hb).max() / np.abs(ha).max())
        a.solve_block(f1, f2)
        b.solve_block(f1, f2)
        for what in "WHPQ":
            bi = ocffm.block_index(f1, f2, f)
            xa, xb = a.get(what, bi), b.get(what, bi)
            print("state", f1, f2, what, np.abs(xa - xb).max() / np.abs(xa).max())
        print("cg", a.cg_log()[-2:], b.cg_log()[-2:])
