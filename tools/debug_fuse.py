"""Compare gradients / Hessian-vector products of every half with the id-field
row fusion (OCFFM_FUSE=2) against the default (FUSE=1), fp64."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "one-class-ffm_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402

import ocffm  # noqa: E402
import synth  # noqa: E402

seg = os.environ.get("SEG", "32")
os.environ["OCFFM_SEG_LEN"] = seg
ds = synth.kkbox(m=1500, n=2000, mean=20.0, seed=3, name="dbg")
res = {}
for fz in ("1", "2"):
    os.environ["OCFFM_FUSE"] = fz
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, with_test=False)
    ocffm.srand(1)
    g.init()
    rng = np.random.default_rng(0)
    out = {}
    f = 5
    for f1 in range(f):
        for f2 in range(f1, f):
            for half in (0, 1):
                G = g.grad(f1, f2, half)
                v = rng.standard_normal(G.size)
                out[(f1, f2, half)] = (G, g.hv(f1, f2, half, v))
    res[fz] = out
    g.close()
for k in res["1"]:
    a, b = res["1"][k], res["2"][k]
    eg = np.abs(a[0] - b[0]).max() / max(1e-300, np.abs(a[0]).max())
    eh = np.abs(a[1] - b[1]).max() / max(1e-300, np.abs(a[1]).max())
    flag = "  <-- DIFF" if max(eg, eh) > 1e-12 else ""
    print(k, f"grad {eg:.2e} hv {eh:.2e}{flag}")
