"""Where the fp64 GPU path and the oracle part at the headline size
(kkbox-shape 30,755 x 100,000, k = 32): block by block over one epoch's
schedule (ffm.cpp:852-870, solved with solve_block), printing before each
block the relative difference of both halves' gradient and Hessian-vector
product (the kernels, from the same state) and after it the state difference
(max over W, H, P, Q of every block, a, b, y~) and the CG counts.

    python tools/fullsize_blocks.py [--json out.json] [--small]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

import ocffm  # noqa: E402
import oracle_lib as O  # noqa: E402
import synth  # noqa: E402


def rel(a, b):
    return float(np.abs(a - b).max() / max(1e-300, np.abs(b).max())) if b.size else 0.0


def main():
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    ds = synth.kkbox_small() if "--small" in sys.argv else synth.kkbox(test_frac=0.05)
    o = O.Oracle(ds, threads=16, with_test=False)
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, with_test=False)
    ocffm.srand(1)
    o.init()
    ocffm.srand(1)
    g.init()
    blocks = [O.block_index(f1, f2, o.f) for f1 in range(o.f) for f2 in range(f1, o.f)]
    order = [(f1, f2) for f1 in range(o.fu) for f2 in range(f1, o.fu)]
    order += [(f1, f2) for f1 in range(o.fu, o.f) for f2 in range(f1, o.f)]
    order += [(f1, f2) for f1 in range(o.fu) for f2 in range(o.fu, o.f)]

    def state_diff():
        d = {}
        for b in blocks:
            for w in "WHPQ":
                d[f"{w}{b}"] = rel(g.get(w, b), o.get(w, b))
        for w in "abuv":
            d[w] = rel(g.get(w), o.get(w))
        worst = max(d, key=d.get)
        return d[worst], worst

    rng = np.random.default_rng(0)
    rows = []
    m0, w0 = state_diff()
    print(f"init: state {m0:.2e} ({w0})", flush=True)
    for f1, f2 in order:
        t0 = time.time()
        kern = []
        for half in (0, 1):
            G0, G1 = o.grad(f1, f2, half), g.grad(f1, f2, half)
            v = rng.standard_normal(G0.size)
            H0, H1 = o.hv(f1, f2, half, v), g.hv(f1, f2, half, v)
            kern.append((rel(G1, G0), rel(H1, H0)))
        n0 = len(o.cg_log())
        o.solve_block(f1, f2)
        g.solve_block(f1, f2)
        cgo, cgg = o.cg_log()[n0:].tolist(), g.cg_log()[n0:].tolist()
        m, w = state_diff()
        rows.append({"block": [f1, f2], "grad_hv": kern, "state": m, "worst": w, "cg_oracle": cgo, "cg_gpu": cgg})
        print(f"({f1},{f2}) grad/hv W {kern[0][0]:.1e}/{kern[0][1]:.1e} H {kern[1][0]:.1e}/{kern[1][1]:.1e}  "
              f"state {m:.2e} ({w})  cg {cgo} {cgg}  {time.time() - t0:.1f}s", flush=True)
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
