"""Run-to-run bit-identity of fp32 epochs under execution knobs (bisecting
an order-dependent sum).  Usage: python tools/det_check.py [epochs]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
import ocffm  # noqa: E402
import synth  # noqa: E402

CONFIGS = [dict(kv.split("=") for kv in a.split(",")) if a != "-" else {} for a in sys.argv[2:]] or [{}]


def run(ds, kw, epochs):
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, with_test=False, **kw)
    ocffm.srand(1)
    g.init()
    snaps = []
    for e in range(epochs):
        g.one_epoch()
        snaps.append([g.get(w, b) for b in range(g.n_blocks()) for w in "WH"
                      if kw.get("self_side", True) or b in blocks(g)])
    cg = g.cg_log().copy()
    g.close()
    return snaps, cg


def blocks(g):
    f = g.f
    fu = f - 1
    return {f2 + (f - 1) * f1 - f1 * (f1 - 1) // 2 for f1 in range(fu) for f2 in range(fu, f)}


def main():
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ds = synth.cfg5(m=20000, n=3000, d_user=2000, seed=3)
    kw = dict(k=32, self_side=False)
    for cfg in CONFIGS:
        for k in list(os.environ):
            if k.startswith("OCFFM_"):
                del os.environ[k]
        os.environ.update(cfg)
        a, ca = run(ds, kw, epochs)
        b, cb = run(ds, kw, epochs)
        c, cc = run(ds, kw, epochs)
        for bb, cbb in ((b, cb), (c, cc), (c, cc) if False else (b, cb)):
          res = []
          for e in range(epochs):
            diff = [i for i, (x, y) in enumerate(zip(a[e], bb[e])) if not np.array_equal(x, y)]
            res.append(f"epoch {e + 1}: {len(diff)} tables differ" + (f" (first {diff[0]})" if diff else ""))
          print(cfg, "cg equal" if np.array_equal(ca, cbb) else "cg DIFFER", "; ".join(res), flush=True)
          if not np.array_equal(ca, cbb):
            dd = np.where(ca != cbb)[0]
            print("   first cg diff at half", dd[0], "counts", ca[dd[0]-2:dd[0]+3].tolist(), cbb[dd[0]-2:dd[0]+3].tolist(), flush=True)
        d12 = [e for e in range(epochs) if any(not np.array_equal(x, y) for x, y in zip(b[e], c[e]))]
        print("   run1 vs run2:", "equal" if not d12 else f"differ from epoch {d12[0] + 1}", flush=True)
        continue
        res = []
        for e in range(epochs):
            diff = [i for i, (x, y) in enumerate(zip(a[e], b[e])) if not np.array_equal(x, y)]
            res.append(f"epoch {e + 1}: {len(diff)} tables differ" + (f" (first {diff[0]})" if diff else ""))
        print(cfg, "cg equal" if np.array_equal(ca, cb) else "cg DIFFER", "; ".join(res), flush=True)


if __name__ == "__main__":
    main()
