"""fp64 drift of the GPU path against the oracle at the headline size
(kkbox-shape 30,755 x 100,000, k = 32), per execution knob.

The oracle (16 threads) runs E epochs once; each GPU configuration (an env
setting, read at problem creation) runs the same epochs from the same
srand(1) init.  Prints, per configuration and epoch, the max relative
difference over W, H, P, Q of every block, a, b and both y~ orientations,
the worst table, and whether the CG logs agree.

    python tools/fullsize_drift.py [E] [--json out.json] [CONFIG ...]
CONFIG: "default" or VAR=VAL[,VAR=VAL...]
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


def state(x, blocks):
    st = {f"{w}{b}": x.get(w, b) for b in blocks for w in "WHPQ"}
    st.update({w: x.get(w) for w in "abuv"})
    return st


def main():
    args = [a for a in sys.argv[1:]]
    out = None
    if "--json" in args:
        i = args.index("--json")
        out = args[i + 1]
        del args[i:i + 2]
    E = int(args.pop(0)) if args and args[0].isdigit() else 2
    configs = args or ["default", "OCFFM_EXACT_R2=1"]
    ds = synth.kkbox(test_frac=0.05)
    t0 = time.time()
    o = O.Oracle(ds, threads=16, with_test=False)
    blocks = [O.block_index(f1, f2, o.f) for f1 in range(o.f) for f2 in range(f1, o.f)]
    ocffm.srand(1)
    o.init()
    ref = []
    for _ in range(E):
        o.one_epoch()
        ref.append(state(o, blocks))
    cg_ref = o.cg_log().copy()
    print(f"oracle {E} epochs in {time.time() - t0:.1f}s; cg {cg_ref.tolist()}", flush=True)
    res = {}
    for cfg in configs:
        env = {} if cfg == "default" else dict(kv.split("=", 1) for kv in cfg.split(","))
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, with_test=False)
            ocffm.srand(1)
            g.init()
            per = []
            for e in range(E):
                g.one_epoch()
                st = state(g, blocks)
                d = {k: rel(st[k], ref[e][k]) for k in ref[e]}
                worst = max(d, key=d.get)
                per.append({"max": d[worst], "worst": worst,
                            "top": sorted(d.items(), key=lambda kv: -kv[1])[:5]})
            cg = g.cg_log().copy()
            g.close()
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        res[cfg] = {"epochs": per, "cg_equal": bool(np.array_equal(cg, cg_ref)),
                    "cg_diff": [(i, int(a), int(b)) for i, (a, b) in enumerate(zip(cg, cg_ref)) if a != b][:10]}
        print(f"{cfg:40s} " + "  ".join(f"e{e + 1} {p['max']:.2e} ({p['worst']})" for e, p in enumerate(per)) +
              f"  cg_equal={res[cfg]['cg_equal']} {res[cfg]['cg_diff']}", flush=True)
        for e, p in enumerate(per):
            print("    e%d top: %s" % (e + 1, ", ".join(f"{k} {v:.2e}" for k, v in p["top"])), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump({"epochs": E, "cg_ref": cg_ref.tolist(), "configs": res}, f, indent=1)


if __name__ == "__main__":
    main()
