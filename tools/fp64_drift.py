"""fp64 parity drift, measured (round-3 verdict item 1).

For the sets whose fp64 parity had been held for one epoch only (k = 64 /
100, the wide --ns set, the config-5 shape, heavy columns, outbrain shape),
run E epochs of:
  * the oracle at 1 thread (the checker) and twice at 8 threads — the
    reference's own arithmetic reassociated (per-thread partial sums under
    schedule(guided), ffm.cpp:557,759), i.e. the drift the reference allows
    against itself;
  * the GPU fp64 path with the expanded CG residual (default) and with the
    exact one (OCFFM_EXACT_R2=1: |R|^2 recomputed after R -= alpha Hv, as
    ffm.cpp:807-808).
Prints, per set and epoch, the max relative state difference (W, H, P, Q of
every block, a, b, both y~ orientations) of each run against the 1-thread oracle, and whether the CG logs agree.

    python tools/fp64_drift.py [epochs] [--json out.json]
    python tools/fp64_drift.py [epochs] --envelope tests/golden/fp64_envelope.json [--sets a,b]

--envelope (CPU only): the oracle at 2, 3, 4, 6, 8 and 16 threads, twice
each, and at 8 threads with its cblas_ddot restatement summed in the orders
of optimised BLAS builds (SIMD accumulators, a threaded ddot's chunks:
ffm.cpp:57-60 calls cblas_ddot, whose order the BLAS build decides; round 6);
per set and epoch the largest drift from the 1-thread serial run is the
envelope of the reference's own arithmetic, which the GPU parity tests use
as their bound where it exceeds 1e-9 (tests/test_gpu_parity.py fp64_tol).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

import oracle_lib as O  # noqa: E402
import synth  # noqa: E402


def rel(a, b):
    return float(np.abs(a - b).max() / max(1e-300, np.abs(b).max())) if b.size else 0.0


def names(o):
    return [O.block_index(f1, f2, o.f) for f1 in range(o.f) for f2 in range(f1, o.f)
            if o.self_side or (f1 < o.fu <= f2)]


SETS = {
    "k64": (lambda: synth.tiny(seed=4, m=300), dict(k=64)),
    "k100": (lambda: synth.tiny(seed=4, m=300), dict(k=100)),
    "k128": (lambda: synth.tiny(seed=4, m=300), dict(k=128)),
    "wide_ns": (lambda: synth.general(seed=33, m=200, n=40, fu=39, fv=1, k=8, d_user=[20] * 39, d_item=[40],
                                      mean_pos=3.0, test_rows=20, name="wide_ns"), dict(self_side=False)),
    "cfg5_shape": (lambda: synth.general(seed=41, m=300, n=60, fu=39, fv=1, k=64, d_user=[50] * 39, d_item=[60],
                                         mean_pos=4.0, test_rows=30, name="cfg5_small"), dict(self_side=False, k=64)),
    "heavy": (lambda: synth.general(seed=13, m=1500, n=300, fu=2, fv=2, k=8, d_user=[1500, 3], d_item=[300, 2],
                                    nnz_user=1, mean_pos=12.0, vals="real"), dict()),
    "outbrain": (lambda: synth.general(seed=32, m=400, n=60, fu=2, fv=2, k=64, mean_pos=1.0, test_rows=40,
                                       name="outbrain"), dict(k=64)),
    # the headline configuration at its own size (30,755 x 100,000, k = 32,
    # 2.1 M positives; tests/test_gpu_parity.py test_kkbox_full_size_parity_fp64)
    "kkbox_full": (lambda: synth.kkbox(test_frac=0.05), dict()),
    # config 2 at its own size (500 k x 50 k, k = 16; test_kdd12_full_size_parity_fp64)
    "kdd12_full": (lambda: synth.kdd12(test_rows=500), dict()),
}


def state(x, o=None):
    """Everything the parity tests compare (assert_state): W, H, P, Q of every
    block, the biases and both orientations of y~."""
    o = o or x
    st = {(w, b): x.get(w, b) for b in names(o) for w in "WHPQ"}
    st.update({(w, 0): x.get(w) for w in "abuv"})
    return st


def run_oracle(ds, kw, threads, E, dot=None):
    o = O.Oracle(ds, threads=threads, with_test=False, **kw)
    if dot:
        o.set_dot_order(*dot)
    O.lib().orc_srand(1)
    o.init()
    st = []
    for _ in range(E):
        o.one_epoch()
        st.append(state(o))
    return st, o.cg_log().copy(), o


def run_gpu(ds, kw, E, exact):
    import ocffm
    if exact:
        os.environ["OCFFM_EXACT_R2"] = "1"
    else:
        os.environ.pop("OCFFM_EXACT_R2", None)
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, with_test=False, **kw)
    ocffm.srand(1)
    g.init()
    o = O.Oracle(ds, with_test=False, **kw)
    st = []
    for _ in range(E):
        g.one_epoch()
        st.append(state(g, o))
    cg = g.cg_log().copy()
    g.close()
    os.environ.pop("OCFFM_EXACT_R2", None)
    return st, cg


BLAS_ORDERS = [(4, 1), (16, 1), (32, 1), (16, 8), (16, 16)]


def envelope(E, path, only=None):
    res, cg_res = {}, {}
    E_file = E
    if only and os.path.exists(path):  # add / refresh some sets of an existing envelope
        prev = json.load(open(path))
        res = prev["sets"]
        cg_res = prev.get("cg_differs", {})
        E_file = max(E, prev.get("epochs", E))
    for name, (mk, kw) in SETS.items():
        if only and name not in only:
            continue
        ds = mk()
        ref, cg1, _ = run_oracle(ds, kw, 1, E)
        env = [0.0] * E
        runs = [(th, None) for th in (2, 3, 4, 6, 8, 16) for _ in range(2)]
        # the cblas_ddot order of optimised BLAS builds (Problem::dot): SIMD
        # accumulators (AVX2: 16 doubles in flight, AVX-512: 32), a threaded
        # ddot's contiguous chunks
        runs += [(8, dot) for dot in BLAS_ORDERS]
        cgdiff = 0  # halves whose CG count differs from the 1-thread serial run (the worst variant)
        for th, dot in runs:
            st, cg, _ = run_oracle(ds, kw, th, E, dot)
            nd = int(np.sum(cg != cg1)) if cg.shape == cg1.shape else len(cg1)
            if nd:
                print(f"  {name}: {nd} CG count(s) differ at {th} threads, ddot order {dot}", flush=True)
            cgdiff = max(cgdiff, nd)
            env = [max(env[e], max(rel(st[e][key], ref[e][key]) for key in ref[e])) for e in range(E)]
        res[name] = env
        if cgdiff:
            cg_res[name] = cgdiff
        print(f"{name:11s} " + " ".join(f"{x:.2e}" for x in env) + (f"  cg differs in {cgdiff} halves" if cgdiff else ""),
              flush=True)
    with open(path, "w") as f:
        json.dump({"epochs": E_file, "threads": [2, 3, 4, 6, 8, 16], "repeats": 2,
                   "blas_orders": [list(x) for x in BLAS_ORDERS],
                   "what": "max relative difference (W, H, P, Q, a, b, y~) of the oracle at T threads, and with the "
                           "ddot orders of optimised BLAS builds (lanes, chunks) at 8 threads, vs 1 thread serial, "
                           "per epoch",
                   "sets": res,
                   "cg_differs": cg_res}, f, indent=1)


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 3
    if "--envelope" in sys.argv:
        only = sys.argv[sys.argv.index("--sets") + 1].split(",") if "--sets" in sys.argv else None
        return envelope(E, sys.argv[sys.argv.index("--envelope") + 1], only)
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    gpu = "--cpu-only" not in sys.argv
    only = sys.argv[sys.argv.index("--sets") + 1].split(",") if "--sets" in sys.argv else list(SETS)
    res = {}
    for name in only:
        mk, kw = SETS[name]
        ds = mk()
        ref, cg1, _ = run_oracle(ds, kw, 1, E)
        runs = {"oracle_c8a": run_oracle(ds, kw, 8, E)[:2], "oracle_c8b": run_oracle(ds, kw, 8, E)[:2]}
        if gpu:
            runs["gpu_expanded"] = run_gpu(ds, kw, E, False)
            runs["gpu_exact"] = run_gpu(ds, kw, E, True)
        res[name] = {}
        for rn, (st, cg) in runs.items():
            d = [max(rel(st[e][key], ref[e][key]) for key in ref[e]) for e in range(E)]
            res[name][rn] = {"rel_per_epoch": d, "cg_equal": bool(np.array_equal(cg, cg1))}
            print(f"{name:11s} {rn:13s} " + " ".join(f"{x:.2e}" for x in d) + f"  cg_equal={res[name][rn]['cg_equal']}",
                  flush=True)
    if out:
        with open(out, "w") as f:
            json.dump({"epochs": E, "sets": res}, f, indent=1)


if __name__ == "__main__":
    main()
