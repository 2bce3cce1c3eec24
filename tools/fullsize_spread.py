"""The reference arithmetic's own spread at the kdd12 and outbrain shapes'
full sizes (500 k users x 50 k ads, k = 16; config 4:
one GPU's 250 k-row shard, 10 k ads, k = 64), for
tests/test_gpu_parity.py::test_{kdd12,outbrain}_full_size_parity_fp64.

One fp64 epoch of the oracle from the srand(1) init at 1, 3, 4 and 16
threads and at 8 threads with two cblas_ddot orders of optimised BLAS builds
(oracle Problem::dot), then validate() on a 500-row test split.  At this
size the reference's own CG counts differ between these runs (kdd12: up to
6 of the 42 halves; the ad fields' halves end at the 20-step cap or near
the 0.09 threshold), so no state parity is defined; the validation metrics
are compared instead.  Writes tests/golden/<shape>_full_spread.json: per
metric the range (max - min) over the runs, and the most CG counts two runs
differ in.  CPU only (kdd12 ~3 min, outbrain ~10 min on 8 cores).

    python tools/fullsize_spread.py kdd12|outbrain
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

RUNS = [(1, None), (3, None), (4, None), (16, None), (8, (4, 1)), (8, (16, 8))]


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "kdd12"
    ds = getattr(synth, shape)(test_rows=500)
    runs = []
    for th, dot in RUNS:
        o = O.Oracle(ds, threads=th, with_test=True)
        if dot:
            o.set_dot_order(*dot)
        O.lib().orc_srand(1)
        o.init()
        o.one_epoch()
        v = o.validate()
        runs.append(dict(threads=th, dot=dot, loss=float(v["loss"]), prec=v["prec"].tolist(),
                         ndcg=v["ndcg"].tolist(), cg=o.cg_log().tolist()))
        print(th, dot, v["loss"], v["prec"], v["ndcg"], flush=True)
    loss = np.array([r["loss"] for r in runs])
    prec = np.array([r["prec"] for r in runs])
    ndcg = np.array([r["ndcg"] for r in runs])
    cg = np.array([r["cg"] for r in runs])
    cgd = max(int(np.sum(a != b)) for a in cg for b in cg)
    out = dict(what=f"range (max - min) over the oracle runs of one fp64 epoch of synth.{shape}(test_rows=500)",
               runs=runs, loss_range=float(loss.max() - loss.min()), prec_range=(prec.max(0) - prec.min(0)).tolist(),
               ndcg_range=(ndcg.max(0) - ndcg.min(0)).tolist(), cg_halves_differ=cgd)
    path = os.path.join(REPO, "tests", "golden", f"{shape}_full_spread.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "runs"}))


if __name__ == "__main__":
    main()
