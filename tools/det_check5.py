"""All blocks' W/H/P/Q and the biases across two runs after init and after
each of two epochs: where the first run-to-run difference appears."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
import ocffm  # noqa: E402
import synth  # noqa: E402


def snap(g, fu):
    out = {}
    for f1 in range(fu):
        b = fu + (fu + 1 - 1) * f1 - f1 * (f1 - 1) // 2
        for w in "WHPQ":
            out[f"{w}{f1}"] = g.get(w, b)
    for w in "abuv":
        out[w] = g.get(w)
    return out


def main():
    if len(sys.argv) > 1:
        os.environ["OCFFM_NO_MFMA"] = "1"
    ds = synth.cfg5(m=20000, n=3000, d_user=2000, seed=3)
    fu, k = 39, 32
    runs = []
    for r in range(2):
        g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, with_test=False, k=k, self_side=False)
        ocffm.srand(1)
        g.init()
        s = [snap(g, fu)]
        for e in range(2):
            g.one_epoch()
            s.append(snap(g, fu))
        runs.append(s)
        g.close()
    for t in range(3):
        bad = [key for key in runs[0][t] if not np.array_equal(runs[0][t][key], runs[1][t][key])]
        print(["init", "epoch1", "epoch2"][t], len(bad), "differ:", bad[:12], flush=True)


if __name__ == "__main__":
    main()
