"""Per-half CG iteration counts of kkbox-shape epochs (solve order)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "one-class-ffm_amd"))
import ocffm  # noqa: E402
import synth  # noqa: E402

prec = ocffm.FP64 if (len(sys.argv) > 1 and sys.argv[1] == "fp64") else ocffm.FP32
g = ocffm.problem_from_dataset(synth.kkbox(), precision=prec, with_test=False)
ocffm.srand(1)
g.init()
names = []
for f1, f2 in [(0, 0), (0, 1), (1, 1), (2, 2), (2, 3), (2, 4), (3, 3), (3, 4), (4, 4),
               (0, 2), (0, 3), (0, 4), (1, 2), (1, 3), (1, 4)]:
    names += [f"({f1},{f2})W", f"({f1},{f2})H"]
for e in range(4):
    g.one_epoch()
    cg = g.cg_log()[-30:]
    print(f"epoch {e}: total {cg.sum()}  " + " ".join(f"{n}:{c}" for n, c in zip(names, cg)))
