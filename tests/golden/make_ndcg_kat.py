"""Regenerate the nDCG known-answer fixtures (run in the build container only).

The reference's only known-answer test is ``script/nDCG_degub_tool``: a
debug build forces the item scores to z_j = n - j and prints nDCG per test
row; ``gen_ans.py`` computes the expected values independently
(``ndcg(label, rank, k)``, gen_ans.py:24-26, with ``rank = [0..9]``: the
forced order of the tool's 10 items, test_item.mf).

This script copies the tool's data files (``case1.mf``, ``user1.mf``,
``test_item.mf``) into ``tests/golden/ndcg_kat/`` and, in a scratch
directory holding a copy of ``case1.mf`` (the module opens it and writes
``ans.txt`` relative to its working directory when imported), imports the
reference's ``gen_ans.py`` and calls its ``ndcg()`` on every row of
``case1.mf`` and ``user1.mf`` at each k the reference build reports
(top_k = 5, 10, 20, 40, 80; ffm.cpp:901-912, 1059-1128).  With 10 items,
the build's ranking stops after 10 positions (max_z_idx = |popular|,
ffm.cpp:1064-1066) exactly as ``dcg()`` stops at the end of ``rank``.

Outputs (the fixtures; nothing here runs at test time):
  expected_ndcg10.txt     — gen_ans.py's own stdout on case1.mf (4 d.p., k=10)
  expected_ndcg_<file>.txt — per row: nDCG@5 @10 @20 @40 @80, repr precision
"""
import contextlib
import importlib.util
import io
import os
import shutil
import subprocess
import sys
import tempfile

REF = "/root/reference/script/nDCG_degub_tool"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ndcg_kat")
TOP_K = (5, 10, 20, 40, 80)


def labels_of(path):
    rows = []
    with open(path) as f:
        for line in f:
            if line.strip():
                rows.append(list(map(int, line.strip().split()[0].split(","))))
    return rows


def main() -> int:
    os.makedirs(OUT, exist_ok=True)
    for name in ("case1.mf", "user1.mf", "test_item.mf"):
        shutil.copyfile(os.path.join(REF, name), os.path.join(OUT, name))
    with tempfile.TemporaryDirectory() as tmp:
        shutil.copyfile(os.path.join(REF, "case1.mf"), os.path.join(tmp, "case1.mf"))
        # the tool as its readme runs it: stdout = per-row nDCG@10, 4 d.p.
        res = subprocess.run([sys.executable, os.path.join(REF, "gen_ans.py")], cwd=tmp,
                             capture_output=True, text=True, check=True)
        with open(os.path.join(OUT, "expected_ndcg10.txt"), "w") as f:
            f.write(res.stdout)
        # its ndcg() at every k, on both label files
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            spec = importlib.util.spec_from_file_location("gen_ans", os.path.join(REF, "gen_ans.py"))
            mod = importlib.util.module_from_spec(spec)
            with contextlib.redirect_stdout(io.StringIO()):
                spec.loader.exec_module(mod)
        finally:
            os.chdir(cwd)
        for name in ("case1.mf", "user1.mf"):
            lines = []
            for lab in labels_of(os.path.join(OUT, name)):
                lines.append(" ".join(repr(float(mod.ndcg(lab, mod.rank, k))) for k in TOP_K))
            with open(os.path.join(OUT, "expected_ndcg_" + name.replace(".mf", ".txt")), "w") as f:
                f.write("\n".join(lines) + "\n")
            print(name, len(lines), "rows")
    return 0


if __name__ == "__main__":
    sys.exit(main())
