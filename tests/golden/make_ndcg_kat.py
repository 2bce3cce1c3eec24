"""Regenerate the nDCG known-answer fixture (run in the build container only).

The reference's only known-answer test is ``script/nDCG_degub_tool``: a
debug build forces the item scores to z_j = n - j and prints nDCG@10 per
test row; ``gen_ans.py`` computes the expected values independently.  This
script copies the tool's data files (``case1.mf``, ``test_item.mf``) into
``tests/golden/ndcg_kat/`` and runs the reference's ``gen_ans.py`` in a
scratch directory (it opens ``case1.mf`` and writes ``ans.txt`` relative to
its working directory), saving its stdout as ``expected_ndcg10.txt``.

Nothing here is needed at test time: the committed files are the fixture.
"""
import os
import shutil
import subprocess
import sys
import tempfile

REF = "/root/reference/script/nDCG_degub_tool"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ndcg_kat")


def main() -> int:
    os.makedirs(OUT, exist_ok=True)
    for name in ("case1.mf", "test_item.mf"):
        shutil.copyfile(os.path.join(REF, name), os.path.join(OUT, name))
    with tempfile.TemporaryDirectory() as tmp:
        shutil.copyfile(os.path.join(REF, "case1.mf"), os.path.join(tmp, "case1.mf"))
        res = subprocess.run([sys.executable, os.path.join(REF, "gen_ans.py")], cwd=tmp,
                             capture_output=True, text=True, check=True)
    with open(os.path.join(OUT, "expected_ndcg10.txt"), "w") as f:
        f.write(res.stdout)
    print(res.stdout)
    return 0


if __name__ == "__main__":
    sys.exit(main())
