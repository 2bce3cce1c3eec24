"""CPU tests of the product boundary: the C-ABI library loads and exports
every symbol include/ocffm.h declares; the host data layer (parser, per-field
CSR, transY) reproduces the reference's ImpData on edge-case inputs; the CLI
keeps train.cpp's argv grammar and exit codes.  No GPU compute here."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import ocffm
import oracle_lib as O
import synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ocffm.h")
TRAIN = os.path.join(REPO, "one-class-ffm_amd", "train")


def header_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(ocffm_[a-z_0-9]+)\s*\(", text)) - {"ocffm_allreduce_fn"})


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(ocffm.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(ocffm.EXPORTS) == syms


def test_param_defaults_are_reference_code_defaults():
    p = ocffm.Parameter()
    # ffm.h:48: omega 0.1, lambda 1e-5, r -1, nr_pass 20, k 4, threads 1, self_side
    assert (p.omega, p.lambda_, p.r, p.nr_pass, p.k, p.nr_threads, p.self_side, p.freq) == \
        (0.1, 1e-5, -1.0, 20, 4, 1, 1, 0)
    assert p.precision == ocffm.FP64


EDGE_TRAIN = """0,3 0:1:1 1:2:0.5
2 0:0:1

1,1,4 1:7:2.5 0:2:1
3\t0:4:1  1:0:1\r
0 0:1:1 1:1:
5,2 0:9:1 bad 1:3:1
"""
EDGE_ITEM = """0:0:1 1:1:1
0:1:1
0:2:1 1:0:0.25

0:4:1
0:5:1
"""
EDGE_TEST = """1 0:1:1 1:99:1
4 0:50:1
0,2 1:2:1 2:1:1
"""


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_parser_matches_reference_semantics(tmp_path):
    tr = _write(tmp_path, "tr", EDGE_TRAIN)
    it = _write(tmp_path, "it", EDGE_ITEM)
    te = _write(tmp_path, "te", EDGE_TEST)
    U = ocffm.ImpData.read(tr, True)
    V = ocffm.ImpData.read(it, False)
    V.trans_y(U)
    Ut = ocffm.ImpData.read(te, True, U.Ds)
    oU = O.data_read(tr, True)
    oV = O.data_read(it, False)
    oUt = O.data_read(te, True, O.data_ds(oU))
    L = O.lib()
    for mine, ref in ((U, oU), (V, oV), (Ut, oUt)):
        info = mine.info
        assert info["m"] == L.orc_data_m(ref)
        assert info["f"] == L.orc_data_f(ref)
        np.testing.assert_array_equal(mine.Ds, O.data_ds(ref))
    # the empty line re-uses the previous label block (ffm.cpp:93) and counts as a row
    assert U.info["m"] == 7
    assert U.info["nnz_y"] == 2 + 1 + 1 + 3 + 1 + 1 + 2
    # test features with idx >= train Ds are dropped (ffm.cpp:104,149)
    assert Ut.info["nnz_x"] == 1 + 0 + 1


def test_bad_label_is_invalid_argument(tmp_path):
    tr = _write(tmp_path, "tr", "1,,2 0:1:1\n")
    with pytest.raises(ocffm.OcffmError) as e:
        ocffm.ImpData.read(tr, True)
    assert e.value.code == ocffm.E_ARG


def test_missing_file_is_io_error(tmp_path):
    with pytest.raises(ocffm.OcffmError) as e:
        ocffm.ImpData.read(str(tmp_path / "nope"), True)
    assert e.value.code == ocffm.E_IO


def test_rows_and_text_give_identical_data(tiny, tmp_path):
    paths = tiny.write(str(tmp_path))
    a = ocffm.ImpData.read(paths["train"], True)
    b = ocffm.ImpData.from_rows(tiny.train)
    assert a.info == b.info
    np.testing.assert_array_equal(a.Ds, b.Ds)


def test_cli_usage_and_errors(tmp_path):
    r = subprocess.run([TRAIN], capture_output=True, text=True)
    assert r.returncode == 1 and "usage: train" in r.stderr
    r = subprocess.run([TRAIN, "-k"], capture_output=True, text=True)
    assert r.returncode == 1
    r = subprocess.run([TRAIN, "-k", "abc", "a", "b"], capture_output=True, text=True)
    assert r.returncode == 1 and "number" in r.stderr
    r = subprocess.run([TRAIN, "only_one_path"], capture_output=True, text=True)
    assert r.returncode == 1


def test_problem_needs_trans_y_and_valid_labels(tiny):
    U = ocffm.ImpData.from_rows(tiny.train)
    V = ocffm.ImpData.from_rows(tiny.item)
    with pytest.raises(ocffm.OcffmError) as e:
        ocffm.ImpProblem(U, None, V, ocffm.Parameter())
    # without a GPU the create call fails loudly with E_HIP before the check
    assert e.value.code in (ocffm.E_STATE, ocffm.E_HIP)
