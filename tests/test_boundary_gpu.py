"""The drop-in boundary pinned on the HIP path (all `-m gpu`).

1. The reference's nDCG known-answer test (script/nDCG_degub_tool) run
   through the GPU ranking kernel: ocffm_problem_validate_forced forces the
   scores to z_j = n - j as the reference's EBUG_nDCG build does
   (ffm.cpp:988-993); per-row nDCG@10 must equal gen_ans.py's values
   (tests/golden/ndcg_kat/expected_ndcg10.txt, 4 d.p., as the build prints).
2. The text model writer (ffm.cpp:1163-1237) byte-exact: the oracle's fp64
   tables loaded into the GPU problem give the identical model file.
3. The binary snapshot in the reference's save_binary_model layout
   (ffm.cpp:1239-1267) and the load the reference meant to write
   (ffm.cpp:1269-1301): the oracle's file loads bit-exactly, training goes on
   as the oracle's does, and saving again reproduces the file byte for byte.
"""
import os
import struct

import numpy as np
import pytest

import ocffm
import oracle_lib as O
import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ndcg_kat")


def _pair(ds, **kw):
    o = O.Oracle(ds, **kw)
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, **kw)
    ocffm.srand(1)
    o.init()
    ocffm.srand(1)
    g.init()
    return o, g


@pytest.mark.parametrize("train,test", [("case1.mf", "case1.mf"), ("case1.mf", "user1.mf"),
                                        ("user1.mf", "user1.mf")])
def test_ndcg_known_answer_on_gpu(train, test):
    # readme:10: `train -k 8 -t 1 -p case1.mf test_item.mf case1.mf`; user1.mf
    # (the tool's second label file) as the test rows too
    U = ocffm.ImpData.read(os.path.join(GOLD, train), True)
    V = ocffm.ImpData.read(os.path.join(GOLD, "test_item.mf"), False)
    V.trans_y(U)
    Ut = ocffm.ImpData.read(os.path.join(GOLD, test), True, U.Ds)
    prm = ocffm.Parameter(k=8, nr_pass=1, precision=ocffm.FP64)
    g = ocffm.ImpProblem(U, Ut, V, prm)
    ocffm.srand(1)
    g.init()
    met, rows = g.validate_forced()
    # gen_ans.py's ndcg() (gen_ans.py:24-26) at k = 5, 10, 20, 40, 80
    expected = np.loadtxt(os.path.join(GOLD, "expected_ndcg_" + test.replace(".mf", ".txt")))
    assert rows.shape == expected.shape == (20, 5)
    np.testing.assert_allclose(rows, expected, rtol=0, atol=1e-12)
    if test == "case1.mf":  # gen_ans.py's printout, 4 d.p., as the build prints
        np.testing.assert_array_equal(np.round(rows[:, 1], 4), np.loadtxt(os.path.join(GOLD, "expected_ndcg10.txt")))
    # the run's nDCG@k is the mean of the per-row values (ffm.cpp:1012-1015)
    np.testing.assert_allclose(met["ndcg"], rows.mean(axis=0), rtol=0, atol=1e-12)
    g.close()


def test_validate_forced_rejects_small_buffer():
    """The per-row buffer's capacity is checked (5 doubles per test row)."""
    import ctypes as C
    U = ocffm.ImpData.read(os.path.join(GOLD, "case1.mf"), True)
    V = ocffm.ImpData.read(os.path.join(GOLD, "test_item.mf"), False)
    V.trans_y(U)
    Ut = ocffm.ImpData.read(os.path.join(GOLD, "case1.mf"), True, U.Ds)
    g = ocffm.ImpProblem(U, Ut, V, ocffm.Parameter(k=8, nr_pass=1, precision=ocffm.FP64))
    ocffm.srand(1)
    g.init()
    assert g.test_rows() == 20
    m = ocffm._Metrics()
    buf = np.zeros(99)
    assert ocffm.lib().ocffm_problem_validate_forced(g.h, C.byref(m), buf.ctypes.data_as(C.c_void_p), 99) \
        == ocffm.E_ARG
    g.close()


def _state_blocks(o):
    return [O.block_index(f1, f2, o.f) for f1 in range(o.f) for f2 in range(f1, o.f)
            if o.self_side or (f1 < o.fu <= f2)]


@pytest.mark.parametrize("self_side", [True, False])
def test_text_model_byte_exact(tmp_path, self_side):
    ds = synth.tiny(seed=12)
    o, g = _pair(ds, self_side=self_side)
    o.one_epoch()
    for b12 in _state_blocks(o):  # the oracle's fp64 tables, bit for bit
        g.set("W", b12, o.get("W", b12))
        g.set("H", b12, o.get("H", b12))
    o.save_model(str(tmp_path / "cpu.model"))
    g.save_model(str(tmp_path / "gpu.model"))
    a = (tmp_path / "cpu.model").read_bytes()
    b = (tmp_path / "gpu.model").read_bytes()
    assert len(a) > 1000 and a == b


def _read_binary(path):
    """The reference's save_binary_model layout (ffm.cpp:1239-1267)."""
    raw = open(path, "rb").read()
    f, fu, fv, k = struct.unpack_from("<4I", raw, 0)
    off = 16
    ds = struct.unpack_from(f"<{fu + fv}Q", raw, off)
    off += 8 * (fu + fv)
    blocks = {}
    while off < len(raw):
        b12, nw, nh = struct.unpack_from("<IQQ", raw, off)
        off += 20
        w = np.frombuffer(raw, np.float64, nw, off)
        off += 8 * nw
        h = np.frombuffer(raw, np.float64, nh, off)
        off += 8 * nh
        blocks[b12] = (w, h)
    return (f, fu, fv, k), ds, blocks


@pytest.mark.parametrize("self_side", [True, False])
def test_binary_snapshot_roundtrip(tmp_path, self_side):
    ds = synth.general(seed=17, m=150, n=60, fu=2, fv=2, k=6, nnz_user=2, mean_pos=3.0, vals="real", test_rows=20)
    o = O.Oracle(ds, self_side=self_side)
    ocffm.srand(1)
    o.init()
    o.one_epoch()
    po = str(tmp_path / "cpu.bin")
    o.save_binary(po)
    (f, fu, fv, k), dsz, blocks = _read_binary(po)
    assert (f, fu, fv, k) == (o.f, o.fu, o.fv, o.k)
    assert sorted(blocks) == sorted(_state_blocks(o))
    for b12, (w, h) in blocks.items():
        np.testing.assert_array_equal(w, o.get("W", b12))
        np.testing.assert_array_equal(h, o.get("H", b12))
    # a fresh GPU problem restored from the oracle's file (no init)
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, self_side=self_side)
    g.load_binary(po)
    for b12 in _state_blocks(o):
        np.testing.assert_array_equal(g.get("W", b12), o.get("W", b12))
        np.testing.assert_array_equal(g.get("H", b12), o.get("H", b12))
        for what in "PQ":
            a, b = g.get(what, b12), o.get(what, b12)
            assert np.abs(a - b).max() <= 1e-12 * np.abs(b).max(), (what, b12)
    for what in "abuv":
        a, b = g.get(what), o.get(what)
        assert np.abs(a - b).max() <= 1e-9 * max(1.0, np.abs(b).max()), what
    pg = str(tmp_path / "gpu.bin")
    g.save_binary(pg)
    assert open(pg, "rb").read() == open(po, "rb").read()
    # training goes on as the oracle's
    o.cg_log_clear()
    o.one_epoch()
    g.one_epoch()
    np.testing.assert_array_equal(g.cg_log(), o.cg_log())
    for b12 in _state_blocks(o):
        for what in "WH":
            a, b = g.get(what, b12), o.get(what, b12)
            assert np.abs(a - b).max() <= 1e-9 * np.abs(b).max(), (what, b12)
    vo, vg = o.validate(), g.validate()
    assert abs(vg["loss"] - vo["loss"]) <= 1e-9 * vo["loss"]
    g.close()


def test_binary_snapshot_rejects_other_problem(tmp_path):
    ds = synth.tiny(seed=3)
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
    ocffm.srand(1)
    g.init()
    p = str(tmp_path / "m.bin")
    g.save_binary(p)
    other = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, k=5)
    with pytest.raises(ocffm.OcffmError) as e:
        other.load_binary(p)
    assert e.value.code == ocffm.E_DATA
    raw = open(p, "rb").read()
    open(p, "wb").write(raw[: len(raw) // 2])
    g2 = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
    with pytest.raises(ocffm.OcffmError) as e:
        g2.load_binary(p)
    assert e.value.code == ocffm.E_DATA


def test_binary_load_failure_leaves_state(tmp_path):
    """A short or padded file is rejected before the device state is touched
    (solver.hip load_binary reads and checks the whole file first): an
    initialised problem keeps its tables and trains on exactly as before."""
    ds = synth.tiny(seed=3)
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
    ocffm.srand(1)
    g.init()
    g.one_epoch()
    p = str(tmp_path / "m.bin")
    g.save_binary(p)
    g.one_epoch()  # the file now differs from the live tables
    o = O.Oracle(ds)
    before = {(w, b): g.get(w, b) for b in _state_blocks(o) for w in "WHPQ"}
    raw = open(p, "rb").read()
    for bad in (raw[:-8], raw + b"\0" * 8):
        open(p, "wb").write(bad)
        with pytest.raises(ocffm.OcffmError) as e:
            g.load_binary(p)
        assert e.value.code == ocffm.E_DATA
        for (w, b), t in before.items():
            np.testing.assert_array_equal(g.get(w, b), t)
    # training goes on bit-identically to a twin that never saw the bad files
    twin = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
    ocffm.srand(1)
    twin.init()
    twin.one_epoch()
    twin.one_epoch()
    g.one_epoch()
    twin.one_epoch()
    for b in _state_blocks(o):
        np.testing.assert_array_equal(g.get("W", b), twin.get("W", b))
    g.close()
    twin.close()
