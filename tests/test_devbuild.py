"""On-device data layout build (devbuild.h) against the
host build (all `-m gpu`).

The device build does ImpData::split_fields (ffm.cpp:185-257), the
item-major transpose of transY (ffm.cpp:259-294), the item popularity
(ffm.cpp:143,172-176) and this repo's CSCs, feature-pass jobs and positive
segments with histograms, scans and stable radix sorts.  The host build
(OCFFM_HOST_BUILD=1) restates the reference's sequential loops.  Every array
of the layout must be bit-identical: ocffm_problem_layout_digest hashes each
one (names in the failure message), over data sets that reach every branch:
test rows, several nodes per field, duplicate features inside a row,
rows/items without positives and empty columns, heavy (multi-chunk)
columns, multi-segment rows, one-node and id-like fields, --freq, --ns with
39 user fields, k = 64 (another subgroup count), both precisions, and the
two-rank sharding with its owned-field masks.
"""
import numpy as np
import pytest

import ocffm
import synth

pytestmark = pytest.mark.gpu

HEAVY = dict(seed=13, m=1500, n=300, fu=2, fv=2, k=8, d_user=[1500, 3], d_item=[300, 2], nnz_user=1,
             mean_pos=12.0, vals="real")


def _with_duplicates(ds):
    """Every train row gets a copy of its first node (same fid and idx,
    half the value) at its end: a feature twice in one row."""
    r = ds.train
    feats = []
    for i in range(r.m):
        a, b = int(r.xptr[i]), int(r.xptr[i + 1])
        row = [(int(r.fid[p]), int(r.idx[p]), float(r.val[p])) for p in range(a, b)]
        if row:
            row.append((row[0][0], row[0][1], row[0][2] * 0.5))
        feats.append(row)
    labels = [r.ycol[int(r.yptr[i]):int(r.yptr[i + 1])] for i in range(r.m)]
    ds.train = synth._build_rows(feats, labels)
    ds.name += "_dup"
    return ds


def _digest(monkeypatch, ds, host, precision=ocffm.FP32, env=None, **kw):
    if host:
        monkeypatch.setenv("OCFFM_HOST_BUILD", "1")
    else:
        monkeypatch.delenv("OCFFM_HOST_BUILD", raising=False)
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    g = ocffm.problem_from_dataset(ds, precision=precision, **kw)
    d = g.layout_digest()
    g.close()
    return d


def _compare(dev, host):
    assert list(dev) == list(host)
    bad = [n for n in dev if dev[n] != host[n]]
    assert not bad, f"device build differs from the host build in {bad}"


CASES = {
    "tiny": lambda: (synth.tiny(seed=4), {}, {}),
    "multi_nnz_dup": lambda: (_with_duplicates(synth.general(seed=9, m=150, n=70, fu=3, fv=2, k=8, nnz_user=3,
                                                             mean_pos=40.0, vals="real", test_rows=30)), {}, {}),
    "sparse": lambda: (synth.general(seed=13, m=120, n=90, fu=2, fv=2, k=4, d_user=[300, 7], d_item=[200, 5],
                                     mean_pos=0.7, test_rows=20), {}, {}),
    "heavy_cgram": lambda: (synth.general(**HEAVY), {}, {"OCFFM_CGRAM": "2"}),
    "kkbox_seg3": lambda: (synth.kkbox(m=3000, n=4000, mean=20.0, seed=11, name="kk_det"), {},
                           {"OCFFM_SEG_LEN": "3"}),
    "freq": lambda: (synth.tiny(seed=5), {"freq": True}, {}),
    "wide_ns_k64": lambda: (synth.general(seed=41, m=300, n=60, fu=39, fv=1, k=64, d_user=[50] * 39, d_item=[60],
                                          mean_pos=3.0, test_rows=30), {"k": 64, "self_side": False}, {}),
}


@pytest.mark.parametrize("precision", [ocffm.FP32, ocffm.FP64])
@pytest.mark.parametrize("case", list(CASES))
def test_device_build_equals_host_build(monkeypatch, case, precision):
    ds, kw, env = CASES[case]()
    dev = _digest(monkeypatch, ds, False, precision, env, **kw)
    host = _digest(monkeypatch, ds, True, precision, env, **kw)
    _compare(dev, host)


@pytest.mark.parametrize("owned", [False, True])
def test_device_build_two_rank_shards(monkeypatch, owned):
    """Each rank's shard (users split contiguously; all-item counts for the
    item side halves; owned-field masks of a listener-id field)."""
    if owned:  # field 0: one id per user (D = m), owned by the rank of its row
        ds = synth.general(seed=21, m=400, n=50, fu=2, fv=2, k=8, d_user=[400, 9], d_item=[50, 6], mean_pos=4.0,
                           test_rows=40)
        r = ds.train
        r.idx[r.fid == 0] = np.arange(r.m, dtype=np.uint64)
    else:
        ds = synth.tiny(seed=7)

    def never(arr):  # create() does not all-reduce
        raise AssertionError("all-reduce during set-up")

    for rank in range(2):
        dev = _digest(monkeypatch, ds, False, rank=rank, nranks=2, allreduce=never)
        host = _digest(monkeypatch, ds, True, rank=rank, nranks=2, allreduce=never)
        _compare(dev, host)
        if owned:
            assert any(n.endswith(".own") and dev[n] != 0 for n in dev)


def test_device_build_trains_like_host_build(monkeypatch):
    """Same layout, same arithmetic: fp32 epochs bit-identical."""
    ds = synth.kkbox(m=3000, n=4000, mean=20.0, seed=11, name="kk_det")
    out = []
    for host in (False, True):
        if host:
            monkeypatch.setenv("OCFFM_HOST_BUILD", "1")
        else:
            monkeypatch.delenv("OCFFM_HOST_BUILD", raising=False)
        g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, with_test=False)
        ocffm.srand(1)
        g.init()
        g.one_epoch()
        g.one_epoch()
        out.append((g.get("W", 1).copy(), g.get("u").copy(), g.cg_log().copy()))
        g.close()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("precision", [ocffm.FP32, ocffm.FP64])
@pytest.mark.parametrize("k", [1, 5, 32, 37, 64, 100])
def test_device_draw_equals_host_draw(monkeypatch, precision, k):
    """init_mat (ffm.cpp:71-78) drawn on the device (minstd_rand0 jump-ahead,
    generate_canonical, uniform_real_distribution) equals the host draw of
    init_table bit for bit (and P, Q = X W, X H computed from them)."""
    ds = synth.tiny(seed=3, m=300)
    tabs = []
    for host in (False, True):
        if host:
            monkeypatch.setenv("OCFFM_HOST_INIT", "1")
        else:
            monkeypatch.delenv("OCFFM_HOST_INIT", raising=False)
        g = ocffm.problem_from_dataset(ds, precision=precision, with_test=False, k=k)
        ocffm.srand(1)
        g.init()
        tabs.append([g.get(w, b).copy() for b in range(g.n_blocks()) for w in "WHPQ"])
        g.close()
    for a, b in zip(tabs[0], tabs[1]):
        np.testing.assert_array_equal(a, b)
