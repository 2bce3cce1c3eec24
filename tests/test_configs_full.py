"""BASELINE configs[1] and configs[3] at their SURVEY §8d sizes (one GPU).

* kdd12-shape: m = 500 k users, n = 50 k ads, k = 16, user fields UserID and
  {QueryID, Depth}, ad fields TitleID, DescriptionID, KeywordID and {AdID,
  DisplayURL, AdvertiserID} (script/kdd12.tools/user_ffm.py:5-7,
  ad_ffm.py:5-9), ~3 positives per row.
* outbrain-shape: one GPU's 250 k-row shard of the 2 M-row 8-GPU run, n =
  10 k ads, k = 64, context fields {platform, geo} and {source, publisher,
  document}, ad fields {source, publisher, document} and {campaign,
  advertiser} (script/outbrain.tools/context_ffm.py:6-7, item_ffm.py:6-7),
  ~1 positive per row.

The fp64 oracle cannot run these sizes inside a test (the structures are
parity-tested at m = 400 in test_gpu_parity.py::test_variants_fp64), so the
checks are size-independent properties of one fp32 epoch, as for the kkbox
and config-5 sizes:
  * every half's CG count is in 1..20 (ffm.cpp:761-762), 2 halves per block;
  * y~ is finite and both orientations hold the same values (ffm.cpp:455,462);
  * P = X W still holds on sampled rows after the epoch's incremental
    updates P += X S (ffm.cpp:439-449), for every cross block's user table
    (multi-node fields: the sum over the row's nodes of the field);
  * validation on 2,000 test rows gives a finite loss, p@k / nDCG@k in [0, 1].
"""
import numpy as np
import pytest

import ocffm
import oracle_lib as O
import synth

pytestmark = pytest.mark.gpu


def _check(ds, k, samples=5000):
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, k=k)
    ocffm.srand(1)
    g.init()
    g.one_epoch()
    fu = int(ds.train.fid.max()) + 1
    fv = int(ds.item.fid.max()) + 1
    f = fu + fv
    cg = g.cg_log()
    assert cg.size == f * (f + 1) and cg.min() >= 1 and cg.max() <= 20, cg
    yu, yv = g.get("u"), g.get("v")
    assert yu.size == ds.n_positives and np.isfinite(yu).all()
    assert np.array_equal(np.sort(yu), np.sort(yv))
    m = ds.train.m
    rng = np.random.default_rng(0)
    rows = rng.choice(m, min(samples, m), replace=False)
    xptr = np.asarray(ds.train.xptr, dtype=np.int64)
    fid = np.asarray(ds.train.fid)
    idx = np.asarray(ds.train.idx, dtype=np.int64)
    val = np.asarray(ds.train.val)
    for f1 in range(fu):
        for f2 in range(fu, f):
            b12 = O.block_index(f1, f2, f)
            W = g.get("W", b12).reshape(-1, k)
            P = g.get("P", b12).reshape(-1, k)
            ref = np.zeros((rows.size, k))
            for t, i in enumerate(rows):
                for p in range(xptr[i], xptr[i + 1]):
                    if fid[p] == f1:
                        ref[t] += val[p] * W[idx[p]]
            assert np.abs(P[rows] - ref).max() <= 1e-5 * max(1e-30, np.abs(ref).max()), (f1, f2)
    met = g.validate()
    assert np.isfinite(met["loss"])
    assert np.all((met["prec"] >= 0) & (met["prec"] <= 1))
    assert np.all((met["ndcg"] >= 0) & (met["ndcg"] <= 1))
    g.close()


@pytest.mark.timeout(300)
def test_kdd12_full_size_properties():
    _check(synth.kdd12(test_rows=2000), 16)


@pytest.mark.timeout(300)
def test_outbrain_shard_properties():
    _check(synth.outbrain(test_rows=2000), 64)
