"""BASELINE configs[4] at full per-GPU size (SURVEY §8d restated: one GPU's
row shard of the 100 M-row, 8-GPU run): --ns, 39 user fields of 250,000
features, 1 item field (250,000 items), k = 64, 12,500,000 rows, fp32.  The
39 user-side P caches alone are 39 x 12.5 M x 64 x 4 B = 125 GB, so every pass
streams from HBM, not from the 256 MB Infinity Cache.

The fp64 oracle cannot run this size in a test, so the checks are
size-independent properties of one epoch (the structure itself is
parity-tested at small size in test_gpu_parity.py::test_cfg5_shape_*):
  * every half's CG count is in 1..20 (ffm.cpp:761-762) and 78 halves ran;
  * y~ is finite and both orientations hold the same values (ffm.cpp:455,462);
  * P = X W still holds on sampled rows after the epoch's incremental
    updates P += X S (ffm.cpp:439-449), for the first and last block;
  * validation over 2,000 test rows x 250,000 items gives a finite loss and
    p@k / nDCG@k in [0, 1].
"""
import time

import numpy as np
import pytest

import ocffm
import oracle_lib as O
import synth

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(400)
def test_cfg5_full_size_properties():
    m, fu, k = 12_500_000, 39, 64
    t0 = time.perf_counter()
    ds = synth.cfg5(m=m, test_rows=2000)
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, self_side=False, k=k)
    ocffm.srand(1)
    g.init()
    g.one_epoch()
    cg = g.cg_log()
    assert cg.size == 2 * fu and cg.min() >= 1 and cg.max() <= 20
    yu, yv = g.get("u"), g.get("v")
    assert yu.size == ds.n_positives and np.isfinite(yu).all()
    assert np.array_equal(np.sort(yu), np.sort(yv))
    rng = np.random.default_rng(0)
    rows = rng.choice(m, 20000, replace=False)
    idx = np.asarray(ds.train.idx).reshape(m, fu)
    for f1 in (0, fu - 1):
        b12 = O.block_index(f1, fu, fu + 1)
        W = g.get("W", b12).reshape(-1, k)
        P = g.get("P", b12).reshape(-1, k)
        ref = W[idx[rows, f1]]
        assert np.abs(P[rows] - ref).max() <= 1e-5 * np.abs(ref).max(), f1
        del W, P
    met = g.validate()
    assert np.isfinite(met["loss"])
    assert np.all((met["prec"] >= 0) & (met["prec"] <= 1))
    assert np.all((met["ndcg"] >= 0) & (met["ndcg"] <= 1))
    g.close()
    print(f"config-5 shard of {m} rows: {time.perf_counter() - t0:.1f} s for data, one epoch and the checks")
