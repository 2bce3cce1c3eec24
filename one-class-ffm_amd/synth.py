"""Seeded synthetic inputs in the reference's text format.

The reference ships no datasets, so every parity test and benchmark runs on
inputs generated here.  Each generator returns a ``Dataset`` holding the three
files the reference's ``train`` binary reads (``train.cpp:163-193``):

* the *train* file: ``j1,j2,... fid:idx:val ...`` per user row (labels are a
  comma-separated list of positive item ids, ``ffm.cpp:92-100``);
* the *item* file: ``fid:idx:val ...`` per item row, no label column;
* an optional *test* file in the train format.

The same content is also kept as flat arrays (row pointers, ``fid``/``idx``/
``val`` nodes, label lists) so the benchmark can hand rows to the C-ABI
without going through the text parser.  Feature values are rounded to three
decimals *before* they are stored, so parsing the text (``strtod``) and using
the arrays give bit-identical doubles.
"""
from __future__ import annotations

import dataclasses
import os
from typing import List, Optional

import numpy as np


@dataclasses.dataclass
class Rows:
    """Rows of one input file (mirrors ``ImpData`` before ``split_fields``)."""

    xptr: np.ndarray  # uint64 [m+1]
    fid: np.ndarray  # uint32 [nnz]
    idx: np.ndarray  # uint64 [nnz]
    val: np.ndarray  # float64 [nnz]
    yptr: Optional[np.ndarray] = None  # uint64 [m+1]
    ycol: Optional[np.ndarray] = None  # uint64 [nnz_y]

    @property
    def m(self) -> int:
        return len(self.xptr) - 1

    def lines(self) -> List[str]:
        out = []
        xptr, fid, idx, val = self.xptr, self.fid, self.idx, self.val
        for i in range(self.m):
            toks = []
            if self.yptr is not None:
                ys = self.ycol[self.yptr[i]:self.yptr[i + 1]]
                toks.append(",".join(str(int(j)) for j in ys))
            for p in range(int(xptr[i]), int(xptr[i + 1])):
                toks.append(f"{int(fid[p])}:{int(idx[p])}:{_fmt(val[p])}")
            out.append(" ".join(toks))
        return out

    def write(self, path: str) -> None:
        with open(path, "w") as f:
            for line in self.lines():
                f.write(line)
                f.write("\n")


def _fmt(v: float) -> str:
    if v == 1.0:
        return "1"
    return repr(float(v))


@dataclasses.dataclass
class Dataset:
    name: str
    train: Rows
    item: Rows
    test: Optional[Rows]
    k: int
    params: dict

    def write(self, directory: str) -> dict:
        os.makedirs(directory, exist_ok=True)
        paths = {
            "train": os.path.join(directory, f"{self.name}.tr.ffm"),
            "item": os.path.join(directory, f"{self.name}.item.ffm"),
        }
        self.train.write(paths["train"])
        self.item.write(paths["item"])
        if self.test is not None:
            paths["test"] = os.path.join(directory, f"{self.name}.te.ffm")
            self.test.write(paths["test"])
        return paths

    @property
    def n_positives(self) -> int:
        return int(self.train.yptr[-1])


def _build_rows(feats: List[List[tuple]], labels: Optional[List[np.ndarray]]) -> Rows:
    m = len(feats)
    counts = np.fromiter((len(f) for f in feats), dtype=np.uint64, count=m)
    xptr = np.zeros(m + 1, dtype=np.uint64)
    np.cumsum(counts, out=xptr[1:])
    nnz = int(xptr[-1])
    fid = np.empty(nnz, dtype=np.uint32)
    idx = np.empty(nnz, dtype=np.uint64)
    val = np.empty(nnz, dtype=np.float64)
    p = 0
    for row in feats:
        for (a, b, c) in row:
            fid[p], idx[p], val[p] = a, b, c
            p += 1
    rows = Rows(xptr, fid, idx, val)
    if labels is not None:
        lc = np.fromiter((len(l) for l in labels), dtype=np.uint64, count=m)
        yptr = np.zeros(m + 1, dtype=np.uint64)
        np.cumsum(lc, out=yptr[1:])
        rows.yptr = yptr
        rows.ycol = (np.concatenate(labels).astype(np.uint64) if m else np.zeros(0, np.uint64))
    return rows


def _fast_rows(m, fields, labels_ptr=None, labels_col=None) -> Rows:
    """Vectorised builder: ``fields`` is a list of (fid, idx[m, c], val[m, c])."""
    per_row = sum(f[1].shape[1] for f in fields)
    xptr = (np.arange(m + 1, dtype=np.uint64) * np.uint64(per_row))
    fid = np.empty((m, per_row), dtype=np.uint32)
    idx = np.empty((m, per_row), dtype=np.uint64)
    val = np.empty((m, per_row), dtype=np.float64)
    c0 = 0
    for (fi, ix, vx) in fields:
        c = ix.shape[1]
        fid[:, c0:c0 + c] = fi
        idx[:, c0:c0 + c] = ix
        val[:, c0:c0 + c] = vx
        c0 += c
    rows = Rows(xptr, fid.reshape(-1), idx.reshape(-1), val.reshape(-1))
    if labels_ptr is not None:
        rows.yptr = labels_ptr.astype(np.uint64)
        rows.ycol = labels_col.astype(np.uint64)
    return rows


def tiny(seed: int = 1, m: int = 1000, n: int = 50, m_test: int = 100) -> Dataset:
    """Config 1: 1,000 rows, fu=2 (D=30, D=20), items fv=1 (D=50), k=4."""
    rng = np.random.default_rng(seed)

    def user_rows(count):
        f0 = rng.integers(0, 30, size=count)
        f1 = rng.integers(0, 20, size=count)
        v1 = np.round(rng.random(count), 3)
        v1 = np.where(v1 == 0.0, 0.001, v1)
        labels = []
        for _ in range(count):
            c = int(rng.integers(1, 6))
            labels.append(np.sort(rng.choice(n, size=c, replace=False)))
        feats = [[(0, int(a), 1.0), (1, int(b), float(c))] for a, b, c in zip(f0, f1, v1)]
        return _build_rows(feats, labels)

    train = user_rows(m)
    test = user_rows(m_test)
    item = _build_rows([[(0, j, 1.0)] for j in range(n)], None)
    return Dataset("tiny", train, item, test, k=4,
                   params=dict(k=4, t=20, l=1e-5, w=0.1, r=-1.0))


def _positives(rng, m, n, mean, alpha=1.2):
    """Per-row positive lists: max(1, floor(Exp(mean))) draws, each uniform
    w.p. 1/2 else Lomax(alpha) (= Pareto - 1) clipped to n-1; dedup + sort."""
    draws = np.maximum(1, np.floor(rng.exponential(mean, size=m))).astype(np.int64)
    tot = int(draws.sum())
    uni = rng.integers(0, n, size=tot)
    par = np.minimum(np.floor(rng.pareto(alpha, size=tot)), n - 1).astype(np.int64)
    pick = rng.random(tot) < 0.5
    items = np.where(pick, uni, par)
    row = np.repeat(np.arange(m, dtype=np.int64), draws)
    key = np.unique(row * n + items)  # dedup + sort by (row, item)
    r = key // n
    c = key % n
    ptr = np.zeros(m + 1, dtype=np.int64)
    np.cumsum(np.bincount(r, minlength=m), out=ptr[1:])
    return ptr, c


def kkbox(seed: int = 7, m: int = 30755, n: int = 100000, mean: float = 120.0,
          test_frac: float = 0.1, name: str = "kkbox") -> Dataset:
    """Config 3 (headline): user fields listener-id (D=m, 1 nnz)
    and context (D=120, 2 nnz); item fields song-id (D=n), artist (D=n/20),
    genre (D=50), one nnz each; values 1; k=32, -l 4 -w 2^-7 -r -1."""
    rng = np.random.default_rng(seed)
    ptr, col = _positives(rng, m, n, mean)
    ctx = np.sort(np.stack([rng.choice(120, size=2, replace=False) for _ in range(m)]), axis=1) \
        if m <= 4096 else _two_distinct(rng, m, 120)
    uid = np.arange(m, dtype=np.uint64)[:, None]
    train = _fast_rows(m, [(0, uid, np.ones((m, 1))), (1, ctx.astype(np.uint64), np.ones((m, 2)))],
                       ptr, col)
    n_art = max(1, n // 20)
    art = rng.integers(0, n_art, size=n).astype(np.uint64)[:, None]
    gen = rng.integers(0, 50, size=n).astype(np.uint64)[:, None]
    sid = np.arange(n, dtype=np.uint64)[:, None]
    item = _fast_rows(n, [(0, sid, np.ones((n, 1))), (1, art, np.ones((n, 1))),
                          (2, gen, np.ones((n, 1)))])
    mt = max(1, int(m * test_frac))
    tptr, tcol = _positives(rng, mt, n, 10.0)
    test = _fast_rows(mt, [(0, uid[:mt], np.ones((mt, 1))),
                           (1, ctx[:mt].astype(np.uint64), np.ones((mt, 2)))], tptr, tcol)
    return Dataset(name, train, item, test, k=32,
                   params=dict(k=32, t=20, l=4.0, w=0.0078125, r=-1.0))


def cfg5(m: int = 2_000_000, n: int = 250_000, fu: int = 39, d_user: int = 250_000, k: int = 64,
         mean_pos: float = 4.0, seed: int = 5, test_rows: int = 0, name: str = "cfg5") -> Dataset:
    """BASELINE configs[4] as restated in SURVEY §8d (one GPU's row shard of
    the 100 M-row run): --ns, fu = 39 user fields of D = 250,000 features
    each (one node per row, value 1), fv = 1 item field (the item id, D = n),
    ~4 positives per row, k = 64.  Feature ids are half uniform, half
    Lomax(1.2)-skewed (a popular head per field, like real CTR fields); the
    positives are drawn like kkbox's (uniform w.p. 1/2, else the Pareto head)."""
    rng = np.random.default_rng(seed)
    ptr, col = _positives(rng, m, n, mean_pos)
    # one generator per (table, field), filled by a thread pool: numpy's
    # bulk draws release the GIL, so the 12.5 M-row shard (BASELINE
    # configs[4] / 8 GPUs: 487 M nodes) is drawn in seconds, not minutes
    seeds = np.random.SeedSequence(seed + 1).spawn(2 * fu)

    def user_rows(count, table, lab_ptr, lab_col):
        xptr = np.arange(count + 1, dtype=np.uint64) * np.uint64(fu)
        fid = np.tile(np.arange(fu, dtype=np.uint32), count)
        ids = np.empty((count, fu), dtype=np.uint64)

        def field(f):
            g = np.random.default_rng(seeds[table * fu + f])
            for c0 in range(0, count, 1 << 22):
                c = min(count - c0, 1 << 22)
                uni = g.integers(0, d_user, size=c)
                par = np.minimum(np.floor(g.pareto(1.2, size=c)), d_user - 1).astype(np.int64)
                # a field-specific permutation keeps the heads of different fields apart
                par = (par * 7919 + f * 104729) % d_user
                ids[c0:c0 + c, f] = np.where(g.random(c) < 0.5, uni, par)

        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(max_workers=max(1, min(16, os.cpu_count() or 1))) as ex:
            list(ex.map(field, range(fu)))
        return Rows(xptr, fid, ids.reshape(-1), np.ones(count * fu, dtype=np.float64),
                    lab_ptr.astype(np.uint64), lab_col.astype(np.uint64))

    train = user_rows(m, 0, ptr, col)
    item = _fast_rows(n, [(0, np.arange(n, dtype=np.uint64)[:, None], np.ones((n, 1)))])
    test = None
    if test_rows:
        tptr, tcol = _positives(rng, test_rows, n, mean_pos)
        test = user_rows(test_rows, 1, tptr, tcol)
    return Dataset(name, train, item, test, k=k,
                   params=dict(k=k, t=20, l=4.0, w=0.0078125, r=-1.0))


def _skewed(rng, size, d, salt=0):
    """Feature ids in [0, d): half uniform, half a Lomax(1.2) head (permuted
    per salt so that the heads of different columns are different ids)."""
    uni = rng.integers(0, d, size=size)
    par = np.minimum(np.floor(rng.pareto(1.2, size=size)), d - 1).astype(np.int64)
    par = (par * 7919 + salt * 104729) % d
    return np.where(rng.random(size) < 0.5, uni, par).astype(np.uint64)


def _multi_field(rng, count, parts, salt):
    """One field made of several id columns (the reference's data-prep puts
    e.g. QueryID and Depth into one field, kdd12.tools/user_ffm.py:5-7): each
    column c has its own block of the field's index space [off_c, off_c + d_c)."""
    cols, off = [], 0
    for c, d in enumerate(parts):
        cols.append(_skewed(rng, count, d, salt * 16 + c) + np.uint64(off))
        off += d
    return np.stack(cols, axis=1), off


def kdd12(m: int = 500_000, n: int = 50_000, mean_pos: float = 3.0, seed: int = 12, test_rows: int = 0,
          name: str = "kdd12") -> Dataset:
    """BASELINE configs[1] at its SURVEY §8d size, vectorised: m = 500 k users,
    n = 50 k ads, k = 16, ~3 positives per row.  Field structure of the
    reference's data prep: user fields UserID (an id, one node) and
    {QueryID, Depth} (two nodes; kdd12.tools/user_ffm.py:5-7); ad fields
    TitleID, DescriptionID, KeywordID (one node each) and {AdID, DisplayURL,
    AdvertiserID} (three nodes; kdd12.tools/ad_ffm.py:5-9).  The reference's
    loss is squared (it has no log-loss), so this is its ffm-ffm
    mode on that shape."""
    rng = np.random.default_rng(seed)
    ptr, col = _positives(rng, m, n, mean_pos)
    uid = np.arange(m, dtype=np.uint64)[:, None]
    q, _ = _multi_field(rng, m, [max(2, m // 5), 3], 1)
    train = _fast_rows(m, [(0, uid, np.ones((m, 1))), (1, q, np.ones((m, 2)))], ptr, col)
    t0 = _skewed(rng, n, max(2, n // 2), 2)[:, None]
    t1 = _skewed(rng, n, max(2, n // 2), 3)[:, None]
    t2 = _skewed(rng, n, max(2, n // 5), 4)[:, None]
    ad = np.arange(n, dtype=np.uint64)[:, None]
    rest, _ = _multi_field(rng, n, [max(2, n // 10), max(2, n // 50)], 5)
    t3 = np.concatenate([ad, rest + np.uint64(n)], axis=1)
    item = _fast_rows(n, [(0, t0, np.ones((n, 1))), (1, t1, np.ones((n, 1))), (2, t2, np.ones((n, 1))),
                          (3, t3, np.ones((n, 3)))])
    test = None
    if test_rows:
        tptr, tcol = _positives(rng, test_rows, n, mean_pos)
        tq, _ = _multi_field(rng, test_rows, [max(2, m // 5), 3], 1)
        test = _fast_rows(test_rows, [(0, uid[:test_rows], np.ones((test_rows, 1))),
                                      (1, tq, np.ones((test_rows, 2)))], tptr, tcol)
    return Dataset(name, train, item, test, k=16, params=dict(k=16, t=20, l=4.0, w=0.00048828125, r=-1.0))


def outbrain(m: int = 250_000, n: int = 10_000, mean_pos: float = 1.0, seed: int = 13, test_rows: int = 0,
             name: str = "outbrain") -> Dataset:
    """BASELINE configs[3] per GPU (2 M display rows over 8 GPUs
    = 250 k rows per GPU), vectorised: n = 10 k ads, k = 64, ~1 positive
    per row (one click per display, outbrain.tools/add_label.py).  Context
    fields {platform, geo_location} and {source_id, publisher_id,
    document_id} (outbrain.tools/context_ffm.py:6-7); ad fields {source_id,
    publisher_id, document_id} and {campaign_id, advertiser_id}
    (outbrain.tools/item_ffm.py:6-7)."""
    rng = np.random.default_rng(seed)
    ptr, col = _positives(rng, m, n, mean_pos)
    c0, _ = _multi_field(rng, m, [3, 2000], 1)
    c1, _ = _multi_field(rng, m, [5000, 1000, 100_000], 2)
    train = _fast_rows(m, [(0, c0, np.ones((m, 2))), (1, c1, np.ones((m, 3)))], ptr, col)
    i0, _ = _multi_field(rng, n, [5000, 1000, 100_000], 3)
    i1, _ = _multi_field(rng, n, [max(2, n // 3), max(2, n // 10)], 4)
    item = _fast_rows(n, [(0, i0, np.ones((n, 3))), (1, i1, np.ones((n, 2)))])
    test = None
    if test_rows:
        tptr, tcol = _positives(rng, test_rows, n, mean_pos)
        t0, _ = _multi_field(rng, test_rows, [3, 2000], 1)
        t1, _ = _multi_field(rng, test_rows, [5000, 1000, 100_000], 2)
        test = _fast_rows(test_rows, [(0, t0, np.ones((test_rows, 2))), (1, t1, np.ones((test_rows, 3)))],
                          tptr, tcol)
    return Dataset(name, train, item, test, k=64, params=dict(k=64, t=20, l=4.0, w=0.0009765625, r=-1.0))


def kkbox_small(seed: int = 11) -> Dataset:
    """A kkbox-shaped input small enough for the fp64 oracle in a few seconds."""
    return kkbox(seed=seed, m=2000, n=3000, mean=30.0, name="kkbox_small")


def kkbox_s(seed: int = 7) -> Dataset:
    """kkbox-shape-S: m=30,000, n=20,000, mean 30."""
    return kkbox(seed=seed, m=30000, n=20000, mean=30.0, name="kkbox_s")


def _two_distinct(rng, m, d):
    a = rng.integers(0, d, size=m)
    b = rng.integers(0, d - 1, size=m)
    b = np.where(b >= a, b + 1, b)
    return np.stack([np.minimum(a, b), np.maximum(a, b)], axis=1)


def general(seed: int, m: int, n: int, fu: int, fv: int, k: int, d_user=None, d_item=None,
            nnz_user=1, mean_pos=4.0, test_rows=0, vals="ones", name="general") -> Dataset:
    """Generic multi-field generator used by the parity tests for ragged and
    edge-case shapes (several nnz per field, empty rows, real-valued x)."""
    rng = np.random.default_rng(seed)
    d_user = d_user or [max(2, m // (3 + f)) for f in range(fu)]
    d_item = d_item or [max(2, n // (2 + f)) for f in range(fv)]

    def rows(count, nfields, dims, with_labels, mean):
        feats, labels = [], []
        for _ in range(count):
            row = []
            for f in range(nfields):
                c = int(rng.integers(0, nnz_user + 1)) if nnz_user > 1 else 1
                for _ in range(c):
                    v = 1.0 if vals == "ones" else float(np.round(rng.random() * 2, 3) or 0.5)
                    row.append((f, int(rng.integers(0, dims[f])), v))
            feats.append(row)
            if with_labels:
                c = max(1, int(rng.poisson(mean)))
                labels.append(np.sort(rng.choice(n, size=min(c, n), replace=False)))
        return _build_rows(feats, labels if with_labels else None)

    train = rows(m, fu, d_user, True, mean_pos)
    item = rows(n, fv, d_item, False, 0)
    test = rows(test_rows, fu, d_user, True, mean_pos) if test_rows else None
    return Dataset(name, train, item, test, k=k, params=dict(k=k, t=3, l=0.5, w=0.05, r=-1.0))
