"""SGD / AdaGrad mode with on-device negative sampling (include/ocffm.h, SGD
mode; BASELINE.json north_star extras).

The reference has no counterpart (its solver is the block Newton-CG of
ffm.cpp), so these results are "parity unpinned" against the reference.  The
GPU kernel is pinned against oracle/sgd_oracle.cpp, an independent serial CPU
statement of the same algorithm: the one-wave (serial) mode must reproduce
it epoch after epoch within an fp32 tolerance (the sums run in another
order), the alias table must be identical, phi must equal a numpy evaluation,
and the HOGWILD mode must train (loss falls, close to the serial run).
"""
import ctypes as C
import os

import numpy as np
import pytest

import synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_lib = None


def sgo():
    global _lib
    if _lib is None:
        _lib = C.CDLL(os.path.join(REPO, "oracle", "libsgd_oracle.so"))
        _lib.sgo_alias.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        _lib.sgo_alias.restype = None
        _lib.sgo_epoch.restype = C.c_double
        _lib.sgo_epoch.argtypes = ([C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p]
                                   + [C.c_void_p] * 8 + [C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_float,
                                                         C.c_float, C.c_int, C.c_int, C.c_uint64, C.c_uint64,
                                                         C.c_uint64, C.c_uint64])
    return _lib


def P(a):
    return a.ctypes.data_as(C.c_void_p)


def dims(rows, nf):
    D = np.zeros(nf, dtype=np.uint64)
    for f in range(nf):
        sel = rows.fid == f
        if sel.any():
            D[f] = int(rows.idx[sel].max()) + 1
    return D


def nodes(rows, fbase, off):
    """Row node lists, field-major within a row, file order within a field."""
    ptr = [0]
    nd, fd, vl = [], [], []
    nf = int(rows.fid.max()) + 1 if rows.fid.size else 0
    for i in range(rows.m):
        b, e = int(rows.xptr[i]), int(rows.xptr[i + 1])
        for f in range(nf):
            for t in range(b, e):
                if rows.fid[t] == f:
                    nd.append(int(off[fbase + f] + rows.idx[t]))
                    fd.append(fbase + f)
                    vl.append(rows.val[t])
        ptr.append(len(nd))
    return (np.array(ptr, np.uint64), np.array(nd or [0], np.uint32), np.array(fd or [0], np.uint32),
            np.array(vl or [0], np.float32))


class OracleSgd:
    def __init__(self, ds, F, kp, prm):
        tr, it = ds.train, ds.item
        fu = int(tr.fid.max()) + 1
        fv = int(it.fid.max()) + 1
        D = np.concatenate([dims(tr, fu), dims(it, fv)])
        off = np.concatenate([[0], np.cumsum(D)]).astype(np.uint64)
        self.u = nodes(tr, 0, off)
        self.v = nodes(it, fu, off)
        self.pu = np.repeat(np.arange(tr.m, dtype=np.uint32), np.diff(tr.yptr).astype(np.int64))
        self.pv = tr.ycol.astype(np.uint32)
        self.n_items = it.m
        cnt = np.bincount(tr.ycol.astype(np.int64), minlength=it.m).astype(np.float64)
        self.w = np.where(cnt > 0, cnt ** prm["neg_power"], 0.0)
        self.prob = np.ones(it.m, np.float32)
        self.alias = np.zeros(it.m, np.uint32)
        sgo().sgo_alias(it.m, P(self.w), P(self.prob), P(self.alias))
        self.F, self.kp, self.prm = F, kp, prm

    def epoch(self, W, G, epoch, A, B):
        p = self.prm
        return sgo().sgo_epoch(self.pu.size, P(self.pu), P(self.pv), p["nneg"], self.n_items, P(self.prob),
                               P(self.alias), *[P(x) for x in self.u], *[P(x) for x in self.v], self.F, self.kp,
                               P(W), P(G), p["eta"], p["lambda"], p["adagrad"], p["norm"], p["seed"], epoch, A, B)


def test_oracle_alias_table_is_exact():
    """Vose's table: slot i keeps prob[i], hands 1 - prob[i] to alias[i];
    the implied probabilities equal the weights (no GPU)."""
    rng = np.random.default_rng(2)
    for w in (rng.random(500) ** 3, np.r_[np.zeros(10), rng.integers(1, 50, 300).astype(float)], np.ones(7)):
        n = w.size
        prob = np.ones(n, np.float32)
        alias = np.zeros(n, np.uint32)
        sgo().sgo_alias(n, P(np.ascontiguousarray(w)), P(prob), P(alias))
        implied = prob.astype(np.float64).copy()
        np.add.at(implied, alias.astype(np.int64), 1.0 - prob.astype(np.float64))
        np.testing.assert_allclose(implied / n, w / w.sum(), atol=1e-6)


def _trainer(ds, **kw):
    import ocffm
    U = ocffm.ImpData.from_rows(ds.train)
    V = ocffm.ImpData.from_rows(ds.item)
    return ocffm.SgdTrainer(U, V, **kw)


PRM = {"eta": 0.2, "lambda": 2e-5, "nneg": 1, "neg_power": 0.75, "adagrad": 1, "norm": 1, "seed": 5}


@pytest.mark.gpu
@pytest.mark.parametrize("k,adagrad,nneg", [(4, 1, 1), (32, 1, 2), (16, 0, 1), (64, 1, 1), (100, 1, 0), (1, 1, 3)])
def test_serial_mode_matches_oracle(k, adagrad, nneg):
    ds = synth.tiny(seed=3, m=300, n=40)
    prm = dict(PRM, adagrad=adagrad, nneg=nneg)
    t = _trainer(ds, k=k, serial=1, **prm)
    info = t.info
    o = OracleSgd(ds, info["n_fields"], info["kp"], prm)
    np.testing.assert_array_equal(t.get("p"), o.prob)
    np.testing.assert_array_equal(t.get("a"), o.alias)
    W = t.get("W").copy()
    G = t.get("G").copy()
    assert np.all(G == 1.0)
    for e in range(2):
        lg = t.epoch()
        A, B, T = (int(x) for x in t.get("o"))
        assert T == info["instances"] == o.pu.size * (1 + nneg)
        lo = o.epoch(W, G, e, A, B) / T
        Wg = t.get("W")
        scale = np.abs(W).max()
        assert np.abs(Wg - W).max() <= 2e-4 * scale, (e, np.abs(Wg - W).max(), scale)
        assert abs(lg - lo) <= 1e-4 * abs(lo), (lg, lo)
        if adagrad:
            np.testing.assert_allclose(t.get("G"), G, rtol=1e-3, atol=1e-6)
        W = Wg.copy()  # continue both from the GPU state (no drift accumulation)
        G = t.get("G").copy()


@pytest.mark.gpu
def test_phi_matches_numpy():
    ds = synth.kkbox(seed=4, m=200, n=300, mean=6.0, name="kk_sgd")
    t = _trainer(ds, k=32, **PRM)
    info = t.info
    t.epoch()  # move W off its init
    F, kp = info["n_fields"], info["kp"]
    W = t.get("W").astype(np.float64).reshape(-1, F, kp)
    o = OracleSgd(ds, F, kp, PRM)
    rng = np.random.default_rng(1)
    users = rng.integers(0, ds.train.m, 64).astype(np.uint32)
    items = rng.integers(0, ds.item.m, 64).astype(np.uint32)
    got = t.phi(users, items)
    uptr, unode, ufld, uval = o.u
    vptr, vnode, vfld, vval = o.v
    for q in range(64):
        u, v = users[q], items[q]
        j = np.r_[unode[uptr[u]:uptr[u + 1]], vnode[vptr[v]:vptr[v + 1]]]
        f = np.r_[ufld[uptr[u]:uptr[u + 1]], vfld[vptr[v]:vptr[v + 1]]]
        x = np.r_[uval[uptr[u]:uptr[u + 1]], vval[vptr[v]:vptr[v + 1]]].astype(np.float64)
        phi = sum(W[j[a], f[b]] @ W[j[b], f[a]] * x[a] * x[b] for a in range(j.size) for b in range(a + 1, j.size))
        phi /= (x * x).sum()
        assert abs(got[q] - phi) <= 1e-5 * max(1.0, abs(phi)), (q, got[q], phi)


@pytest.mark.gpu
def test_hogwild_trains_like_serial():
    ds = synth.kkbox_small()
    hog = _trainer(ds, k=32, **dict(PRM, seed=9))
    ser = _trainer(ds, k=32, serial=1, **dict(PRM, seed=9))
    lh = [hog.epoch() for _ in range(3)]
    ls = [ser.epoch() for _ in range(3)]
    assert lh[2] < lh[0] and ls[2] < ls[0], (lh, ls)
    assert abs(lh[2] - ls[2]) <= 0.05 * ls[2], (lh, ls)


@pytest.mark.gpu
def test_rccl_one_rank_average_is_identity():
    """The RCCL averaging path (ncclAllReduce of W and G, scale by 1/N) on a
    one-rank communicator leaves the serial run's state bit-identical."""
    import ocffm
    ds = synth.tiny(seed=3, m=300, n=40)
    a = _trainer(ds, k=16, serial=1, **PRM)
    U = ocffm.ImpData.from_rows(ds.train)
    V = ocffm.ImpData.from_rows(ds.item)
    b = ocffm.SgdTrainer(U, V, rank=0, nranks=1, comm=ocffm.comm_id(), k=16, serial=1, **PRM)
    for _ in range(2):
        assert a.epoch() == b.epoch()
        b.average()
    np.testing.assert_array_equal(a.get("W"), b.get("W"))
    np.testing.assert_array_equal(a.get("G"), b.get("G"))


def _sgd_worker(rank, port, out_dir, world):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ocffm

    def allreduce(arr):
        dist.all_reduce(torch.from_numpy(arr))

    ds = synth.tiny(seed=3, m=300, n=40)
    U = ocffm.ImpData.from_rows(ds.train)
    V = ocffm.ImpData.from_rows(ds.item)
    t = ocffm.SgdTrainer(U, V, rank=rank, nranks=world, allreduce=allreduce, k=16, serial=1, **PRM)
    W0, G0 = t.get("W").copy(), t.get("G").copy()
    loss = t.epoch()
    W1, G1, o = t.get("W").copy(), t.get("G").copy(), t.get("o").copy()
    t.average()
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), W0=W0, G0=G0, W1=W1, G1=G1, o=o, loss=loss,
             Wa=t.get("W"), Ga=t.get("G"), inst=t.info["instances"])
    t.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_shards_match_oracle_and_average():
    """Two ranks on one GPU (host all-reduce hook over gloo): each rank's
    epoch over its contiguous user shard matches the serial oracle on that
    shard's positives, and average() leaves the mean of the two models."""
    import socket
    import tempfile
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ds = synth.tiny(seed=3, m=300, n=40)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_sgd_worker, args=(port, d, world), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"s{r}.npz"))) for r in range(world)]
    m = ds.train.m
    assert sum(int(r["inst"]) for r in res) == int(ds.train.yptr[-1]) * (1 + PRM["nneg"])
    for rank, r in enumerate(res):
        np.testing.assert_array_equal(r["W0"], res[0]["W0"])  # same initial model on every rank
        o = OracleSgd(ds, None, None, PRM)
        u0, u1 = m * rank // world, m * (rank + 1) // world
        keep = (o.pu >= u0) & (o.pu < u1)
        o.pu, o.pv = np.ascontiguousarray(o.pu[keep]), np.ascontiguousarray(o.pv[keep])
        F = int(ds.train.fid.max()) + 1 + int(ds.item.fid.max()) + 1
        o.F, o.kp = F, 16
        W, G = r["W0"].copy(), r["G0"].copy()
        A, B, T = (int(x) for x in r["o"])
        assert T == o.pu.size * (1 + PRM["nneg"])
        lo = o.epoch(W, G, 0, A, B) / T
        assert np.abs(r["W1"] - W).max() <= 2e-4 * np.abs(W).max()
        assert abs(float(r["loss"]) - lo) <= 1e-4 * abs(lo)
        np.testing.assert_allclose(r["G1"], G, rtol=1e-3, atol=1e-6)
    mean_w = (res[0]["W1"] + res[1]["W1"]) * np.float32(0.5)
    mean_g = (res[0]["G1"] + res[1]["G1"]) * np.float32(0.5)
    for r in res:
        np.testing.assert_allclose(r["Wa"], mean_w, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(r["Ga"], mean_g, rtol=1e-6, atol=1e-7)
