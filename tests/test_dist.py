"""Row-sharded data parallelism.

CPU (world_size 2, gloo): the decomposition the library uses — every
gradient / Hessian-vector quantity is a sum over users, item-side aggregates
(oQ, bQ, Grams, n1, sum a, sb) are taken over the local users only, and one
all-reduce of the D x k partial plus lambda*W once gives the exact result —
reproduces the oracle's gd_* / hs_* (ffm.cpp:537-742) for every block and half.

GPU: two ranks on one device, all-reduces through the library's host hook
(gloo), must match a single-rank run (fp64, 1e-9) epoch after epoch.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
import synth

WORLD = 2


def _dense(rows, nfields, dims):
    X = [np.zeros((rows.m, dims[f])) for f in range(nfields)]
    for i in range(rows.m):
        for p in range(int(rows.xptr[i]), int(rows.xptr[i + 1])):
            X[int(rows.fid[p])][i, int(rows.idx[p])] += rows.val[p]
    return X


def _problem():
    ds = synth.general(seed=21, m=40, n=25, fu=2, fv=2, k=4, d_user=[7, 5], d_item=[9, 4], nnz_user=2,
                       mean_pos=3.0, vals="real")
    o = O.Oracle(ds, k=4, omega=0.2, lam=0.3, r=-0.7, with_test=False)
    O.lib().orc_srand(1)
    o.init()
    return ds, o


def _partials(rank, ds, o, world=WORLD):
    """This rank's partial gradients / Hv products for every half."""
    k, w, r, lam = o.k, o.omega, o.r, o.lam
    fu, f, m, n = o.fu, o.f, o.m, o.n
    du = [int(x) for x in O.data_ds(O.data_from_rows(ds.train))]
    dv = [int(x) for x in O.data_ds(O.data_from_rows(ds.item))]
    Xu, Xv = _dense(ds.train, fu, du), _dense(ds.item, o.fv, dv)
    Y = np.zeros((m, n))
    for i in range(m):
        for p in range(int(ds.train.yptr[i]), int(ds.train.yptr[i + 1])):
            Y[i, int(ds.train.ycol[p])] = 1.0
    a, b = o.get("a"), o.get("b")
    u0, u1 = m * rank // world, m * (rank + 1) // world
    sh = slice(u0, u1)
    B = lambda f1, f2: O.block_index(f1, f2, f)  # noqa: E731
    P = {}
    Q = {}
    for f1 in range(f):
        for f2 in range(f1, f):
            b12 = B(f1, f2)
            P[b12] = o.get("P", b12).reshape(-1, k)
            Q[b12] = o.get("Q", b12).reshape(-1, k)
    cross = [B(f1, f2) for f1 in range(fu) for f2 in range(fu, f)]
    yt = a[:, None] + b[None, :] + sum(P[c] @ Q[c].T for c in cross) - 1
    coef = Y * ((1 - w) * yt - w * (1 - r))
    sa = sum(P[c] @ Q[c].sum(0) for c in cross)
    sb_loc = sum(Q[c] @ P[c][sh].sum(0) for c in cross)
    rng = np.random.default_rng(7)
    out = {}
    for f1 in range(f):
        for f2 in range(f1, f):
            b12 = B(f1, f2)
            for half in (0, 1):
                fl = f1 if half == 0 else f2
                user = fl < fu
                X = Xu[fl] if user else Xv[fl - fu]
                D = X.shape[1]
                Q1 = Q[b12] if half == 0 else P[b12]
                v = rng.standard_normal((D, k))
                if (f1 < fu) != (f2 < fu):  # cross
                    if user:
                        Xs = X[sh]
                        oQ, bQ = Q1.sum(0), b @ Q1
                        T = sum(P[c][sh] @ (Q[c].T @ Q1) for c in cross)
                        g = coef[sh] @ Q1 + w * (T + (a[sh] - r)[:, None] * oQ + bQ)
                        QTQ = Q1.T @ Q1
                        phi = Xs @ v
                        hv = (1 - w) * (((phi @ Q1.T) * Y[sh]) @ Q1) + w * phi @ QTQ
                    else:
                        Xs = X
                        P1 = Q1[sh]
                        oQ, bQ = P1.sum(0), a[sh] @ P1
                        T = sum(Q[c] @ (P[c][sh].T @ P1) for c in cross)
                        g = coef[sh].T @ P1 + w * (T + (b - r)[:, None] * oQ + bQ)
                        QTQ = P1.T @ P1
                        phi = Xs @ v
                        hv = (1 - w) * (((phi @ P1.T) * Y[sh].T) @ P1) + w * phi @ QTQ
                else:  # side
                    if user:
                        Xs, q = X[sh], Q1[sh]
                        z = w * (n * (a[sh] - r) + b.sum() + sa[sh]) + coef[sh].sum(1)
                        d = (1 - w) * Y[sh].sum(1) + w * n
                    else:
                        Xs, q = X, Q1
                        z = w * ((u1 - u0) * (b - r) + a[sh].sum() + sb_loc) + coef[sh].sum(0)
                        d = (1 - w) * Y[sh].sum(0) + w * (u1 - u0)
                    g = z[:, None] * q
                    phi = Xs @ v
                    hv = (d * (phi * q).sum(1))[:, None] * q
                out[(b12, half)] = (Xs.T @ g, Xs.T @ hv, v)
    return out


def _worker(rank, port, result_path, world=WORLD):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ds, o = _problem()
    parts = _partials(rank, ds, o, world)
    worst = 0.0
    for (b12, half), (g, hv, v) in sorted(parts.items()):
        tg = torch.from_numpy(np.ascontiguousarray(g))
        th = torch.from_numpy(np.ascontiguousarray(hv))
        dist.all_reduce(tg)
        dist.all_reduce(th)
        f1, f2 = [(a, b) for a in range(o.f) for b in range(a, o.f) if O.block_index(a, b, o.f) == b12][0]
        W = o.get("W" if half == 0 else "H", b12).reshape(-1, o.k)
        G = tg.numpy() + o.lam * W
        Hv = th.numpy() + o.lam * v
        G_ref = o.grad(f1, f2, half).reshape(-1, o.k)
        H_ref = o.hv(f1, f2, half, v.ravel()).reshape(-1, o.k)
        worst = max(worst, np.abs(G - G_ref).max() / np.abs(G_ref).max(),
                    np.abs(Hv - H_ref).max() / np.abs(H_ref).max())
    if rank == 0:
        np.save(result_path, np.array([worst]))
    dist.destroy_process_group()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_decomposition_gloo(world):
    # world 3: uneven user shards (40 rows: 13 / 13 / 14)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "worst.npy")
        mp.spawn(_worker, args=(_free_port(), path, world), nprocs=world, join=True)
        worst = float(np.load(path)[0])
    assert worst < 1e-10, worst


# ------------------------------------------------------------------ GPU ---
def _dist_dataset(name):
    if name == "tiny":
        return synth.tiny(seed=8)
    if name == "lowcard":
        # one-node low-cardinality fields on both sides (user field 1: D = 6,
        # item field 1: D = 5): with OCFFM_CGRAM=2 their side halves run on
        # per-column Grams, partial per rank (k_hv_cgram MODE 2 + k_fin) on the
        # user side and replicated (the item side halves' CG in full on every
        # rank); their cross halves take the column-tau term before the all-reduce
        return synth.general(seed=23, m=300, n=200, fu=2, fv=2, k=8, d_user=[300, 6], d_item=[200, 5],
                             nnz_user=1, mean_pos=5.0, test_rows=30, name="lowcard")
    if name == "one_item":
        # a single item: with two ranks the second owns no item at all
        # (item-owned CG steps forced by OCFFM_ITEM_OWNED=2)
        return synth.kkbox(seed=6, m=200, n=1, mean=1.0, name="one_item")
    if name == "uneven":
        # 301 users and 37 items: on 3 / 4 ranks the user shards are uneven
        # (100/100/101, 75/75/75/76) and so are the owned item chunks
        # (ceil(37/N): 13/13/11, 10/10/10/7: the all-gather slots r >= 2 hold
        # short chunks); the listener-id field is owned
        return synth.kkbox(seed=9, m=301, n=37, mean=8.0, name="uneven")
    if name == "outbrain":
        # BASELINE configs[3]'s data-parallel workload at test size (SURVEY
        # §8d): fu = 2, fv = 2, k = 64, ~1 positive per row
        return synth.general(seed=32, m=400, n=60, fu=2, fv=2, k=64, mean_pos=1.0, test_rows=40, name="outbrain")
    # a listener-id field (D = m): every feature belongs to one rank's rows,
    # so its CG vectors stay sharded and only dot products are summed
    return synth.kkbox(seed=5, m=300, n=400, mean=12.0, name="kkbox_dist")


# Several ranks share the one GPU in these tests, so the persistent CG
# kernel's grid (k_cg_cgram, on the replicated halves) can find CUs held by
# other ranks' kernels: it then gives up on its barrier and the solve is
# finished per step (solver.hip cgp_recover), which these runs exercise.


def _gpu_worker(rank, port, out_dir, world, name="tiny"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ocffm

    def allreduce(arr):
        t = torch.from_numpy(arr)
        dist.all_reduce(t)

    ds = _dist_dataset(name)
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, rank=rank, nranks=world, allreduce=allreduce)
    ocffm.srand(1)
    g.init()
    g.set_profiling(True)
    for _ in range(2):
        g.one_epoch()
    ks = g.kernel_stats()
    steps = ks.get("cg_step", {}).get("launches", 0)
    io = ks.get("hs_cross_io", {}).get("launches", 0)
    met = g.validate()
    nb = g.n_blocks()
    W = [g.get("W", b) for b in range(nb)] + [g.get("H", b) for b in range(nb)]
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), cg=g.cg_log(), loss=met["loss"], ndcg=met["ndcg"],
             prec=met["prec"], steps=steps, io=io, *W)
    g.close()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("name,env", [("tiny", {}), ("owned", {}), ("lowcard", {"OCFFM_CGRAM": "2"}),
                                      ("lowcard", {"OCFFM_CGRAM": "2", "OCFFM_FUSE": "0"}), ("outbrain", {}),
                                      ("outbrain", {"OCFFM_EXACT_R2": "1"}), ("owned", {"OCFFM_CCG": "2"}),
                                      ("lowcard", {"OCFFM_CCG": "2", "OCFFM_HOT": "2"}),
                                      ("owned", {"OCFFM_ITEM_OWNED": "0"}),
                                      ("owned", {"OCFFM_ITEM_OWNED": "0", "OCFFM_CCG": "2"}),
                                      ("owned", {"OCFFM_EXACT_R2": "1"}), ("one_item", {"OCFFM_ITEM_OWNED": "2"})])
def test_two_ranks_match_one_rank_on_gpu(name, env, monkeypatch):
    import ocffm
    for k, v in env.items():  # inherited by the spawned ranks
        monkeypatch.setenv(k, v)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gpu_worker, args=(_free_port(), d, WORLD, name), nprocs=WORLD, join=True)
        r0 = np.load(os.path.join(d, "r0.npz"))
        r1 = np.load(os.path.join(d, "r1.npz"))
        ds = _dist_dataset(name)
        g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
        ocffm.srand(1)
        g.init()
        for _ in range(2):
            g.one_epoch()
        met = g.validate()
        nb = g.n_blocks()
        # the owned-field path ran on the listener-id halves, and the song-id
        # item halves' CG steps ran item-owned (the default on several ranks)
        # unless OCFFM_ITEM_OWNED=0
        if name == "owned":
            assert int(r0["steps"]) > 0
            io_on = env.get("OCFFM_ITEM_OWNED", "1") != "0"
            assert (int(r0["io"]) > 0) == io_on and (int(r1["io"]) > 0) == io_on
        if name == "one_item":  # rank 1 owns no item: it only joins the collectives
            assert int(r0["io"]) > 0 and int(r1["io"]) == 0
        np.testing.assert_array_equal(r0["cg"], g.cg_log())
        np.testing.assert_array_equal(r1["cg"], g.cg_log())
        for idx, (what, b) in enumerate([("W", b) for b in range(nb)] + [("H", b) for b in range(nb)]):
            ref = g.get(what, b)
            for r in (r0, r1):
                x = r[f"arr_{idx}"]
                assert np.abs(x - ref).max() <= 1e-9 * np.abs(ref).max(), (what, b)
        assert abs(float(r0["loss"]) - met["loss"]) <= 1e-9 * met["loss"]
        np.testing.assert_allclose(r0["ndcg"], met["ndcg"], atol=1e-12)
        np.testing.assert_allclose(r0["prec"], met["prec"], atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("world,name,env", [(3, "uneven", {}), (4, "uneven", {}), (4, "uneven", {"OCFFM_CCG": "2"}),
                                            (3, "uneven", {"OCFFM_ITEM_OWNED": "0"}),
                                            (3, "one_item", {"OCFFM_ITEM_OWNED": "2"}), (4, "outbrain", {})])
def test_n_ranks_match_one_rank_on_gpu(world, name, env, monkeypatch):
    """3 and 4 ranks on one device (all-reduces through the host hook):
    uneven user shards, owned listener-id fields, item-owned CG steps whose
    all-gather slots r >= 2 hold short chunks, ranks that own no item
    (one_item: ranks 1.. own nothing).  fp64 within 1e-9 of one rank,
    identical CG counts, every rank's tables."""
    import ocffm
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gpu_worker, args=(_free_port(), d, world, name), nprocs=world, join=True)
        rs = [np.load(os.path.join(d, f"r{q}.npz")) for q in range(world)]
        ds = _dist_dataset(name)
        g = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
        ocffm.srand(1)
        g.init()
        for _ in range(2):
            g.one_epoch()
        met = g.validate()
        nb = g.n_blocks()
        if name == "uneven":
            io_on = env.get("OCFFM_ITEM_OWNED", "1") != "0"
            assert all((int(r["io"]) > 0) == io_on for r in rs)
            assert all(int(r["steps"]) > 0 for r in rs)  # owned listener-id halves
        if name == "one_item":
            assert int(rs[0]["io"]) > 0 and all(int(r["io"]) == 0 for r in rs[1:])
        for r in rs:
            np.testing.assert_array_equal(r["cg"], g.cg_log())
        for idx, (what, b) in enumerate([("W", b) for b in range(nb)] + [("H", b) for b in range(nb)]):
            ref = g.get(what, b)
            for r in rs:
                assert np.abs(r[f"arr_{idx}"] - ref).max() <= 1e-9 * np.abs(ref).max(), (what, b)
        assert abs(float(rs[0]["loss"]) - met["loss"]) <= 1e-9 * met["loss"]
        np.testing.assert_allclose(rs[0]["ndcg"], met["ndcg"], atol=1e-12)


@pytest.mark.gpu
def test_rccl_one_rank_item_owned():
    """The item-owned CG steps through RCCL (ncclAllGather in place, the dot
    products by ncclAllReduce) on a one-rank communicator (OCFFM_ITEM_OWNED=2
    takes the path without a second rank): fp64 within 1e-9 of the plain run,
    identical CG counts."""
    import ocffm
    ds = _dist_dataset("owned")
    a = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
    os.environ["OCFFM_ITEM_OWNED"] = "2"
    try:
        b = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, rank=0, nranks=1, comm=ocffm.comm_id())
    finally:
        os.environ.pop("OCFFM_ITEM_OWNED", None)
    b.set_profiling(True)
    for g in (a, b):
        ocffm.srand(1)
        g.init()
        for _ in range(2):
            g.one_epoch()
    assert b.kernel_stats().get("hs_cross_io", {}).get("launches", 0) > 0
    np.testing.assert_array_equal(a.cg_log(), b.cg_log())
    for bl in range(a.n_blocks()):
        for what in "WH":
            ref = a.get(what, bl)
            assert np.abs(b.get(what, bl) - ref).max() <= 1e-9 * np.abs(ref).max(), (what, bl)


@pytest.mark.gpu
def test_rccl_one_rank_matches_single():
    """The RCCL code path (scatter pass, ncclAllReduce, k_fin) on a one-rank
    communicator must reproduce the single-GPU fused path (fp64, 1e-9)."""
    import ocffm
    ds = synth.tiny(seed=8)
    a = ocffm.problem_from_dataset(ds, precision=ocffm.FP64)
    b = ocffm.problem_from_dataset(ds, precision=ocffm.FP64, rank=0, nranks=1, comm=ocffm.comm_id())
    for g in (a, b):
        ocffm.srand(1)
        g.init()
        for _ in range(2):
            g.one_epoch()
    np.testing.assert_array_equal(a.cg_log(), b.cg_log())
    for bl in range(6):
        for what in "WH":
            ref = a.get(what, bl)
            assert np.abs(b.get(what, bl) - ref).max() <= 1e-9 * np.abs(ref).max(), (what, bl)
    ma, mb = a.validate(), b.validate()
    assert abs(ma["loss"] - mb["loss"]) <= 1e-9 * ma["loss"]


def _fp32_worker(rank, port, out_dir, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ocffm

    def allreduce(arr):
        dist.all_reduce(torch.from_numpy(arr))

    ds = synth.kkbox_small()
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, rank=rank, nranks=world, allreduce=allreduce)
    ocffm.srand(1)
    g.init()
    g.set_profiling(True)
    for _ in range(4):
        g.one_epoch()
    ks = g.kernel_stats()
    met = g.validate()
    nb = g.n_blocks()
    W = [g.get("W", b) for b in range(nb)] + [g.get("H", b) for b in range(nb)]
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), cg=g.cg_log(), loss=met["loss"], ndcg=met["ndcg"],
             ccg=ks.get("hv_cgram", {}).get("launches", 0), *W)
    g.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_fp32_default_path():
    """The multi-rank line the scale bench runs (fp32, default knobs) on a
    kkbox-shaped set: the artist / genre item halves go on per-column cross
    Grams on both ranks (eligibility from the whole data, ccg_field_all), the
    ranks' replicated tables stay bit-identical, and the run tracks a
    one-rank run (the all-reduce reorders fp32 sums, so within 1e-3)."""
    import ocffm
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fp32_worker, args=(_free_port(), d, WORLD), nprocs=WORLD, join=True)
        r0 = np.load(os.path.join(d, "r0.npz"))
        r1 = np.load(os.path.join(d, "r1.npz"))
    assert int(r0["ccg"]) > 0 and int(r1["ccg"]) > 0
    np.testing.assert_array_equal(r0["cg"], r1["cg"])
    nw = len([k for k in r0.files if k.startswith("arr_")])
    for i in range(nw):
        np.testing.assert_array_equal(r0[f"arr_{i}"], r1[f"arr_{i}"])
    ds = synth.kkbox_small()
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32)
    ocffm.srand(1)
    g.init()
    for _ in range(4):
        g.one_epoch()
    met = g.validate()
    g.close()
    assert abs(float(r0["loss"]) - met["loss"]) <= 1e-3 * met["loss"]
    np.testing.assert_allclose(r0["ndcg"], met["ndcg"], atol=0.02)
