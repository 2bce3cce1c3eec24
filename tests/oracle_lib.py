"""ctypes binding of the CPU oracle (oracle/liboracle.so) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_data_from_rows.restype = C.c_void_p
        L.orc_data_from_rows.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.orc_data_read.restype = C.c_void_p
        L.orc_data_read.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_uint64]
        L.orc_data_m.restype = C.c_uint64
        L.orc_data_m.argtypes = [C.c_void_p]
        L.orc_data_f.restype = C.c_uint64
        L.orc_data_f.argtypes = [C.c_void_p]
        L.orc_data_ds.argtypes = [C.c_void_p, _u64p]
        L.orc_problem_new.restype = C.c_void_p
        L.orc_problem_new.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_double, C.c_double, C.c_double,
                                      C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int]
        for name in ("orc_problem_free", "orc_init", "orc_one_epoch", "orc_cache_sasb", "orc_refresh"):
            getattr(L, name).argtypes = [C.c_void_p]
        L.orc_srand.argtypes = [C.c_uint32]
        L.orc_solve_block.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_func.restype = C.c_double
        L.orc_func.argtypes = [C.c_void_p]
        L.orc_set_threads.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_set_dot_order.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_validate.argtypes = [C.c_void_p, C.c_int, _f64p, C.c_void_p, C.c_uint64]
        L.orc_validate.restype = C.c_uint64
        L.orc_cg_log.restype = C.c_int
        L.orc_cg_log.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.orc_cg_log_clear.argtypes = [C.c_void_p]
        L.orc_get.restype = C.c_uint64
        L.orc_get.argtypes = [C.c_void_p, C.c_char, C.c_uint32, C.c_void_p, C.c_uint64]
        L.orc_set.argtypes = [C.c_void_p, C.c_char, C.c_uint32, _f64p, C.c_uint64]
        L.orc_grad.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, _f64p]
        L.orc_hv.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, _f64p, _f64p]
        L.orc_save_model.argtypes = [C.c_void_p, C.c_char_p]
        L.orc_save_binary.argtypes = [C.c_void_p, C.c_char_p]
        L.orc_times.argtypes = [C.c_void_p, C.c_int]
        L.orc_time_epochs.restype = C.c_double
        L.orc_time_epochs.argtypes = [C.c_void_p, C.c_uint32]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def data_from_rows(rows, ds=None):
    L = lib()
    keep = [rows.xptr, rows.fid, rows.idx, rows.val, rows.yptr, rows.ycol, ds]
    h = L.orc_data_from_rows(rows.m, _ptr(rows.xptr), _ptr(rows.fid), _ptr(rows.idx), _ptr(rows.val),
                             _ptr(rows.yptr), _ptr(rows.ycol), _ptr(ds), 0 if ds is None else len(ds))
    del keep
    return h


def data_read(path, has_label, ds=None):
    L = lib()
    h = L.orc_data_read(path.encode(), int(has_label), _ptr(ds), 0 if ds is None else len(ds))
    if not h:
        raise RuntimeError("oracle read failed: " + path)
    return h


def data_ds(h):
    L = lib()
    f = L.orc_data_f(h)
    out = np.zeros(f, dtype=np.uint64)
    L.orc_data_ds(h, out)
    return out


def block_index(f1, f2, f):
    return f2 + (f - 1) * f1 - f1 * (f1 - 1) // 2


class Oracle:
    """The restated reference problem (ImpProblem, ffm.h:82-151)."""

    def __init__(self, ds, k=None, omega=None, lam=None, r=None, t=None, threads=1, self_side=True,
                 freq=False, with_test=True, seed=1):
        L = lib()
        p = ds.params
        self.k = k if k is not None else p["k"]
        self.omega = omega if omega is not None else p["w"]
        self.lam = lam if lam is not None else p["l"]
        self.r = r if r is not None else p["r"]
        self.t = t if t is not None else p["t"]
        self.self_side = self_side
        U = data_from_rows(ds.train)
        V = data_from_rows(ds.item)
        Ut = None
        if with_test and ds.test is not None:
            Ut = data_from_rows(ds.test, ds=data_ds(U))
        self.fu = int(L.orc_data_f(U))
        self.fv = int(L.orc_data_f(V))
        self.f = self.fu + self.fv
        self.m = int(L.orc_data_m(U))
        self.n = int(L.orc_data_m(V))
        self.h = L.orc_problem_new(U, Ut, V, self.omega, self.lam, self.r, self.t, self.k, threads,
                                   int(self_side), int(freq))
        L.orc_srand(seed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_problem_free(self.h)
            self.h = None

    def init(self):
        lib().orc_init(self.h)

    def one_epoch(self):
        lib().orc_one_epoch(self.h)

    def refresh(self):
        lib().orc_refresh(self.h)

    def solve_block(self, f1, f2):
        lib().orc_solve_block(self.h, f1, f2)

    def func(self):
        return lib().orc_func(self.h)

    def get(self, what, b12=0):
        L = lib()
        nn = L.orc_get(self.h, what.encode(), b12, None, 0)
        out = np.zeros(nn, dtype=np.float64)
        L.orc_get(self.h, what.encode(), b12, _ptr(out), nn)
        return out

    def set(self, what, b12, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        lib().orc_set(self.h, what.encode(), b12, arr, arr.size)

    def validate(self, forced=False, per_row=False):
        """per_row: also the nDCG@5,10,20,40,80 of every test row (rows x 5)."""
        out = np.zeros(11, dtype=np.float64)
        need = lib().orc_validate(self.h, int(forced), out, None, 0) if per_row else 0
        rows = np.zeros(max(1, need), dtype=np.float64) if per_row else None
        lib().orc_validate(self.h, int(forced), out, _ptr(rows), need)
        res = dict(loss=out[0], prec=out[1:6].copy(), ndcg=out[6:11].copy())
        if per_row:
            res["ndcg_rows"] = rows[:need].reshape(-1, 5)
        return res

    def cg_log(self):
        buf = np.zeros(1 << 16, dtype=np.int32)
        nn = lib().orc_cg_log(self.h, _ptr(buf), buf.size)
        return buf[:min(nn, buf.size)].copy()

    def cg_log_clear(self):
        lib().orc_cg_log_clear(self.h)

    def grad(self, f1, f2, half):
        b12 = block_index(f1, f2, self.f)
        size = self.get("W" if half == 0 else "H", b12).size
        out = np.zeros(size, dtype=np.float64)
        lib().orc_grad(self.h, f1, f2, half, out)
        return out

    def hv(self, f1, f2, half, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        out = np.zeros_like(v)
        lib().orc_hv(self.h, f1, f2, half, v, out)
        return out

    def save_model(self, path):
        lib().orc_save_model(self.h, path.encode())

    def save_binary(self, path):
        lib().orc_save_binary(self.h, path.encode())

    def set_dot_order(self, lanes, chunks=1):
        """Sum the cblas_ddot restatement (inner(), ffm.cpp:57-60) in the
        order of an optimised BLAS build: `lanes` interleaved accumulators
        over `chunks` contiguous chunks (1, 1: serial, the default)."""
        lib().orc_set_dot_order(self.h, lanes, chunks)

    def time_epochs(self, epochs, threads=None):
        if threads is not None:
            lib().orc_set_threads(self.h, threads)
        return lib().orc_time_epochs(self.h, epochs)
