"""Python mirror of the reference's C++ interface over the C ABI (include/ocffm.h).

Names follow the reference (``ffm.h:42-154``): ``Parameter``, ``ImpData``,
``ImpProblem`` with ``init``, ``one_epoch``, ``solve``, ``validate`` and
``save_model``.  Every call runs the HIP path in ``libocffm.so``; there is no
CPU fallback: if the library or a GPU is missing, calls raise ``OcffmError``.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

try:  # one HIP runtime per process: let torch's libamdhip64 load first if present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the library itself
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OCFFM_LIB") or os.path.join(HERE, "libocffm.so")  # override: experiment builds

OK, E_ARG, E_IO, E_DATA, E_HIP, E_COMM, E_STATE = range(7)
FP64, FP32 = 64, 32
COMM_ID_BYTES = 128


class OcffmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[ocffm error {code}] {msg}")
        self.code = code


class _Param(C.Structure):
    _fields_ = [("omega", C.c_double), ("lambda_", C.c_double), ("r", C.c_double),
                ("nr_pass", C.c_uint32), ("k", C.c_uint32), ("nr_threads", C.c_uint32),
                ("self_side", C.c_int32), ("freq", C.c_int32), ("precision", C.c_int32),
                ("device", C.c_int32)]


class _Info(C.Structure):
    _fields_ = [("m", C.c_uint64), ("n", C.c_uint64), ("f", C.c_uint64), ("nnz_x", C.c_uint64),
                ("nnz_y", C.c_uint64)]


class _Metrics(C.Structure):
    _fields_ = [("loss", C.c_double), ("prec", C.c_double * 5), ("ndcg", C.c_double * 5),
                ("top_k", C.c_uint32 * 5)]


class _KStat(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_uint64), ("total_ms", C.c_double),
                ("alg_bytes", C.c_double), ("alg_flops", C.c_double)]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p)

EXPORTS = [
    "ocffm_param_default", "ocffm_last_error", "ocffm_device_count", "ocffm_data_read",
    "ocffm_data_from_rows", "ocffm_data_trans_y", "ocffm_data_get_info", "ocffm_data_get_ds",
    "ocffm_data_get_labels", "ocffm_data_get_field", "ocffm_data_free", "ocffm_problem_create", "ocffm_comm_id", "ocffm_problem_create_dist",
    "ocffm_problem_create_dist_host", "ocffm_problem_init", "ocffm_problem_one_epoch",
    "ocffm_problem_solve_block", "ocffm_problem_cache_sasb", "ocffm_problem_solve",
    "ocffm_problem_validate", "ocffm_print_header", "ocffm_print_epoch", "ocffm_problem_get",
    "ocffm_problem_set", "ocffm_problem_grad", "ocffm_problem_hv", "ocffm_problem_save_model",
    "ocffm_problem_validate_forced", "ocffm_problem_test_rows", "ocffm_problem_save_binary", "ocffm_problem_load_binary",
    "ocffm_problem_cg_log", "ocffm_problem_set_profiling", "ocffm_problem_set_profile_filter",
    "ocffm_problem_kernel_stats",
    "ocffm_problem_reset_stats", "ocffm_problem_alg_bytes", "ocffm_problem_counter", "ocffm_problem_sync",
    "ocffm_problem_layout_digest", "ocffm_problem_destroy",
    "ocffm_sgd_param_default", "ocffm_sgd_create", "ocffm_sgd_create_dist", "ocffm_sgd_create_dist_host", "ocffm_sgd_epoch",
    "ocffm_sgd_average", "ocffm_sgd_phi", "ocffm_sgd_get", "ocffm_sgd_set_w", "ocffm_sgd_get_info",
    "ocffm_sgd_sync", "ocffm_sgd_destroy",
]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OcffmError(E_STATE, f"{LIB_PATH} not built (run __graft_entry__.build() or make -C one-class-ffm_amd)")
    L = C.CDLL(LIB_PATH)
    vp, u64, u32, i32, dbl = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int, C.c_double
    L.ocffm_last_error.restype = C.c_char_p
    L.ocffm_param_default.argtypes = [C.POINTER(_Param)]
    L.ocffm_device_count.argtypes = [C.POINTER(C.c_int)]
    L.ocffm_data_read.argtypes = [C.c_char_p, i32, vp, u32, C.POINTER(vp)]
    L.ocffm_data_from_rows.argtypes = [u64, vp, vp, vp, vp, vp, vp, vp, u32, C.POINTER(vp)]
    L.ocffm_data_trans_y.argtypes = [vp, vp]
    L.ocffm_data_get_info.argtypes = [vp, C.POINTER(_Info)]
    L.ocffm_data_get_ds.argtypes = [vp, vp]
    L.ocffm_data_get_labels.argtypes = [vp, vp, vp]
    L.ocffm_data_get_field.argtypes = [vp, u32, vp, vp, vp, vp]
    L.ocffm_data_free.argtypes = [vp]
    L.ocffm_data_free.restype = None
    L.ocffm_problem_create.argtypes = [vp, vp, vp, C.POINTER(_Param), C.POINTER(vp)]
    L.ocffm_comm_id.argtypes = [vp]
    L.ocffm_problem_create_dist.argtypes = [vp, vp, vp, C.POINTER(_Param), i32, i32, vp, C.POINTER(vp)]
    L.ocffm_problem_create_dist_host.argtypes = [vp, vp, vp, C.POINTER(_Param), i32, i32, ALLREDUCE_FN, vp,
                                                 C.POINTER(vp)]
    for name in ("ocffm_problem_init", "ocffm_problem_one_epoch", "ocffm_problem_cache_sasb",
                 "ocffm_problem_solve", "ocffm_problem_reset_stats", "ocffm_problem_sync"):
        getattr(L, name).argtypes = [vp]
    L.ocffm_problem_solve_block.argtypes = [vp, u32, u32]
    L.ocffm_problem_validate.argtypes = [vp, C.POINTER(_Metrics)]
    L.ocffm_print_epoch.argtypes = [C.POINTER(_Metrics), u32]
    L.ocffm_problem_get.argtypes = [vp, C.c_char, u32, vp, u64, C.POINTER(u64)]
    L.ocffm_problem_set.argtypes = [vp, C.c_char, u32, vp, u64]
    L.ocffm_problem_grad.argtypes = [vp, u32, u32, i32, vp]
    L.ocffm_problem_hv.argtypes = [vp, u32, u32, i32, vp, vp]
    L.ocffm_problem_save_model.argtypes = [vp, C.c_char_p]
    L.ocffm_problem_validate_forced.argtypes = [vp, C.POINTER(_Metrics), vp, u64]
    L.ocffm_problem_test_rows.argtypes = [vp, C.POINTER(u64)]
    L.ocffm_problem_save_binary.argtypes = [vp, C.c_char_p]
    L.ocffm_problem_load_binary.argtypes = [vp, C.c_char_p]
    L.ocffm_problem_cg_log.argtypes = [vp, vp, i32, C.POINTER(C.c_int)]
    L.ocffm_problem_set_profiling.argtypes = [vp, i32]
    L.ocffm_problem_set_profile_filter.argtypes = [vp, C.c_char_p]
    L.ocffm_problem_kernel_stats.argtypes = [vp, C.POINTER(_KStat), i32, C.POINTER(C.c_int)]
    L.ocffm_problem_alg_bytes.argtypes = [vp, C.POINTER(dbl)]
    L.ocffm_problem_counter.argtypes = [vp, C.c_char_p, C.POINTER(C.c_int64)]
    L.ocffm_problem_layout_digest.argtypes = [vp, vp, vp, i32, C.POINTER(C.c_int)]
    L.ocffm_problem_destroy.argtypes = [vp]
    L.ocffm_problem_destroy.restype = None
    L.ocffm_sgd_param_default.argtypes = [vp]
    L.ocffm_sgd_param_default.restype = None
    L.ocffm_sgd_create.argtypes = [vp, vp, vp, C.POINTER(vp)]
    L.ocffm_sgd_create_dist.argtypes = [vp, vp, vp, i32, i32, vp, C.POINTER(vp)]
    L.ocffm_sgd_create_dist_host.argtypes = [vp, vp, vp, i32, i32, ALLREDUCE_FN, vp, C.POINTER(vp)]
    L.ocffm_sgd_epoch.argtypes = [vp, C.POINTER(dbl)]
    L.ocffm_sgd_average.argtypes = [vp]
    L.ocffm_sgd_phi.argtypes = [vp, u64, vp, vp, vp]
    L.ocffm_sgd_get.argtypes = [vp, C.c_char, vp, u64, C.POINTER(u64)]
    L.ocffm_sgd_set_w.argtypes = [vp, vp, u64]
    L.ocffm_sgd_get_info.argtypes = [vp, vp]
    L.ocffm_sgd_sync.argtypes = [vp]
    L.ocffm_sgd_destroy.argtypes = [vp]
    L.ocffm_sgd_destroy.restype = None
    _lib = L
    return L


def _check(st: int) -> None:
    if st != OK:
        raise OcffmError(st, lib().ocffm_last_error().decode(errors="replace"))


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def device_count() -> int:
    c = C.c_int(0)
    _check(lib().ocffm_device_count(C.byref(c)))
    return c.value


def block_index(f1: int, f2: int, f: int) -> int:
    """index_vec (ffm.cpp:53-55)."""
    return f2 + (f - 1) * f1 - f1 * (f1 - 1) // 2


class Parameter:
    """class Parameter (ffm.h:42-49) with the reference's code defaults."""

    def __init__(self, **kw):
        p = _Param()
        lib().ocffm_param_default(C.byref(p))
        self._p = p
        for key, v in kw.items():
            setattr(self, key, v)

    def __setattr__(self, key, value):
        if key == "_p":
            object.__setattr__(self, key, value)
            return
        if key == "lambda":
            key = "lambda_"
        setattr(self._p, key, value)

    def __getattr__(self, key):
        if key == "lambda":
            key = "lambda_"
        return getattr(object.__getattribute__(self, "_p"), key)


class ImpData:
    """class ImpData (ffm.h:51-79): read + split_fields, transY."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def read(cls, path: str, has_label: bool, ds: Optional[np.ndarray] = None) -> "ImpData":
        h = C.c_void_p()
        dsa = None if ds is None else np.ascontiguousarray(ds, dtype=np.uint64)
        _check(lib().ocffm_data_read(path.encode(), int(has_label), _ptr(dsa), 0 if dsa is None else len(dsa),
                                     C.byref(h)))
        return cls(h)

    @classmethod
    def from_rows(cls, rows, ds: Optional[np.ndarray] = None) -> "ImpData":
        h = C.c_void_p()
        dsa = None if ds is None else np.ascontiguousarray(ds, dtype=np.uint64)
        arrs = [np.ascontiguousarray(rows.xptr, np.uint64), np.ascontiguousarray(rows.fid, np.uint32),
                np.ascontiguousarray(rows.idx, np.uint64), np.ascontiguousarray(rows.val, np.float64)]
        ya = None if rows.yptr is None else np.ascontiguousarray(rows.yptr, np.uint64)
        yc = None if rows.ycol is None else np.ascontiguousarray(rows.ycol, np.uint64)
        _check(lib().ocffm_data_from_rows(rows.m, *[_ptr(a) for a in arrs], _ptr(ya), _ptr(yc), _ptr(dsa),
                                          0 if dsa is None else len(dsa), C.byref(h)))
        return cls(h)

    def trans_y(self, U: "ImpData") -> None:
        _check(lib().ocffm_data_trans_y(self.h, U.h))

    @property
    def info(self) -> dict:
        i = _Info()
        _check(lib().ocffm_data_get_info(self.h, C.byref(i)))
        return dict(m=i.m, n=i.n, f=i.f, nnz_x=i.nnz_x, nnz_y=i.nnz_y)

    @property
    def Ds(self) -> np.ndarray:
        out = np.zeros(max(1, self.info["f"]), dtype=np.uint64)
        _check(lib().ocffm_data_get_ds(self.h, _ptr(out)))
        return out[: self.info["f"]]

    def labels(self):
        """(yptr, ycol) as parsed (ffm.cpp:93-101)."""
        i = self.info
        yptr = np.zeros(i["m"] + 1, dtype=np.uint64)
        ycol = np.zeros(max(1, i["nnz_y"]), dtype=np.uint64)
        _check(lib().ocffm_data_get_labels(self.h, _ptr(yptr), _ptr(ycol)))
        return yptr, ycol[: i["nnz_y"]]

    def field(self, fi: int):
        """(xptr, xidx, xval) of one field after split_fields (ffm.cpp:185-257)."""
        nnz = C.c_uint64(0)
        _check(lib().ocffm_data_get_field(self.h, fi, None, None, None, C.byref(nnz)))
        xptr = np.zeros(self.info["m"] + 1, dtype=np.int64)
        xidx = np.zeros(max(1, nnz.value), dtype=np.uint32)
        xval = np.zeros(max(1, nnz.value), dtype=np.float64)
        _check(lib().ocffm_data_get_field(self.h, fi, _ptr(xptr), _ptr(xidx), _ptr(xval), C.byref(nnz)))
        return xptr, xidx[: nnz.value], xval[: nnz.value]

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ocffm_data_free(self.h)
            self.h = None


class _SgdParam(C.Structure):
    _fields_ = [("k", C.c_uint32), ("eta", C.c_float), ("lambda_", C.c_float), ("nneg", C.c_uint32),
                ("neg_power", C.c_double), ("adagrad", C.c_int32), ("norm", C.c_int32), ("serial", C.c_int32),
                ("seed", C.c_uint64), ("device", C.c_int32)]


class _SgdInfo(C.Structure):
    _fields_ = [("n_features", C.c_uint64), ("n_fields", C.c_uint32), ("kp", C.c_uint32),
                ("positives", C.c_uint64), ("instances", C.c_uint64)]


class SgdTrainer:
    """Field-aware FM by per-instance SGD / AdaGrad with HOGWILD writes and
    on-device negative sampling (include/ocffm.h, SGD mode).  North-star
    extra with no reference counterpart: parity is against
    oracle/sgd_oracle.cpp, not the reference."""

    def __init__(self, U: "ImpData", V: "ImpData", rank: int = 0, nranks: int = 1, comm: Optional[bytes] = None,
                 allreduce=None, **kw):
        p = _SgdParam()
        lib().ocffm_sgd_param_default(C.byref(p))
        for key, val in kw.items():
            setattr(p, "lambda_" if key == "lambda" else key, val)
        self.param = p
        self._keep = (U, V)
        h = C.c_void_p()
        if allreduce is not None:  # average() through a host all-reduce (float32 arrays)
            def cb(buf, count, is_double, user):
                try:
                    allreduce(np.ctypeslib.as_array(C.cast(buf, C.POINTER(C.c_float)), shape=(count,)))
                    return 0
                except Exception:  # pragma: no cover
                    return 1
            self._cb = ALLREDUCE_FN(cb)
            _check(lib().ocffm_sgd_create_dist_host(U.h, V.h, C.byref(p), rank, nranks, self._cb, None, C.byref(h)))
        elif nranks > 1 or comm is not None:
            idb = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(comm)
            _check(lib().ocffm_sgd_create_dist(U.h, V.h, C.byref(p), rank, nranks, idb, C.byref(h)))
        else:
            _check(lib().ocffm_sgd_create(U.h, V.h, C.byref(p), C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ocffm_sgd_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    @property
    def info(self) -> dict:
        i = _SgdInfo()
        _check(lib().ocffm_sgd_get_info(self.h, C.byref(i)))
        return dict(n_features=i.n_features, n_fields=i.n_fields, kp=i.kp, positives=i.positives,
                    instances=i.instances)

    def epoch(self) -> float:
        loss = C.c_double(0)
        _check(lib().ocffm_sgd_epoch(self.h, C.byref(loss)))
        return loss.value

    def average(self) -> None:
        _check(lib().ocffm_sgd_average(self.h))

    def phi(self, users, items) -> np.ndarray:
        u = np.ascontiguousarray(users, dtype=np.uint32)
        v = np.ascontiguousarray(items, dtype=np.uint32)
        out = np.zeros(max(1, u.size), dtype=np.float32)
        _check(lib().ocffm_sgd_phi(self.h, u.size, _ptr(u), _ptr(v), _ptr(out)))
        return out[: u.size]

    def get(self, what: str) -> np.ndarray:
        n = C.c_uint64(0)
        _check(lib().ocffm_sgd_get(self.h, what.encode(), None, 0, C.byref(n)))
        dt = {"W": np.float32, "G": np.float32, "p": np.float32, "a": np.uint32, "o": np.uint64}[what]
        out = np.zeros(max(1, n.value), dtype=dt)
        _check(lib().ocffm_sgd_get(self.h, what.encode(), _ptr(out), n.value, C.byref(n)))
        return out[: n.value]

    def set_w(self, w) -> None:
        a = np.ascontiguousarray(w, dtype=np.float32)
        _check(lib().ocffm_sgd_set_w(self.h, _ptr(a), a.size))

    def sync(self) -> None:
        _check(lib().ocffm_sgd_sync(self.h))


def comm_id() -> bytes:
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    _check(lib().ocffm_comm_id(buf))
    return bytes(buf)


class ImpProblem:
    """class ImpProblem (ffm.h:82-151) on the GPU.

    ``nranks > 1`` shards the training rows (one process per GPU); the
    partial gradient / Hessian-vector sums are all-reduced with RCCL
    (``comm_id`` from rank 0), or through ``allreduce(np_array)`` on the host
    when given (tests: gloo)."""

    def __init__(self, U: ImpData, Uva: Optional[ImpData], V: ImpData, param: Parameter, rank: int = 0,
                 nranks: int = 1, comm: Optional[bytes] = None, allreduce=None):
        h = C.c_void_p()
        self._keep = (U, Uva, V)
        self.param = param
        uva = None if Uva is None else Uva.h
        if allreduce is not None:
            def cb(buf, count, is_double, user):
                try:
                    ctype = C.c_double if is_double else C.c_float
                    arr = np.ctypeslib.as_array(C.cast(buf, C.POINTER(ctype)), shape=(count,))
                    allreduce(arr)
                    return 0
                except Exception:  # pragma: no cover
                    return 1
            self._cb = ALLREDUCE_FN(cb)
            _check(lib().ocffm_problem_create_dist_host(U.h, uva, V.h, C.byref(param._p), rank, nranks, self._cb,
                                                        None, C.byref(h)))
        elif nranks > 1 or comm is not None:
            idb = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(comm)
            _check(lib().ocffm_problem_create_dist(U.h, uva, V.h, C.byref(param._p), rank, nranks, idb,
                                                   C.byref(h)))
        else:
            _check(lib().ocffm_problem_create(U.h, uva, V.h, C.byref(param._p), C.byref(h)))
        self.h = h
        self.f = int(U.info["f"] + V.info["f"])
        self.k = int(param.k)

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ocffm_problem_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def n_blocks(self) -> int:
        """Field-pair blocks f(f+1)/2 (ffm.cpp:53-55); unused ones (--ns) included."""
        return self.f * (self.f + 1) // 2

    def init(self):
        _check(lib().ocffm_problem_init(self.h))

    def one_epoch(self):
        _check(lib().ocffm_problem_one_epoch(self.h))

    def solve_block(self, f1, f2):
        _check(lib().ocffm_problem_solve_block(self.h, f1, f2))

    def cache_sasb(self):
        _check(lib().ocffm_problem_cache_sasb(self.h))

    def solve(self):
        _check(lib().ocffm_problem_solve(self.h))

    def validate(self) -> dict:
        m = _Metrics()
        _check(lib().ocffm_problem_validate(self.h, C.byref(m)))
        return dict(loss=m.loss, prec=np.array(m.prec[:]), ndcg=np.array(m.ndcg[:]), top_k=list(m.top_k))

    def test_rows(self) -> int:
        """This rank's test rows (0 without a test set)."""
        n = C.c_uint64()
        _check(lib().ocffm_problem_test_rows(self.h, C.byref(n)))
        return int(n.value)

    def validate_forced(self):
        """The reference's nDCG known-answer build (ffm.cpp:988-993): metrics
        and the per-row nDCG@5,10,20,40,80 (shape rows x 5) with the scores
        forced to z_j = n - j."""
        m = _Metrics()
        mt = self.test_rows()
        rows = np.zeros(max(1, mt) * 5, dtype=np.float64)
        _check(lib().ocffm_problem_validate_forced(self.h, C.byref(m), _ptr(rows), rows.size))
        return dict(loss=m.loss, prec=np.array(m.prec[:]), ndcg=np.array(m.ndcg[:])), rows[:mt * 5].reshape(mt, 5)

    def save_binary(self, path: str) -> None:
        _check(lib().ocffm_problem_save_binary(self.h, path.encode()))

    def load_binary(self, path: str) -> None:
        _check(lib().ocffm_problem_load_binary(self.h, path.encode()))

    def get(self, what: str, b12: int = 0) -> np.ndarray:
        n = C.c_uint64(0)
        _check(lib().ocffm_problem_get(self.h, what.encode(), b12, None, 0, C.byref(n)))
        out = np.zeros(n.value, dtype=np.float64)
        _check(lib().ocffm_problem_get(self.h, what.encode(), b12, _ptr(out), n.value, C.byref(n)))
        return out

    def set(self, what: str, b12: int, arr) -> None:
        a = np.ascontiguousarray(arr, dtype=np.float64)
        _check(lib().ocffm_problem_set(self.h, what.encode(), b12, _ptr(a), a.size))

    def grad(self, f1, f2, half) -> np.ndarray:
        size = self.get("W" if half == 0 else "H", block_index(f1, f2, self.f)).size
        out = np.zeros(size, dtype=np.float64)
        _check(lib().ocffm_problem_grad(self.h, f1, f2, half, _ptr(out)))
        return out

    def hv(self, f1, f2, half, v) -> np.ndarray:
        v = np.ascontiguousarray(v, dtype=np.float64)
        out = np.zeros_like(v)
        _check(lib().ocffm_problem_hv(self.h, f1, f2, half, _ptr(v), _ptr(out)))
        return out

    def save_model(self, path: str) -> None:
        _check(lib().ocffm_problem_save_model(self.h, path.encode()))

    def cg_log(self) -> np.ndarray:
        n = C.c_int(0)
        _check(lib().ocffm_problem_cg_log(self.h, None, 0, C.byref(n)))
        out = np.zeros(max(1, n.value), dtype=np.int32)
        _check(lib().ocffm_problem_cg_log(self.h, _ptr(out), n.value, C.byref(n)))
        return out[: n.value]

    def set_profiling(self, on: bool) -> None:
        _check(lib().ocffm_problem_set_profiling(self.h, int(on)))

    def set_profile_filter(self, name: Optional[str]) -> None:
        _check(lib().ocffm_problem_set_profile_filter(self.h, (name or "").encode()))

    def kernel_stats(self) -> dict:
        n = C.c_int(0)
        _check(lib().ocffm_problem_kernel_stats(self.h, None, 0, C.byref(n)))
        arr = (_KStat * max(1, n.value))()
        _check(lib().ocffm_problem_kernel_stats(self.h, arr, n.value, C.byref(n)))
        return {arr[i].name.decode(): dict(launches=arr[i].launches, total_ms=arr[i].total_ms,
                                           alg_bytes=arr[i].alg_bytes, alg_flops=arr[i].alg_flops)
                for i in range(n.value)}

    def reset_stats(self) -> None:
        _check(lib().ocffm_problem_reset_stats(self.h))

    def alg_bytes(self) -> float:
        b = C.c_double(0)
        _check(lib().ocffm_problem_alg_bytes(self.h, C.byref(b)))
        return b.value

    def counter(self, name: str) -> int:
        """Diagnostic event counter (include/ocffm.h ocffm_problem_counter)."""
        v = C.c_int64(0)
        _check(lib().ocffm_problem_counter(self.h, name.encode(), C.byref(v)))
        return v.value

    def sync(self) -> None:
        _check(lib().ocffm_problem_sync(self.h))

    def layout_digest(self) -> dict:
        """{array name: FNV-1a digest} of the device data layout (ocffm.h)."""
        n = C.c_int(0)
        _check(lib().ocffm_problem_layout_digest(self.h, None, None, 0, C.byref(n)))
        names = C.create_string_buffer(48 * max(1, n.value))
        dig = (C.c_uint64 * max(1, n.value))()
        _check(lib().ocffm_problem_layout_digest(self.h, names, dig, n.value, C.byref(n)))
        raw = names.raw
        return {raw[48 * i:48 * (i + 1)].split(b"\0", 1)[0].decode(): int(dig[i]) for i in range(n.value)}


def srand(seed: int = 1) -> None:
    """glibc srand(): the reference's init draws from the process rand() stream."""
    C.CDLL(None).srand(C.c_uint(seed))


def problem_from_dataset(ds, precision=FP64, with_test=True, device=0, rank=0, nranks=1, comm=None,
                         allreduce=None, **overrides) -> ImpProblem:
    """Build an ImpProblem from a synth.Dataset (train.cpp:177-196 order)."""
    p = ds.params
    prm = Parameter(omega=overrides.get("omega", p["w"]), lambda_=overrides.get("lam", p["l"]),
                    r=overrides.get("r", p["r"]), nr_pass=overrides.get("t", p["t"]),
                    k=overrides.get("k", p["k"]), precision=precision, device=device,
                    self_side=int(overrides.get("self_side", True)), freq=int(overrides.get("freq", False)))
    U = ImpData.from_rows(ds.train)
    V = ImpData.from_rows(ds.item)
    V.trans_y(U)
    Ut = ImpData.from_rows(ds.test, ds=U.Ds) if (with_test and ds.test is not None) else None
    return ImpProblem(U, Ut, V, prm, rank=rank, nranks=nranks, comm=comm, allreduce=allreduce)
