"""TEST INFRASTRUCTURE ONLY — numpy/ctypes front end of the CPU oracle.

The oracle restates darchr/EmbeddingTables.jl's hot path on the CPU
(``embtab_oracle.c``, function by function with reference file:line citations)
plus a pure-numpy "naive" restatement of the reference's own reference
implementations (``src/lookup.jl:5-13``).  It is the parity checker for the HIP
engine and the timed CPU baseline of ``bench.py``.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import it;
``embeddingtables.jl_amd/`` (the product) never does.

Array conventions follow the engine (a Julia ``D x N`` column-major matrix is
the C-contiguous numpy array of shape ``(N, D)``; indices are 1-based int64).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liborc.so")

F32, F16, F64, I32, I64, BF16 = 0, 1, 2, 3, 4, 5
_DTYPES = {
    np.dtype(np.float32): F32,
    np.dtype(np.float16): F16,
    np.dtype(np.float64): F64,
    np.dtype(np.int32): I32,
    np.dtype(np.int64): I64,
}


class LookupDesc(ctypes.Structure):
    _fields_ = [
        ("table", ctypes.c_void_p),
        ("ld_table", ctypes.c_int64),
        ("nrows", ctypes.c_int64),
        ("dim", ctypes.c_int32),
        ("pool", ctypes.c_int32),
        ("idx", ctypes.c_void_p),
        ("ld_idx", ctypes.c_int64),
        ("dst_row_off", ctypes.c_int64),
    ]


class UpdateDesc(ctypes.Structure):
    _fields_ = [
        ("table", ctypes.c_void_p),
        ("ld_table", ctypes.c_int64),
        ("nrows", ctypes.c_int64),
        ("dim", ctypes.c_int32),
        ("pool", ctypes.c_int32),
        ("delta", ctypes.c_void_p),
        ("ld_delta", ctypes.c_int64),
        ("idx", ctypes.c_void_p),
        ("ld_idx", ctypes.c_int64),
        ("batch", ctypes.c_int64),
    ]


_lib = None


def build():
    """Compile liborc.so with the committed Makefile (gcc only)."""
    import subprocess

    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, i32, dbl, u64 = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                  ctypes.c_double, ctypes.c_uint64)
        L.orc_gather.argtypes = [ctypes.c_int, vp, i64, i32, vp, i64, vp, i64]
        L.orc_pooled_sum.argtypes = [ctypes.c_int, vp, i64, i32, vp, i32, i64, i64, vp, i64,
                                     ctypes.c_int]
        L.orc_maplookup_prealloc.argtypes = [ctypes.c_int, vp, i32, i64, vp, i64, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int]
        L.orc_histogram.argtypes = [vp, i32, i64, i64, i64, ctypes.c_int, vp, vp, vp]
        L.orc_histogram.restype = i64
        L.orc_index_build.argtypes = [vp, i32, i64, i64, i64, ctypes.c_int, vp, vp, vp]
        L.orc_index_build.restype = i64
        L.orc_sgd_f32.argtypes = [vp, dbl, ctypes.c_int, ctypes.c_int]
        L.orc_sgd_multi_f32.argtypes = [vp, i32, dbl, vp, ctypes.c_int, ctypes.c_int]
        L.orc_sgd_typed.argtypes = [vp, ctypes.c_int, ctypes.c_int, dbl, ctypes.c_int,
                                    ctypes.c_int]
        L.orc_sgd_multi_typed.argtypes = [vp, i32, ctypes.c_int, ctypes.c_int, dbl, vp,
                                          ctypes.c_int, ctypes.c_int]
        L.orc_f64_to_f16.argtypes = [dbl]
        L.orc_f64_to_f16.restype = ctypes.c_uint16
        L.orc_fill_uniform.argtypes = [ctypes.c_int, vp, i64, u64, u64, dbl, dbl, ctypes.c_int]
        L.orc_fill_index_uniform.argtypes = [vp, i64, i64, u64, u64, ctypes.c_int]
        L.orc_f32_to_f16.argtypes = [ctypes.c_float]
        L.orc_f32_to_f16.restype = ctypes.c_uint16
        L.orc_now.restype = dbl
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _dt(a: np.ndarray, bf16: bool = False) -> int:
    """Element type code; bfloat16 arrays are uint16 bit patterns flagged by ``bf16``."""
    if bf16:
        assert a.dtype == np.uint16
        return BF16
    return _DTYPES[a.dtype]


def f32_to_bf16(x: np.ndarray) -> np.ndarray:
    """float32 -> bfloat16 bits (uint16), round to nearest even (NaN -> quiet NaN)."""
    b = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    nan = (b & 0x7fffffff) > 0x7f800000
    r = ((b + 0x7fff + ((b >> 16) & 1)) >> 16).astype(np.uint16)
    return np.where(nan, ((b >> 16) | 0x40).astype(np.uint16), r)


def bf16_to_f32(h: np.ndarray) -> np.ndarray:
    return (np.ascontiguousarray(h, np.uint16).astype(np.uint32) << 16).view(np.float32)


def _idx2d(I: np.ndarray) -> np.ndarray:
    """1-D index vector -> (B, 1) bag-major matrix; 2-D (B, P) kept."""
    I = np.ascontiguousarray(I, dtype=np.int64)
    return I.reshape(-1, 1) if I.ndim == 1 else I


# --- lookup ---------------------------------------------------------------------

def gather(table: np.ndarray, I: np.ndarray, bf16: bool = False) -> np.ndarray:
    """src/lookup.jl:51-87 — out[j] = table[I[j]-1] (bit copy)."""
    table = np.ascontiguousarray(table)
    I = np.ascontiguousarray(I, dtype=np.int64)
    out = np.empty((I.shape[0], table.shape[1]), dtype=table.dtype)
    lib().orc_gather(_dt(table, bf16), _ptr(table), table.shape[1], table.shape[1], _ptr(I),
                     I.shape[0], _ptr(out), out.shape[1])
    return out


def pooled_sum(table: np.ndarray, I: np.ndarray, f16_fp32_acc: bool = False,
               bf16: bool = False) -> np.ndarray:
    """src/lookup.jl:108-165 — out[j] = sum_i table[I[j, i]-1], sequential in i."""
    table = np.ascontiguousarray(table)
    I = _idx2d(I)
    B, P = I.shape
    out = np.empty((B, table.shape[1]), dtype=table.dtype)
    lib().orc_pooled_sum(_dt(table, bf16), _ptr(table), table.shape[1], table.shape[1], _ptr(I), P, P,
                         B, _ptr(out), out.shape[1], int(f16_fp32_acc))
    return out


def lookup(table: np.ndarray, I: np.ndarray, bf16: bool = False) -> np.ndarray:
    """Dispatch like src/lookup.jl:35-40: vector -> gather, matrix -> pooled sum."""
    return gather(table, I, bf16) if np.ndim(I) == 1 else pooled_sum(table, I, bf16=bf16)


def maplookup_prealloc(tables, indices, prependrows: int = 0, nthreads: int = 1,
                       worksize_div: int = 8, out: np.ndarray | None = None,
                       f16_fp32_acc: bool = False, bf16: bool = False) -> np.ndarray:
    """src/lookup.jl:305-371 — fused concat, (B, prependrows + sum D) output."""
    tables = [np.ascontiguousarray(t) for t in tables]
    idx = [_idx2d(I) for I in indices]
    B = idx[0].shape[0]
    ld = prependrows + sum(t.shape[1] for t in tables)
    if out is None:
        out = np.zeros((B, ld), dtype=tables[0].dtype)
    descs = (LookupDesc * len(tables))()
    off = prependrows
    for k, (t, I) in enumerate(zip(tables, idx)):
        descs[k] = LookupDesc(_ptr(t), t.shape[1], t.shape[0], t.shape[1], I.shape[1], _ptr(I),
                              I.shape[1], off)
        off += t.shape[1]
    lib().orc_maplookup_prealloc(_dt(out, bf16), ctypes.addressof(descs), len(tables), B, _ptr(out),
                                 ld, nthreads, worksize_div, int(f16_fp32_acc))
    return out


# --- Indexer --------------------------------------------------------------------

def histogram(A: np.ndarray, maxindex: int, dense: bool = False):
    """src/utils.jl:131-167 — returns (keys in first-seen order, order, count)."""
    I = _idx2d(A) if np.ndim(A) == 1 else np.ascontiguousarray(np.asarray(A, np.int64))
    B, P = I.shape
    n = B * P
    keys = np.zeros(n + 1, np.int64)
    order = np.zeros(n + 1, np.int64)
    count = np.zeros(n + 1, np.int64)
    U = lib().orc_histogram(_ptr(I), P, P, B, maxindex, int(dense), _ptr(keys), _ptr(order),
                            _ptr(count))
    return keys[:U], order[:U], count[:U]


def index_build(A: np.ndarray, maxindex: int, dense: bool = False):
    """src/utils.jl:306-314 index! — (cumulative [(col, offset)...], map), 1-based."""
    I = _idx2d(A)
    B, P = I.shape
    n = B * P
    cc = np.zeros(n + 1, np.int64)
    co = np.zeros(n + 1, np.int64)
    m = np.zeros(max(n, 1), np.int64)
    U = lib().orc_index_build(_ptr(I), P, P, B, maxindex, int(dense), _ptr(cc), _ptr(co),
                              _ptr(m))
    return np.stack([cc[:U + 1], co[:U + 1]], axis=1), m[:n]


# --- update ---------------------------------------------------------------------

def _upd_type(table: np.ndarray, bf16: bool) -> int:
    code = _dt(table, bf16)
    assert code in (F32, F64, F16, BF16) and table.flags.c_contiguous
    return code


def sgd(table: np.ndarray, delta: np.ndarray, I: np.ndarray, eta: float, fused: bool = True,
        dense_indexer: bool = False, bf16: bool = False, f16_fp32_acc: bool = False) -> None:
    """src/sparseupdate.jl:160-178 — in-place Descent update; Float32 tables follow the
    reference exactly, Float64 / Float16 / BFloat16 the typed model of
    embtab_oracle.c (``bf16``: uint16 bit patterns; ``delta`` of the table's type)."""
    code = _upd_type(table, bf16)
    I = _idx2d(I)
    delta = np.ascontiguousarray(delta, table.dtype)
    B, P = I.shape
    d = UpdateDesc(_ptr(table), table.shape[1], table.shape[0], table.shape[1], P, _ptr(delta),
                   delta.shape[1], _ptr(I), P, B)
    if code == F32:
        lib().orc_sgd_f32(ctypes.byref(d), float(eta), int(fused), int(dense_indexer))
    else:
        lib().orc_sgd_typed(ctypes.byref(d), code, int(f16_fp32_acc), float(eta), int(fused),
                            int(dense_indexer))


def sgd_multi(tables, deltas, indices, eta: float, fused, num_splits: int = 4,
              nthreads: int = 1, delta_ld: int | None = None, delta_offsets=None,
              bf16: bool = False, f16_fp32_acc: bool = False) -> None:
    """src/sparseupdate.jl:199-238 — multi-table threaded update (in place).

    ``deltas`` is either a list of (B, D_t) arrays, or one (B, ld) array with
    ``delta_offsets[t]`` giving each table's first column (Preallocation layout).
    Every table has the same element type.
    """
    n = len(tables)
    keep = []
    descs = (UpdateDesc * n)()
    code = _upd_type(tables[0], bf16)
    for t in range(n):
        I = _idx2d(indices[t])
        keep.append(I)
        B, P = I.shape
        tab = tables[t]
        assert _upd_type(tab, bf16) == code
        es = tab.dtype.itemsize
        if delta_offsets is None:
            dl = np.ascontiguousarray(deltas[t], tab.dtype)
            keep.append(dl)
            dptr, ldd = _ptr(dl), dl.shape[1]
        else:
            big = deltas
            dptr, ldd = _ptr(big) + es * int(delta_offsets[t]), big.shape[1]
        descs[t] = UpdateDesc(_ptr(tab), tab.shape[1], tab.shape[0], tab.shape[1], P, dptr, ldd,
                              _ptr(I), P, B)
    fz = np.asarray([int(f) for f in fused], np.int32)
    if code == F32:
        lib().orc_sgd_multi_f32(ctypes.addressof(descs), n, float(eta), _ptr(fz), num_splits,
                                nthreads)
    else:
        lib().orc_sgd_multi_typed(ctypes.addressof(descs), n, code, int(f16_fp32_acc),
                                  float(eta), _ptr(fz), num_splits, nthreads)


# --- synthetic data ---------------------------------------------------------------

def fill_uniform(shape, dtype, seed: int, offset: int = 0, lo: float = 0.0, hi: float = 1.0,
                 nthreads: int = 8) -> np.ndarray:
    """``dtype`` "bf16" gives bfloat16 bit patterns (uint16)."""
    bf16 = dtype == "bf16"
    a = np.empty(shape, dtype=np.uint16 if bf16 else dtype)
    lib().orc_fill_uniform(BF16 if bf16 else _DTYPES[np.dtype(dtype)], _ptr(a), a.size, seed, offset, lo, hi,
                           nthreads)
    return a


def fill_index_uniform(shape, nrows: int, seed: int, offset: int = 0,
                       nthreads: int = 8) -> np.ndarray:
    a = np.empty(shape, dtype=np.int64)
    lib().orc_fill_index_uniform(_ptr(a), a.size, nrows, seed, offset, nthreads)
    return a


def now() -> float:
    return lib().orc_now()


# --- naive numpy restatement (src/lookup.jl:5-13) -----------------------------------

def naive_lookup(A: np.ndarray, I: np.ndarray) -> np.ndarray:
    """The reference's `lookup(A::AbstractMatrix, I)` with sequential sums.

    ``A[:, I]`` for a vector; for a matrix the per-bag sum is taken sequentially in
    pool order (Julia's `sum` is sequential below 16 terms — SURVEY.md §4 quirk 7)."""
    I = np.asarray(I, np.int64)
    if I.ndim == 1:
        return A[I - 1].copy()
    out = A[I[:, 0] - 1].copy()
    for i in range(1, I.shape[1]):
        out = out + A[I[:, i] - 1]
    return out
