"""lookup / lookup! / maplookup / maplookup! on the HIP engine.

Mirrors src/lookup.jl (darchr/EmbeddingTables.jl):
  destination            :19-22
  lookup / lookup!       :35-43, vector dispatch :90-102, matrix dispatch :167-182
  ColumnWrap / colwrap   :195-213
  DefaultStrategy        :220-241 and its rrule :246-258
  SimpleParallelStrategy :262-276
  PreallocationStrategy  :284-371 and its rrule :374-389

Every hot call is ONE C-ABI launch on torch's current stream; there is no CPU
path.  Names with a trailing underscore are Julia's bang functions
(``lookup_`` = ``lookup!``).
"""
from __future__ import annotations

import ctypes
import threading

import torch

from . import _lib
from .tables import AbstractEmbeddingTable, ArgumentError, featuresize, example


class AbstractExecutionStrategy:
    pass


class DefaultStrategy(AbstractExecutionStrategy):
    """One lookup per table (src/lookup.jl:220-241)."""


class SimpleParallelStrategy(AbstractExecutionStrategy):
    """Per-table parallelism (src/lookup.jl:262-276).  On the GPU every table's lookup
    is already a full-chip launch; the result is identical to DefaultStrategy."""


class PreallocationStrategy(AbstractExecutionStrategy):
    """Fused lookup + concat into one ``(prependrows + sum(D)) x B`` matrix
    (src/lookup.jl:284-291).  ``eltype`` is the reference's type parameter ``T``
    (``Any`` = the tables' element type)."""

    def __init__(self, prependrows: int = 0, eltype: torch.dtype | None = None):
        self.prependrows = int(prependrows)
        self.eltype = eltype

    def __repr__(self):
        return f"PreallocationStrategy({self.prependrows})"


class NoTangent:
    """ChainRulesCore.NoTangent()."""

    _inst = None

    def __new__(cls):
        if cls._inst is None:
            cls._inst = super().__new__(cls)
        return cls._inst

    def __repr__(self):
        return "NoTangent()"


# --- argument plumbing ---------------------------------------------------------------

def _check_table(A):
    if not isinstance(A, AbstractEmbeddingTable):
        raise TypeError(f"expected an AbstractEmbeddingTable, got {type(A).__name__}")
    if not A.example().is_cuda:
        raise ArgumentError("the HIP engine needs tables in device memory")


def _check_idx(I: torch.Tensor) -> torch.Tensor:
    if not isinstance(I, torch.Tensor):
        raise TypeError("indices must be an int64 torch tensor")
    if I.dtype != torch.int64:
        raise TypeError(f"indices must be int64 (Julia Int), got {I.dtype}")
    if not I.is_cuda:
        raise ArgumentError("indices must be in device memory")
    if I.dim() not in (1, 2):
        raise ArgumentError("lookup indices are a vector or a (B, P) matrix")
    if I.numel() > 0 and I.stride(-1) != 1:
        raise ArgumentError("a bag's indices must be contiguous (stride(-1) == 1)")
    return I


def _ld(x: torch.Tensor) -> int:
    """Leading dimension (elements between consecutive Julia columns) of a 2-D tensor."""
    if x.dim() == 1:
        return 1
    return int(x.stride(0)) if x.shape[0] > 1 else max(int(x.shape[1]), 1)


def _check_dst(dst: torch.Tensor, A, B: int):
    if not isinstance(dst, torch.Tensor) or dst.dim() != 2:
        raise ArgumentError("destination must be a 2-D (B, D) tensor")
    if dst.dtype != A.dtype:
        raise ArgumentError(f"destination eltype {dst.dtype} != table eltype {A.dtype}")
    if dst.shape[0] != B or dst.shape[1] != featuresize(A):
        raise ArgumentError(f"destination shape {tuple(dst.shape)} != ({B}, {featuresize(A)})")
    if dst.numel() > 0 and dst.stride(1) != 1:
        raise ArgumentError("destination features must be contiguous")


def _trailing_size(I: torch.Tensor) -> int:
    """src/lookup.jl:19: size(I, ndims(I)) — the batch (torch dim 0)."""
    return int(I.shape[0])


def destination(A: AbstractEmbeddingTable, I: torch.Tensor) -> torch.Tensor:
    """src/lookup.jl:20-22: ``similar(example(A), eltype(A), featuresize(A), B)``."""
    return torch.empty((_trailing_size(I), featuresize(A)), dtype=A.dtype, device=A.device)


# --- lookup ---------------------------------------------------------------------------

def lookup(A: AbstractEmbeddingTable, I: torch.Tensor) -> torch.Tensor:
    """``lookup(A, I)`` (src/lookup.jl:35-40): vector index -> gather, matrix -> pooled sum."""
    _check_table(A)
    _check_idx(I)
    return lookup_(destination(A, I), A, I)


def lookup_(dst: torch.Tensor, A: AbstractEmbeddingTable, I: torch.Tensor,
            nontemporal: bool = True) -> torch.Tensor:
    """``lookup!(dst, A, I)``: one kernel launch; returns ``dst``.

    ``nontemporal`` mirrors the reference's non-temporal stores of the static path
    (src/lookup.jl:161)."""
    _check_table(A)
    _check_idx(I)
    B = _trailing_size(I)
    _check_dst(dst, A, B)
    L = _lib.load()
    D, R = A.size()
    flags = _lib.ET_FLAG_NONTEMPORAL if nontemporal else 0
    table, cpp = A.device_table()
    if cpp:
        # paged table (SplitEmbedding): the descriptor entry point addresses pages
        descs = (_lib.LookupDesc * 1)()
        descs[0] = _lib.LookupDesc(table, A.ld, R, D, 1 if I.dim() == 1 else int(I.shape[1]),
                                   I.data_ptr(), 1 if I.dim() == 1 else _ld(I), 0, cpp)
        rc = L.et_maplookup_prealloc(_lib.et_dtype(dst), ctypes.addressof(descs), 1, B,
                                     dst.data_ptr(), _ld(dst), flags,
                                     _lib.stream_handle(dst.device))
    elif I.dim() == 1:
        rc = L.et_gather(_lib.et_dtype(dst), table, A.ld, R, D, I.data_ptr(), B,
                         dst.data_ptr(), _ld(dst), flags, _lib.stream_handle(dst.device))
    else:
        P = int(I.shape[1])
        rc = L.et_pooled_sum(_lib.et_dtype(dst), table, A.ld, R, D, I.data_ptr(), P,
                             _ld(I), B, dst.data_ptr(), _ld(dst), flags,
                             _lib.stream_handle(dst.device))
    _lib.check(rc)
    return dst


# --- ColumnWrap (src/lookup.jl:195-213) --------------------------------------------------

def colwrap(I):
    """Vector of index arrays -> as is; a stacked tensor -> its per-table slices.

    A Julia ``B x T`` matrix / ``P x B x T`` array is a torch ``(T, B)`` / ``(T, B, P)``
    tensor, so table ``t`` is ``I[t]``."""
    if isinstance(I, (list, tuple)):
        return list(I)
    if isinstance(I, torch.Tensor):
        if I.dim() < 2:
            raise ArgumentError("a stacked index tensor needs a table dimension")
        return [I[t] for t in range(I.shape[0])]
    raise TypeError(f"unsupported index container {type(I).__name__}")


def _batchsize(I) -> int:
    """src/lookup.jl:296-299."""
    return _trailing_size(colwrap(I)[0])


# --- maplookup --------------------------------------------------------------------------

def maplookup(*args, **kw):
    """``maplookup([strategy], tables, I)`` (src/lookup.jl:221-231, :305-314)."""
    if args and isinstance(args[0], AbstractExecutionStrategy):
        strategy, tables, I = args
    else:
        strategy = DefaultStrategy()
        tables, I = args
    if isinstance(strategy, PreallocationStrategy):
        tables = list(tables)
        ncols = strategy.prependrows + sum(featuresize(t) for t in tables)
        dtype = strategy.eltype or tables[0].dtype
        dst = torch.empty((_batchsize(I), ncols), dtype=dtype, device=tables[0].device)
        return maplookup_(strategy, dst, tables, I, **kw)
    Is = colwrap(I)
    y = [destination(A, i) for A, i in zip(tables, Is)]
    return maplookup_(strategy, y, tables, Is, **kw)


def maplookup_(strategy: AbstractExecutionStrategy, dst, tables, I, nontemporal: bool = True,
               worksize_div: int = 8, f16_fp32_acc: bool = False):
    """``maplookup!(strategy, dst, tables, I)``.

    Default / SimpleParallel: one launch per table.  Preallocation: ONE fused launch
    for every table (``worksize_div`` is accepted for signature parity; the GPU grid
    replaces the reference's 8-chunks-per-table CPU work queue)."""
    tables = list(tables)
    Is = colwrap(I)
    if len(Is) != len(tables):
        raise ArgumentError(f"{len(tables)} tables but {len(Is)} index arrays")
    if not isinstance(strategy, PreallocationStrategy):
        return [lookup_(y, A, i, nontemporal) for y, A, i in zip(dst, tables, Is)]

    if not tables:
        return dst
    return PreallocationPlan(strategy, dst, tables, Is, nontemporal, f16_fp32_acc)()


# Queue blocks of the per-XCD work-queue schedule (et_maplookup_prealloc_q), one per
# (device, stream, thread): calls that share a block are ordered by their stream.  Zeroed once
# on that stream when made; every launch leaves its block zero again.
# one block per (device, stream handle) PER THREAD, in thread-local storage: two threads never
# share a block, and a thread's blocks are freed when it exits
_QUEUE_BLOCKS = threading.local()


def _queue_block(device: torch.device, stream: int):
    """The queue block for launches on `stream`, or None while the stream is capturing a
    HIP graph (the captured launch keeps the static stripe schedule: a block allocated
    during a capture would be graph-private memory)."""
    with torch.cuda.device(device):  # the capture state of THIS device's current stream
        if torch.cuda.is_current_stream_capturing():
            return None
    blocks = getattr(_QUEUE_BLOCKS, "d", None)
    if blocks is None:
        blocks = _QUEUE_BLOCKS.d = {}
    key = (device.index, stream)
    q = blocks.get(key)
    if q is None:
        q = torch.zeros(_lib.ET_LOOKUP_QUEUE_BYTES // 4, dtype=torch.int32, device=device)
        blocks[key] = q
    return q


class PreallocationPlan:
    """``maplookup!(PreallocationStrategy(k), dst, tables, I)`` with the descriptors
    validated and built once for fixed tables, index buffers and destination: each
    call is one call into the library (no per-table Python work) — for serving loops
    that refill the index buffers in place, and for the sharded step's chunks."""

    def __init__(self, strategy: PreallocationStrategy, dst, tables, I, nontemporal=True,
                 f16_fp32_acc: bool = False):
        tables = list(tables)
        Is = colwrap(I)
        if len(Is) != len(tables):
            raise ArgumentError(f"{len(tables)} tables but {len(Is)} index arrays")
        if not tables:
            raise ArgumentError("a plan needs at least one table")
        B = _batchsize(Is)
        k = strategy.prependrows
        if dst.dim() != 2 or dst.shape[0] != B:
            raise ArgumentError(f"destination must be ({B}, prependrows + sum(D))")
        if dst.numel() > 0 and dst.stride(1) != 1:
            raise ArgumentError("destination features must be contiguous")
        if k + sum(featuresize(t) for t in tables) > dst.shape[1]:
            raise ArgumentError("destination has too few rows for prependrows + sum(D)")
        dtype = tables[0].dtype  # the tables' element type; dst may be another (U)
        descs = (_lib.LookupDesc * len(tables))()
        off = k
        for t, (A, i) in enumerate(zip(tables, Is)):
            _check_table(A)
            _check_idx(i)
            if A.dtype != dtype:
                raise NotImplementedError(
                    f"table {t} eltype {A.dtype} != table 0 eltype {dtype}: one launch takes "
                    "tables of one element type")
            if _trailing_size(i) != B:
                raise ArgumentError(f"table {t}: batch {_trailing_size(i)} != {B}")
            D, R = A.size()
            pool = 1 if i.dim() == 1 else int(i.shape[1])
            table, cpp = A.device_table()
            descs[t] = _lib.LookupDesc(table, A.ld, R, D, pool, i.data_ptr(),
                                       1 if i.dim() == 1 else _ld(i), off, cpp)
            off += D
        self._keep = (dst, tables, Is)  # the buffers the descriptors point into
        self._descs = descs
        self._n = len(tables)
        self._B = B
        self._flags = _lib.ET_FLAG_NONTEMPORAL if nontemporal else 0
        if f16_fp32_acc:  # Float16 tables: fp32 sums, one rounding (not Julia's Float16 ops)
            self._flags |= _lib.ET_FLAG_F16_FP32_ACC
        self._src = _lib.TORCH_TO_ET[dtype]
        self._dst_t = _lib.et_dtype(dst)
        self._dst = dst
        self._ld = _ld(dst)
        self._lib = _lib.load()

    def __call__(self):
        """Launch on the current stream; returns the destination."""
        dst = self._dst
        stream = _lib.stream_handle(dst.device)
        if self._src == self._dst_t:
            q = _queue_block(dst.device, stream)
            _lib.check(self._lib.et_maplookup_prealloc_q(
                self._src, ctypes.addressof(self._descs), self._n, self._B, dst.data_ptr(),
                self._ld, self._flags, q.data_ptr() if q is not None else None, stream))
        else:  # PreallocationStrategy{U}: sums in the table type, converted on the store
            _lib.check(self._lib.et_maplookup_prealloc_to(
                self._src, self._dst_t, ctypes.addressof(self._descs), self._n, self._B,
                dst.data_ptr(), self._ld, self._flags, stream))
        return dst
