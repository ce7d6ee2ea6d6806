"""Sparse gradients, the Indexer and the fused Descent update on the HIP engine.

Mirrors (darchr/EmbeddingTables.jl):
  SparseEmbeddingUpdate / uncompress         src/sparseupdate.jl:6-32
  rrule(lookup)                              src/sparseupdate.jl:35-40
  rrule(maplookup, strategy) (+ Slicer)      src/lookup.jl:247-258, :374-389, src/utils.jl:50-63
  update!(table, grad, indexer, alpha, Val)  src/sparseupdate.jl:46-154 (generic/specialized)
  update!(::Descent, table, grad, ...)       src/sparseupdate.jl:160-178
  Flux.Optimise.update!(opt, x, xbar, ...)   src/sparseupdate.jl:180-189
  multi-table update!(opt, tables, grads, indexers; num_splits, ...)  :199-238
  Indexer / SparseIndexer / DenseIndexer / index! / IndexerView       src/utils.jl:280-338
"""
from __future__ import annotations

import collections
import ctypes
import threading

import torch

from . import _lib
from .lookup import (NoTangent, PreallocationStrategy, AbstractExecutionStrategy, colwrap,
                     lookup, maplookup, _ld, _check_idx)
from .tables import (AbstractEmbeddingTable, AbstractLookupType, ArgumentError, Dynamic,
                     featuresize, fused_update_path)


class SparseEmbeddingUpdate:
    """Lazy gradient of a lookup: ``delta`` (the output gradient, a ``(B, D)`` tensor,
    possibly a column block of a Preallocation gradient) and the forward ``indices``
    (src/sparseupdate.jl:6-13).  Nothing is copied."""

    def __init__(self, lookup_type: AbstractLookupType, delta: torch.Tensor, indices):
        self.lookup_type = lookup_type
        self.delta = delta
        self.indices = indices

    def __repr__(self):
        return (f"SparseEmbeddingUpdate{{{self.lookup_type!r}}}(delta={tuple(self.delta.shape)}, "
                f"indices={tuple(self.indices.shape)})")


def uncompress(x: SparseEmbeddingUpdate, dstcols: int | None = None,
               maxindices: int | None = None) -> torch.Tensor:
    """Densify a sparse gradient into a ``(dstcols, D)`` tensor (src/sparseupdate.jl:16-32).
    A test helper in the reference; done with device tensor ops here."""
    I = x.indices
    if dstcols is None:
        dstcols = int(I.max().item())
    D = x.delta.shape[1]
    dst = torch.zeros((dstcols, D), dtype=x.delta.dtype, device=x.delta.device)
    ncols = x.delta.shape[0] if maxindices is None else min(maxindices, x.delta.shape[0])
    cols = I[:ncols].reshape(ncols, -1) - 1
    pool = cols.shape[1]
    src = x.delta[:ncols].repeat_interleave(pool, dim=0)
    dst.index_add_(0, cols.reshape(-1), src)
    return dst


# --- rrules -----------------------------------------------------------------------------

def rrule(f, *args):
    """``ChainRulesCore.rrule`` for ``lookup`` and ``maplookup``: returns
    ``(y, pullback)``; the pullback returns ``SparseEmbeddingUpdate``s."""
    if f is lookup:
        A, I = args
        S = A.lookup_type
        y = lookup(A, I)

        def lookup_pullback(delta):
            return (NoTangent(), SparseEmbeddingUpdate(S, delta, I), NoTangent())

        return y, lookup_pullback
    if f is maplookup:
        strategy, tables, I = args
        tables = list(tables)
        Is = colwrap(I)
        y = maplookup(strategy, tables, I)
        if isinstance(strategy, PreallocationStrategy):
            # Intended Slicer semantics: table t gets rows
            # prependrows + sum(D[<t]) .+ (1:D_t) of the gradient.
            def maplookup_pullback(delta):
                off = strategy.prependrows
                grads = []
                for A, i in zip(tables, Is):
                    D = featuresize(A)
                    grads.append(SparseEmbeddingUpdate(A.lookup_type, delta[:, off:off + D], i))
                    off += D
                return (NoTangent(), NoTangent(), grads, NoTangent())
        else:
            def maplookup_pullback(deltas):
                grads = [SparseEmbeddingUpdate(A.lookup_type, d, i)
                         for A, d, i in zip(tables, deltas, Is)]
                return (NoTangent(), NoTangent(), grads, NoTangent())
        return y, maplookup_pullback
    raise NotImplementedError(f"no rrule for {f!r}")


# --- optimiser -----------------------------------------------------------------------------

class Descent:
    """Flux.Descent(eta) — the only optimiser the reference supports."""

    def __init__(self, eta: float = 0.1):
        self.eta = float(eta)

    def __repr__(self):
        return f"Descent({self.eta})"


# --- workspaces ------------------------------------------------------------------------------

_ws_cache: "collections.OrderedDict" = collections.OrderedDict()
_WS_STREAMS = 4  # cached workspaces per (key, device): the most recently used streams
_ws_lock = threading.Lock()
_ws_pinned: dict = {}  # workspaces a HIP graph captured: never released (graphs replay into them)


def _workspace(nbytes: int, device, key: str) -> torch.Tensor:
    """A cached device byte buffer of at least ``nbytes`` (allocated outside the C call), one
    per (key, device, stream): the calls that share a workspace are then ordered on their
    stream, while calls on two streams — from two threads, or one thread alternating
    streams — never share one (round 6: a shared workspace let two threads' concurrent
    updates corrupt each other's keys and fault the GPU).  Allocated on that stream (the
    current one), so the caching allocator orders its reuse after the stream's work — which
    also makes dropping one safe while its stream still runs: at most ``_WS_STREAMS`` streams
    per (key, device) keep theirs, the least recently used is released (a program cycling
    through the pool's streams would otherwise hold a config-4-sized buffer per stream)."""
    device = torch.device(device)
    k = (key, str(device), _lib.stream_handle(device))
    with _ws_lock:
        buf = _ws_cache.get(k)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            _ws_cache[k] = buf
        _ws_cache.move_to_end(k)
        if device.type == "cuda":
            with torch.cuda.device(device):
                if torch.cuda.is_current_stream_capturing():
                    # a captured graph replays into this buffer: it outlives the cache
                    _ws_pinned[id(buf)] = buf
        same = [x for x in _ws_cache if x[:2] == k[:2]]
        for x in same[:-_WS_STREAMS]:
            del _ws_cache[x]
    return buf


# --- Indexer ---------------------------------------------------------------------------------

class AbstractIndexer:
    pass


class Indexer(AbstractIndexer):
    """The reference's Indexer (src/utils.jl:288-304), built on the device by
    ``index_``: ``cumulative`` is a ``(U + 1, 2)`` int64 tensor of ``(col, offset)``
    pairs in first-seen order ending with ``(0, n + 1)``; ``map`` holds the gradient
    column (bag, 1-based) of every grouped occurrence.  The Sparse (Dict) and Dense
    (array) flavours give identical results, so both use the same device algorithm."""

    flavour = "sparse"

    def __init__(self):
        self._cumulative = None
        self._map = None
        self._nunique = 0
        self._pending = None  # (indices, maxindex) of a multi-table update!, built on use

    def _defer(self, indices, maxindex: int):
        """The multi-table ``update!`` fills every ``indexers[i]`` in its index phase
        (src/sparseupdate.jl:210-213).  The device update indexes all tables in its own
        fused pipeline, so the reference-layout Indexer is built on first use
        (et_index_build) instead of on every step — from a SNAPSHOT of the index array
        taken by the update's own index phase (et_sparse_sgd_snap: the key pass writes the
        copy as it reads the indices, 8 bytes per occurrence, no separate pass), so a
        caller that refills the index buffer in place before reading ``indexers[i]``
        still gets the Indexer of the indices this update used.  Returns the snapshot
        buffer (contiguous ``(B, P)``) for the update to fill; an unread snapshot's buffer
        is reused by the next update."""
        B = int(indices.shape[0])
        shape = (B,) if indices.dim() == 1 else (B, int(indices.shape[1]))
        old = self._pending[0] if self._pending is not None else None
        if (old is not None and tuple(old.shape) == shape and old.device == indices.device):
            snap = old
        else:
            snap = torch.empty(shape, dtype=torch.int64, device=indices.device)
        self._pending = (snap, int(maxindex))
        return snap

    def _materialise(self):
        if self._pending is not None:
            indices, maxindex = self._pending
            self._pending = None
            index_(self, indices, maxindex)

    @property
    def cumulative(self):
        self._materialise()
        return self._cumulative

    @cumulative.setter
    def cumulative(self, v):
        self._cumulative = v

    @property
    def map(self):
        self._materialise()
        return self._map

    @map.setter
    def map(self, v):
        self._map = v

    @property
    def nunique(self):
        self._materialise()
        return self._nunique

    @nunique.setter
    def nunique(self, v):
        self._nunique = v

    @property
    def histogram(self):
        return None


class SparseIndexer(Indexer):
    flavour = "sparse"


class DenseIndexer(Indexer):
    flavour = "dense"


class IndexerView(AbstractIndexer):
    """A contiguous range of an Indexer's distinct columns (src/utils.jl:320-333)."""

    def __init__(self, I: Indexer, num_splits: int, this_split: int):
        n = I.cumulative.shape[0]  # length(I.cumulative) = U + 1
        split = 1 + (n - 1) // num_splits  # cdiv
        start = (this_split - 1) * split + 1
        stop = min(this_split * split + 1, n)
        self.I = I
        self.range = (start, stop)  # 1-based inclusive view of cumulative

    def entries(self):
        """0-based half-open range of cumulative entries updated through this view."""
        start, stop = self.range
        return start - 1, max(stop - 1, start - 1)


def index_(indexer: Indexer, A: torch.Tensor, maxindex: int) -> Indexer:
    """``index!(indexer, A, maxindex)`` (src/utils.jl:306-314) on the device."""
    _check_idx(A)
    B = int(A.shape[0])
    P = 1 if A.dim() == 1 else int(A.shape[1])
    n = B * P
    dev = A.device
    L = _lib.load()
    nb = ctypes.c_int64(0)
    _lib.check(L.et_index_workspace_size(n, ctypes.byref(nb)))
    ws = _workspace(nb.value, dev, "index")
    cum = torch.empty((2, n + 1), dtype=torch.int64, device=dev)
    mp = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    nu = torch.empty(1, dtype=torch.int64, device=dev)
    _lib.check(L.et_index_build(A.data_ptr(), P, P if A.dim() == 1 else _ld(A), B, int(maxindex),
                                cum[0].data_ptr(), cum[1].data_ptr(), mp.data_ptr(),
                                nu.data_ptr(), ws.data_ptr(), ws.numel(),
                                _lib.stream_handle(dev)))
    U = int(nu.item())
    indexer._pending = None
    indexer.nunique = U
    indexer.cumulative = cum[:, :U + 1].t()
    indexer.map = mp[:n]
    return indexer


def gettranslations(indexer: AbstractIndexer):
    """(cumulative, map) of an Indexer / IndexerView (src/utils.jl:281, :335-338)."""
    if isinstance(indexer, IndexerView):
        b, e = indexer.entries()
        return indexer.I.cumulative[b:e + 1], indexer.I.map
    return indexer.cumulative, indexer.map


# --- update! ------------------------------------------------------------------------------------

_UPDATE_DTYPES = (torch.float32, torch.float64, torch.float16, torch.bfloat16)


def _hot_pass_ok(descs) -> bool:
    """The hot-column pass reads gradients with 16-byte vector loads: every gradient of the
    group must be 16-byte aligned with a leading dimension that is a multiple of 4 (a
    Preallocation gradient with prependrows not a multiple of 4 is not).  The index phase
    plans the pass from the tables alone, so the host drops the flag for such a group
    rather than letting the update phase refuse it."""
    return all(d.delta % 16 == 0 and d.ld_delta % 4 == 0 for d in descs if d.delta)


def _sgd_flags(fused: bool, nontemporal: bool, f64_alpha: bool = False,
               exact: bool | None = False, f16_fp32_acc: bool = False, hot_pass: bool = False):
    flags = _lib.ET_FLAG_NONTEMPORAL if nontemporal else 0
    if hot_pass:
        flags |= _lib.ET_FLAG_SGD_HOT_PASS
    if f16_fp32_acc:
        flags |= _lib.ET_FLAG_F16_FP32_ACC
    if not fused:
        flags |= _lib.ET_FLAG_SGD_UNFUSED
        if f64_alpha:
            flags |= _lib.ET_FLAG_SGD_F64_ALPHA
    if exact is None:  # the bindings' default: exact (the serial-chain path, every dtype)
        flags |= _lib.ET_FLAG_EXACT_IF_FAST
    elif exact:
        flags |= _lib.ET_FLAG_EXACT_UPDATE
    return flags


def _update_desc(table: AbstractEmbeddingTable, grad: SparseEmbeddingUpdate) -> _lib.UpdateDesc:
    I = _check_idx(grad.indices)
    delta = grad.delta
    if table.dtype not in _UPDATE_DTYPES or delta.dtype != table.dtype:
        raise NotImplementedError(
            f"update of a {table.dtype} table with a {delta.dtype} gradient (supported: "
            "Float32 / Float64 / Float16 / BFloat16 tables with gradients of the same type)")
    B = int(I.shape[0])
    P = 1 if I.dim() == 1 else int(I.shape[1])
    D, R = table.size()
    if delta.dim() != 2 or delta.shape[0] != B or delta.shape[1] != D:
        raise ArgumentError(f"gradient shape {tuple(delta.shape)} != ({B}, {D})")
    if delta.numel() > 0 and delta.stride(1) != 1:
        raise ArgumentError("gradient features must be contiguous")
    tp, cpp = table.device_table()
    return _lib.UpdateDesc(tp, table.ld, R, D, P, delta.data_ptr(), _ld(delta),
                           I.data_ptr(), 1 if I.dim() == 1 else _ld(I), B, cpp)


def _sparse_sgd(descs, eta: float, flags: int, device, dtype=torch.float32, snaps=None):
    """One et_sparse_sgd call; `snaps` (one device pointer or None per descriptor) makes it
    et_sparse_sgd_snap, whose key pass copies those tables' index arrays."""
    L = _lib.load()
    n = len(descs)
    arr = (_lib.UpdateDesc * n)(*descs)
    nb = ctypes.c_int64(0)
    _lib.check(L.et_sgd_workspace_size(ctypes.addressof(arr), n, ctypes.byref(nb)))
    ws = _workspace(nb.value, device, "sgd")
    stream = _lib.stream_handle(device)
    if snaps is not None and any(snaps):
        sarr = (ctypes.c_void_p * n)(*snaps)
        _lib.check(L.et_sparse_sgd_snap(_lib.TORCH_TO_ET[dtype], ctypes.addressof(arr), n,
                                        float(eta), flags, ctypes.addressof(sarr), ws.data_ptr(),
                                        ws.numel(), stream))
    else:
        _lib.check(L.et_sparse_sgd(_lib.TORCH_TO_ET[dtype], ctypes.addressof(arr), n, float(eta),
                                   flags, ws.data_ptr(), ws.numel(), stream))


# The exact update (every column's gradient summed serially in the reference's order,
# src/sparseupdate.jl:110-127 — bit-identical) is the default: EXACT_DEFAULT = None passes
# ET_FLAG_EXACT_IF_FAST, which since ABI v9 is exact for every element type and gradient size
# (the serial-chain path: the hand-scheduled Float32 loop, or 64-bit addressed chains for a
# gradient beyond its 32-bit offsets, for a batch of 2^24 bags or more and for Float64 /
# Float16 / BFloat16 tables).  Chains cover batches below 2^27 bags; a larger batch is still
# exact but sums each column in one chunk (one wave per column).
# exact=True is the same; exact=False selects the split mode (columns longer than
# ET_SGD_CHUNK summed as ordered partial sums).
EXACT_DEFAULT = None


def update_(*args, nontemporal: bool | None = None, exact: bool | None = None,
            f16_fp32_acc: bool = False, hot_pass: bool = False, **kw):
    """Julia's ``update!`` (multiple dispatch on the argument types):

    * ``update_(opt::Descent, table, grad, [indexer], [nontemporal])`` — single table,
      index + fused SGD in one device pipeline (src/sparseupdate.jl:160-178);
    * ``update_(opt::Descent, tables, grads, indexers, [nontemporal]; num_splits, nthreads,
      scratchspaces, telemetry_cb)`` — all tables in one pipeline (:199-238);
    * ``update_(table, grad, indexer_or_view, alpha, [nontemporal])`` — update from a
      prebuilt Indexer / IndexerView range (:46-154).

    ``exact=True`` (and the default, EXACT_DEFAULT = None) sums every column's gradient
    serially (bit-identical to the reference even for hot columns: longer columns run as
    serial chains beside the chunk pass, for every element type and gradient size, batches
    below 2^27 bags; a larger batch sums each column in one chunk, exact but slow);
    ``exact=False`` splits occurrence lists longer than ET_SGD_CHUNK (256) into partial
    sums combined in a fixed order (deterministic, not the reference's order).  Float16 tables
    use Julia's Float16 arithmetic unless ``f16_fp32_acc`` (sums in Float32).
    ``hot_pass=True`` (experimental, ET_FLAG_SGD_HOT_PASS) sums the longest occurrence
    lists of Float32 dim-128 tables bag-major (deterministic, not bit-identical to the
    default split)."""
    if exact is None:
        exact = EXACT_DEFAULT
    if args and isinstance(args[0], Descent):
        opt = args[0]
        if isinstance(args[1], AbstractEmbeddingTable):
            table, grad = args[1], args[2]
            nt = args[4] if len(args) > 4 else (True if nontemporal is None else nontemporal)
            indexer = args[3] if len(args) > 3 else kw.get("indexer")
            _update_single(opt, table, grad, nt, exact, f16_fp32_acc, hot_pass, indexer)
            return None
        tables, grads = list(args[1]), list(args[2])
        nt = args[4] if len(args) > 4 else (True if nontemporal is None else nontemporal)
        if len(args) > 3 and args[3] is not None:
            kw["indexers"] = args[3]
        _update_multi(opt, tables, grads, nt, exact, f16_fp32_acc, hot_pass=hot_pass, **kw)
        return None
    table, grad, indexer, alpha = args[:4]
    nt = args[4] if len(args) > 4 else (True if nontemporal is None else nontemporal)
    _update_from_indexer(table, grad, indexer, float(alpha), nt, f16_fp32_acc)
    return None


def _update_single(opt: Descent, table, grad: SparseEmbeddingUpdate, nontemporal: bool,
                   exact: bool, f16_fp32_acc: bool = False, hot_pass: bool = False,
                   indexer=None):
    """src/sparseupdate.jl:159-178: ``index!(indexer, update.indices, size(table, 2))``, then
    the update from it.  The device pipeline indexes on its own; a caller-supplied Indexer is
    filled as the reference's is, from a snapshot of the indices the update's key pass takes
    (et_sparse_sgd_snap), built into the reference layout on first use (Indexer._defer)."""
    if grad.indices.numel() == 0:
        if isinstance(indexer, Indexer):
            indexer._pending = (grad.indices, int(table.size()[1]))
        return
    d = _update_desc(table, grad)
    fused = fused_update_path(table)
    snap = None
    if isinstance(indexer, Indexer):
        snap = indexer._defer(grad.indices, table.size()[1])
    # convert(eltype(table), opt.eta): the library rounds eta to the table type itself
    _sparse_sgd([d], opt.eta, _sgd_flags(fused, nontemporal, False, exact, f16_fp32_acc,
                                         hot_pass),
                table.device, table.dtype, [snap.data_ptr() if snap is not None else None])


def _update_multi(opt: Descent, tables, grads, nontemporal: bool, exact: bool | None,
                  f16_fp32_acc: bool = False, num_splits=4, nthreads=None, scratchspaces=None,
                  telemetry_cb=None, indexers=None, hot_pass: bool = False):
    """src/sparseupdate.jl:199-238: index every table, ``telemetry_cb()``, then update
    every table.  Both phases are one device pipeline per (path, eltype) group of at
    most ET_MAX_TABLES_PER_LAUNCH tables; with a ``telemetry_cb`` they are two calls
    (ET_FLAG_SGD_INDEX_ONLY for every group, the callback on the host once they are
    enqueued — stream order puts it between the phases, as the reference's call between
    its two threaded loops — then ET_FLAG_SGD_APPLY_ONLY from the same workspaces),
    without one a single call per group.  ``indexers[i]`` receives table
    i's Indexer (built from ``grads[i].indices`` on first use — see Indexer._defer).
    ``num_splits`` / ``nthreads`` / ``scratchspaces`` only shape the reference's CPU work
    queue and have no device counterpart."""
    if len(tables) != len(grads):
        raise ArgumentError("tables and grads differ in length")
    if indexers is not None:
        indexers = list(indexers)
        if len(indexers) != len(grads):
            raise ArgumentError("indexers and grads differ in length")
    # Group tables by the reference's per-table path: Static <= 512 B -> specialized
    # (Float32 eta, fused); otherwise generic with the unconverted Float64 eta
    # (src/sparseupdate.jl:232).
    groups: dict = {}
    gsnap: dict = {}
    # indexers[i]: a snapshot of grads[i].indices, written by the update's index phase
    # (by position: one Indexer object may appear at several positions — the reference's
    # sequential index!(indexers[i], ...) leaves it holding the LAST table's indices, so only
    # its last position gets a snapshot; the others pass none)
    snaps = [None] * len(grads)
    if indexers is not None:
        last = {id(ix): i for i, ix in enumerate(indexers) if isinstance(ix, Indexer)}
        for i, (ix, A, g) in enumerate(zip(indexers, tables, grads)):
            if isinstance(ix, Indexer) and last[id(ix)] == i:
                if g.indices.numel() > 0:
                    snaps[i] = ix._defer(g.indices, A.size()[1])
                else:  # nothing to copy: the Indexer of an empty index array
                    ix._pending = (g.indices, int(A.size()[1]))
    for i, (A, g) in enumerate(zip(tables, grads)):
        if g.indices.numel() == 0:
            continue
        key = (fused_update_path(A), A.dtype)
        groups.setdefault(key, []).append(_update_desc(A, g))
        sn = snaps[i]
        gsnap.setdefault(key, []).append(sn.data_ptr() if sn is not None else None)
    calls = []
    if groups:
        dev = tables[0].device
        L = _lib.load()
        stream = _lib.stream_handle(dev)
        for (fused, dtype), descs in groups.items():
            sps = gsnap[(fused, dtype)]
            for c in range(0, len(descs), _lib.ET_MAX_TABLES_PER_LAUNCH):
                part = descs[c:c + _lib.ET_MAX_TABLES_PER_LAUNCH]
                sp = sps[c:c + _lib.ET_MAX_TABLES_PER_LAUNCH]
                flags = _sgd_flags(fused, nontemporal, not fused, exact, f16_fp32_acc,
                                   hot_pass and _hot_pass_ok(part))
                arr = (_lib.UpdateDesc * len(part))(*part)
                sarr = (ctypes.c_void_p * len(part))(*sp) if any(sp) else None
                nb = ctypes.c_int64(0)
                _lib.check(L.et_sgd_workspace_size(ctypes.addressof(arr), len(part),
                                                   ctypes.byref(nb)))
                ws = _workspace(nb.value, dev, f"sgd{len(calls)}")
                calls.append((_lib.TORCH_TO_ET[dtype], arr, len(part), flags, ws, sarr))
        # Without a telemetry callback nothing observes the phase boundary, so each group
        # runs both phases in one call: the same device work in the same stream order
        # (bit-identical), and the exact mode's early chains (small tables, planned from the
        # index arrays) start with the call instead of after every group's index phase.
        phased = telemetry_cb is not None
        for et_t, arr, n, flags, ws, sarr in calls:  # phase 1: index all tables
            f = flags | (_lib.ET_FLAG_SGD_INDEX_ONLY if phased else 0)
            if sarr is None:
                _lib.check(L.et_sparse_sgd(et_t, ctypes.addressof(arr), n, float(opt.eta), f,
                                           ws.data_ptr(), ws.numel(), stream))
            else:
                _lib.check(L.et_sparse_sgd_snap(et_t, ctypes.addressof(arr), n, float(opt.eta),
                                                f, ctypes.addressof(sarr), ws.data_ptr(),
                                                ws.numel(), stream))
    if telemetry_cb is not None:
        telemetry_cb()
        for et_t, arr, n, flags, ws, _ in calls:  # phase 2: update all tables
            _lib.check(L.et_sparse_sgd(et_t, ctypes.addressof(arr), n, float(opt.eta),
                                       flags | _lib.ET_FLAG_SGD_APPLY_ONLY, ws.data_ptr(),
                                       ws.numel(), stream))


def _update_from_indexer(table, grad: SparseEmbeddingUpdate, indexer: AbstractIndexer,
                         alpha: float, nontemporal: bool, f16_fp32_acc: bool = False):
    base = indexer.I if isinstance(indexer, IndexerView) else indexer
    if base.cumulative is None:
        raise ArgumentError("indexer is empty: call index_(indexer, grad.indices, maxindex)")
    if isinstance(indexer, IndexerView):
        b, e = indexer.entries()
    else:
        b, e = 0, base.nunique
    if e <= b:
        return
    delta = grad.delta
    if table.dtype not in _UPDATE_DTYPES or delta.dtype != table.dtype:
        raise NotImplementedError(f"update of a {table.dtype} table with a {delta.dtype} gradient")
    D, R = table.size()
    cum = base.cumulative  # (U+1, 2) view of the (2, n+1) buffer
    fused = fused_update_path(table)
    tp, cpp = table.device_table()
    _lib.check(_lib.load().et_update_indexed(
        _lib.TORCH_TO_ET[table.dtype], tp, table.ld, cpp, R, D, delta.data_ptr(), _ld(delta),
        cum[:, 0].data_ptr(), cum[:, 1].data_ptr(), b, e, base.map.data_ptr(), alpha,
        _sgd_flags(fused, nontemporal, f16_fp32_acc=f16_fp32_acc),
        _lib.stream_handle(table.device)))


class PhasedUpdate:
    """The multi-table ``update!(opt, tables, grads, indexers)`` split at the reference's
    own phase boundary (src/sparseupdate.jl:210-213 "index all", then :216-237 "update
    all"), so the index phase can run while the gradient is still being produced.

    ``index_(stream)`` reads only the index arrays (keys, sort, segments, chunk
    records into this object's own workspaces); ``update_(opt, stream)`` waits for it
    and sums the gradient columns and updates the tables.  The gradients' ``delta``
    tensors are bound at construction (their storage, not their values): fill them
    before ``update_``.  Results are bit-identical to ``update_(opt, tables, grads,
    indexers)`` with the same ``exact`` / ``nontemporal`` / ``f16_fp32_acc``."""

    def __init__(self, tables, grads, *, nontemporal: bool = True, exact: bool | None = None,
                 f16_fp32_acc: bool = False, hot_pass: bool = False):
        if exact is None:
            exact = EXACT_DEFAULT
        tables, grads = list(tables), list(grads)
        if len(tables) != len(grads):
            raise ArgumentError("tables and grads differ in length")
        groups: dict = {}
        for A, g in zip(tables, grads):
            if g.indices.numel() == 0:
                continue
            groups.setdefault((fused_update_path(A), A.dtype), []).append(_update_desc(A, g))
        self.device = tables[0].device if tables else None
        self._keep = (tables, grads)  # the descriptors point into these
        self._calls = []  # (dtype, desc array, n, flags, workspace)
        L = _lib.load()
        for (fused, dtype), descs in groups.items():
            for c in range(0, len(descs), _lib.ET_MAX_TABLES_PER_LAUNCH):
                part = descs[c:c + _lib.ET_MAX_TABLES_PER_LAUNCH]
                flags = _sgd_flags(fused, nontemporal, not fused, exact, f16_fp32_acc,
                                   hot_pass and _hot_pass_ok(part))
                arr = (_lib.UpdateDesc * len(part))(*part)
                nb = ctypes.c_int64(0)
                _lib.check(L.et_sgd_workspace_size(ctypes.addressof(arr), len(part),
                                                   ctypes.byref(nb)))
                ws = torch.empty(max(int(nb.value), 256), dtype=torch.uint8, device=self.device)
                self._calls.append((dtype, arr, len(part), flags, ws))
        self._indexed = None

    def _run(self, eta: float, phase: int, stream):
        L = _lib.load()
        h = stream.cuda_stream
        for dtype, arr, n, flags, ws in self._calls:
            _lib.check(L.et_sparse_sgd(_lib.TORCH_TO_ET[dtype], ctypes.addressof(arr), n,
                                       float(eta), flags | phase, ws.data_ptr(), ws.numel(), h))

    def index_(self, stream=None):
        """Phase 1 on ``stream`` (default: the current stream)."""
        if self.device is None:
            return self
        stream = stream or torch.cuda.current_stream(self.device)
        self._run(0.0, _lib.ET_FLAG_SGD_INDEX_ONLY, stream)
        self._indexed = torch.cuda.Event()
        self._indexed.record(stream)
        return self

    def update_(self, opt: Descent, stream=None):
        """Phase 2 on ``stream`` (default: the current stream), ordered after the last
        ``index_``.  May be repeated (same indices, new gradient values)."""
        if self.device is None:
            return None
        if self._indexed is None:
            raise ArgumentError("PhasedUpdate.update_ before index_")
        stream = stream or torch.cuda.current_stream(self.device)
        stream.wait_event(self._indexed)
        self._run(opt.eta, _lib.ET_FLAG_SGD_APPLY_ONLY, stream)
        return None


def optimise_update_(opt, x, xbar: SparseEmbeddingUpdate, indexer=None, nontemporal=True):
    """``Flux.Optimise.update!(opt, x, xbar::SparseEmbeddingUpdate, ...)``
    (src/sparseupdate.jl:180-189)."""
    return update_(opt, x, xbar, indexer, nontemporal)


def ensemble_update(nthreads: int):
    """src/sparseupdate.jl:195."""
    return [Indexer() for _ in range(nthreads)]
