"""Sharding a PreallocationStrategy maplookup across the GPUs of a node.

No counterpart exists in the single-process reference.  Tables
are independent, and so is every feature of a table (a pooled sum is computed
feature by feature, src/lookup.jl:134-147), so a rank can own any set of
*pieces* — a table, or a contiguous feature range of one — look them up for the
batch with ONE fused launch per feature-width group into a local slab, and the
concat of the reference's PreallocationStrategy (src/lookup.jl:334-340) becomes
an RCCL exchange of the slabs over xGMI plus one assembly kernel
(et_concat_slabs) into the destination.

Plans:
  * ``ShardPlan.tablewise``: whole tables, balanced by count (4,4,3,3,3,3,3,3 for
    26 tables on 8 GPUs);
  * ``ShardPlan.featurewise``: the concatenated feature axis cut into equal
    contiguous ranges at ``granule``-feature boundaries (26 x 128 = 3328 features
    -> 416 per GPU at N = 8): equal slabs (no all-gather padding) and equal
    lookup bytes per rank.  Results are bit-identical to the unsharded lookup.

Exchanges:
  * ``"allgather"`` (the contract, BASELINE config 5): every rank ends with the
    whole ``(B, k + sum D)`` destination; the batch is cut into ``chunks`` so the
    lookup of chunk c+1 overlaps the all-gather + assembly of chunk c on a second
    stream;
  * ``"alltoall"`` (the DLRM layout): rank r ends with rows
    ``[r*B/N, (r+1)*B/N)`` of the destination — N times less data on the links.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from .lookup import _ld

VEC_DIMS = (512, 256, 128, 64, 32, 16)  # the vector kernels' feature widths


@dataclass(frozen=True)
class Piece:
    """Features ``[f0, f0 + dim)`` of global table ``table``; its columns of the
    destination start at ``col`` (prependrows included)."""

    table: int
    f0: int
    dim: int
    col: int


def native_plan(mode: int, dims, world: int, prependrows: int = 0, sizes=None,
                granule: int = 32, elsize: int = 4) -> list[list[Piece]]:
    """et_shard_plan (host-only C++ in the library): every rank's pieces, in slab order."""
    if world <= 0:
        raise ValueError("world must be positive")
    L = _lib.load()
    n = len(dims)
    d = (ctypes.c_int32 * max(1, n))(*dims)
    sz = (ctypes.c_int64 * max(1, n))(*sizes) if sizes is not None else None
    cnt = ctypes.c_int32(0)
    args = (mode, n, ctypes.addressof(d), ctypes.addressof(sz) if sz is not None else None,
            world, prependrows, granule, elsize)
    _lib.check(L.et_shard_plan(*args, None, 0, ctypes.byref(cnt)))
    out = (_lib.ShardPiece * max(1, cnt.value))()
    _lib.check(L.et_shard_plan(*args, ctypes.addressof(out), cnt.value, ctypes.byref(cnt)))
    pieces = [[] for _ in range(world)]
    for i in range(cnt.value):
        p = out[i]
        pieces[p.rank].append(Piece(p.table, p.f0, p.dim, p.col))
    return pieces


def plan_tables(ntables: int, world: int, sizes=None) -> list[list[int]]:
    """Whole tables over ranks balanced by COUNT (every table costs B*P*D*4 bytes per
    lookup whatever its cardinality), contiguous groups, the largest tables spread
    over distinct ranks when ``sizes`` is given (26 tables on 8 GPUs
    -> 4,4,3,3,3,3,3,3).  Thin view of et_shard_plan(ET_PLAN_TABLEWISE)."""
    pieces = native_plan(_lib.ET_PLAN_TABLEWISE, [1] * ntables, world, sizes=sizes)
    return [[p.table for p in ps] for ps in pieces]


def plan_features(dims, world: int, granule: int = 32) -> list[tuple[int, int]]:
    """Feature ranges ``[lo, hi)`` of the concatenated feature axis, one per rank (cut
    points: table edges or multiples of ``granule`` inside a table, each nearest to an
    equal split).  Thin view of et_shard_plan(ET_PLAN_FEATUREWISE)."""
    pieces = native_plan(_lib.ET_PLAN_FEATUREWISE, dims, world, granule=granule)
    out, lo = [], 0
    for ps in pieces:
        hi = max((p.col + p.dim for p in ps), default=lo)
        out.append((lo, hi))
        lo = hi
    return out


class ShardPlan:
    """Which pieces every rank looks up, and where its slab lands in the destination."""

    def __init__(self, dims, prependrows: int, pieces: list[list[Piece]]):
        self.dims = list(dims)
        self.prependrows = prependrows
        self.pieces = pieces
        self.world = len(pieces)
        self.ld = prependrows + sum(self.dims)
        self.widths = [sum(p.dim for p in ps) for ps in pieces]
        # equal slabs for the collective; a multiple of 4 elements keeps 16-B stores aligned
        self.slab_ld = max(4, (max(self.widths) + 3) // 4 * 4)

    @classmethod
    def tablewise(cls, dims, world: int, prependrows: int = 0, sizes=None) -> "ShardPlan":
        return cls(dims, prependrows, native_plan(_lib.ET_PLAN_TABLEWISE, dims, world,
                                                  prependrows, sizes))

    @classmethod
    def featurewise(cls, dims, world: int, prependrows: int = 0,
                    granule: int = 32, elsize: int = 4) -> "ShardPlan":
        return cls(dims, prependrows, native_plan(_lib.ET_PLAN_FEATUREWISE, dims, world,
                                                  prependrows, None, granule, elsize))

    def tables_of(self, rank: int) -> list[int]:
        """Global ids of the tables rank ``rank`` reads (each once, in order)."""
        seen = []
        for p in self.pieces[rank]:
            if p.table not in seen:
                seen.append(p.table)
        return seen

    def runs(self, rank: int):
        """Contiguous ``(slab_col, dst_col, ncols)`` runs of a rank's slab."""
        runs, s = [], 0
        for p in self.pieces[rank]:
            if runs and runs[-1][0] + runs[-1][2] == s and runs[-1][1] + runs[-1][2] == p.col:
                runs[-1] = (runs[-1][0], runs[-1][1], runs[-1][2] + p.dim)
            else:
                runs.append((s, p.col, p.dim))
            s += p.dim
        return runs

    def assembly_launches(self):
        """The et_concat_slabs launches that assemble the destination from the
        gathered slabs: ``(slab_col_shift, ncols[rank], dst_col[rank])`` — one launch
        when every rank's pieces are one contiguous run (featurewise, or tablewise
        without ``sizes``)."""
        all_runs = [self.runs(r) for r in range(self.world)]
        launches = []
        for k in range(max((len(x) for x in all_runs), default=0)):
            per = {}
            for r in range(self.world):
                if k < len(all_runs[r]):
                    s, d, n = all_runs[r][k]
                    rows, offs = per.setdefault(s, ([0] * self.world, [0] * self.world))
                    rows[r], offs[r] = n, d
            for shift in sorted(per):
                launches.append((shift, per[shift][0], per[shift][1]))
        return launches


def piece_table(full, piece: Piece):
    """A rank's view of ``piece`` of a full table (a SimpleEmbedding on a column
    slice; whole-table pieces return the table itself).  The view keeps the
    reference's update dispatch of the parent (fused iff the parent is)."""
    from .tables import Dynamic, SimpleEmbedding, Static, fused_update_path

    D = full.size()[0]
    if piece.f0 == 0 and piece.dim == D:
        return full
    if not isinstance(full, SimpleEmbedding):
        raise NotImplementedError("feature-sharding needs SimpleEmbedding tables")
    view = full.data[:, piece.f0:piece.f0 + piece.dim]
    return SimpleEmbedding(view, Static(piece.dim) if fused_update_path(full) else Dynamic)


def compact_piece_table(full, piece: Piece):
    """``piece`` of a full table as its OWN compact ``(R, dim)`` table (ld = dim): a rank
    that owns a feature slice stores only that slice (feature-wise plans).  Whole-table
    pieces return the table itself.  Same update dispatch as the parent."""
    from .tables import Dynamic, SimpleEmbedding, Static, fused_update_path

    D = full.size()[0]
    if piece.f0 == 0 and piece.dim == D:
        return full
    if not isinstance(full, SimpleEmbedding):
        raise NotImplementedError("feature-sharding needs SimpleEmbedding tables")
    data = full.data[:, piece.f0:piece.f0 + piece.dim].contiguous()
    return SimpleEmbedding(data, Static(piece.dim) if fused_update_path(full) else Dynamic)


class ShardedMapLookup:
    """``maplookup!(PreallocationStrategy(k), dst, tables, I)`` over the ranks of
    ``group`` (RCCL on ROCm; gloo for CPU rehearsal).

    ``piece_tables`` / ``piece_idx`` are this rank's pieces (``piece_table``) and
    their index arrays, in ``plan.pieces[rank]`` order."""

    def __init__(self, plan: ShardPlan, rank: int, world: int, batch: int, dtype, device,
                 group=None, exchange: str = "allgather", chunks: int = 1, native=None,
                 rccl=None, comm=None):
        if plan.world != world:
            raise ValueError("plan and world size differ")
        if exchange not in ("allgather", "alltoall", "p2p"):
            raise ValueError(f"unknown exchange {exchange!r}")
        self.plan, self.rank, self.world, self.batch = plan, rank, world, batch
        self.device, self.group, self.exchange_kind = torch.device(device), group, exchange
        self.chunks = max(1, min(chunks, batch)) if exchange != "alltoall" else 1
        self.dtype = dtype
        self._native = None
        auto = native is None
        if comm is not None:  # a caller-owned communicator (e.g. a loopback rank)
            if exchange == "p2p":
                raise ValueError("exchange='p2p' has no native step: comm= applies to the "
                                 "'allgather' and 'alltoall' exchanges only")
            native, auto = True, False
        if auto:  # the C-ABI step whenever the ranks are real GPU processes
            native = (exchange != "p2p" and self.device.type == "cuda" and
                      (world == 1 or self._nccl_group()))
        if native:
            err = None
            try:
                self._native = NativeShardedStep(plan, rank, world, batch, dtype, self.device,
                                                 group, exchange, self.chunks,
                                                 rccl=world > 1 if rccl is None else rccl,
                                                 comm=comm)
            except _lib.EmbtabError as e:
                if not auto:
                    raise
                err = e
            if auto and world > 1 and not self._all_ranks_ok(err is None):
                # every rank takes the same exchange: if any rank could not make the
                # library's communicator, all of them close theirs and use the
                # torch.distributed exchange (same plan, same kernels, same results)
                if self._native is not None:
                    self._native.close()
                    self._native = None
                if err is None:
                    err = _lib.EmbtabError("another rank could not make the RCCL communicator")
            if err is not None:
                import warnings

                warnings.warn(f"native sharded step unavailable ({err}); using the "
                              "torch.distributed exchange")
                self._native = None
        if self._native is not None:
            self.launches = plan.assembly_launches()
            nat = self._native
            # the slab is the head of the native workspace (for lookup-only timing)
            es = torch.empty((), dtype=dtype).element_size()
            self.slab = nat.workspace[:batch * nat.slab_ld * es].view(dtype).view(
                batch, nat.slab_ld)
            self.bounds = [batch * c // self.chunks for c in range(self.chunks + 1)]
            self.split = [batch * j // world for j in range(world + 1)]
            self.mine = self.split[rank + 1] - self.split[rank]
            self._plans = {}
            return
        ld = plan.slab_ld
        self.slab = (torch.zeros((batch, ld), dtype=dtype, device=device)
                     if exchange != "p2p" else None)
        self._plans = {}  # lookup_chunk descriptor cache
        # chunk c covers batch rows [bounds[c], bounds[c+1])
        self.bounds = [batch * c // self.chunks for c in range(self.chunks + 1)]
        if exchange == "allgather":
            self.gathered = [torch.empty((world, self.bounds[c + 1] - self.bounds[c], ld),
                                         dtype=dtype, device=device)
                             for c in range(self.chunks)]
        elif exchange == "p2p":
            # every rank's whole destination, mapped into every other rank (et_ipc_open);
            # this rank's lookups write its own columns in place and et_push_cols stores
            # them into the peers' copies: no slab, no gathered buffer, no assembly
            self.out = torch.zeros((batch, plan.ld), dtype=dtype, device=device)
            self._peers, self._peer_offs = self._open_peers()
            self._flag = torch.zeros(1, dtype=torch.int32, device=device)
            self._groups = self._run_groups()
        else:
            # rank j receives batch rows [split[j], split[j+1]) from every rank
            self.split = [batch * j // world for j in range(world + 1)]
            self.mine = self.split[rank + 1] - self.split[rank]
            self.gathered = [torch.empty((world, self.mine, ld), dtype=dtype, device=device)]
        self.launches = plan.assembly_launches()
        self._comm = (torch.cuda.Stream(self.device) if self.device.type == "cuda"
                      and (self.chunks > 1 or exchange == "p2p") else None)
        self._events = []

    # --- device work (overridable so that the CPU rehearsal can stand in the oracle) ---
    def lookup_chunk(self, piece_tables, piece_idx, b0: int, b1: int):
        """One fused launch per width group: this rank's pieces, bags [b0, b1) -> slab."""
        from .lookup import PreallocationPlan, PreallocationStrategy

        if not piece_tables:
            return
        # descriptor arrays cached per (chunk, tables, index buffers): a training loop
        # that refills the same index buffers pays one library call per chunk
        key = (b0, b1, tuple((id(t), t.device_table()) for t in piece_tables),
               tuple((i.data_ptr(), tuple(i.shape), tuple(i.stride())) for i in piece_idx))
        plan = self._plans.get(key)
        if plan is None:
            if len(self._plans) >= 64:
                self._plans.clear()
            plan = PreallocationPlan(PreallocationStrategy(0), self.slab[b0:b1], piece_tables,
                                     [i[b0:b1] for i in piece_idx])
            self._plans[key] = plan
        plan()

    def assemble_chunk(self, gathered: torch.Tensor, dst: torch.Tensor):
        """et_concat_slabs: every rank's slab columns into their destination columns."""
        L = _lib.load()
        nb = gathered.shape[1]
        for shift, rows, offs in self.launches:
            rr = (ctypes.c_int32 * self.world)(*rows)
            oo = (ctypes.c_int64 * self.world)(*offs)
            base = gathered.data_ptr() + shift * gathered.element_size()
            _lib.check(L.et_concat_slabs(
                _lib.et_dtype(dst), base, self.world, self.plan.slab_ld, nb,
                ctypes.addressof(rr), ctypes.addressof(oo), dst.data_ptr(), _ld(dst),
                _lib.stream_handle(dst.device)))

    # --- one-sided exchange (exchange="p2p") --------------------------------------------
    def _run_groups(self):
        """``(dst_col, ncols, [piece positions])`` per contiguous run of this rank's pieces."""
        groups, pos = [], 0
        for _, dcol, n in self.plan.runs(self.rank):
            members, width = [], 0
            while width < n:
                members.append(pos)
                width += self.plan.pieces[self.rank][pos].dim
                pos += 1
            groups.append((dcol, n, members))
        return groups

    def _open_peers(self):
        """IPC-map every other rank's ``out`` (handles exchanged over the group)."""
        import torch.distributed as dist

        if self.world == 1:
            return [], []
        L = _lib.load()
        handle = (ctypes.c_char * 64)()
        off = ctypes.c_int64()
        _lib.check(L.et_ipc_handle(self.out.data_ptr(), ctypes.addressof(handle),
                                   ctypes.byref(off)))
        mine = (bytes(handle), off.value)
        every = [None] * self.world
        dist.all_gather_object(every, mine, group=self.group)
        peers, offs = [], []
        for r, (h, o) in enumerate(every):
            if r == self.rank:
                continue
            hb = (ctypes.c_char * 64).from_buffer_copy(h)
            ptr = ctypes.c_void_p()
            _lib.check(L.et_ipc_open(ctypes.addressof(hb), o, ctypes.byref(ptr)))
            peers.append(ptr.value)
            offs.append(o)
        return peers, offs

    def close(self):
        """Release the native step (stream, events, RCCL communicator) or unmap the peers'
        destinations (p2p exchange)."""
        if self._native is not None:
            self._native.close()
        if getattr(self, "_peers", None):
            L = _lib.load()
            for p, o in zip(self._peers, self._peer_offs):
                _lib.check(L.et_ipc_close(p, o))
            self._peers, self._peer_offs = [], []

    def _p2p_barrier(self):
        """Stream-ordered rendezvous: returns on the current stream once every rank's
        work queued before it has finished (its pushes, or its use of ``out``)."""
        import torch.distributed as dist

        if self.world == 1:
            return
        if self._gloo():  # ranks sharing one GPU in rehearsal: host-side barrier
            torch.cuda.current_stream(self.device).synchronize()
            dist.barrier(group=self.group)
        else:
            dist.all_reduce(self._flag, op=dist.ReduceOp.MAX, group=self.group)

    def push_chunk(self, b0: int, b1: int):
        """et_push_cols: this rank's columns of bags [b0, b1) into every peer's ``out``."""
        if not self._peers:
            return
        L = _lib.load()
        out = self.out[b0:b1]
        shift = b0 * _ld(self.out) * out.element_size()  # the chunk's first bag, in every copy
        shifted = (ctypes.c_void_p * len(self._peers))(*[p + shift for p in self._peers])
        for dcol, n, _ in self._groups:
            _lib.check(L.et_push_cols(
                _lib.et_dtype(out), out.data_ptr(), _ld(self.out), b1 - b0, dcol, n,
                ctypes.addressof(shifted), len(self._peers), _lib.stream_handle(out.device)))

    def _lookup_p2p(self, piece_tables, piece_idx, b0: int, b1: int):
        """This rank's lookups for bags [b0, b1), written in place into ``out``."""
        from .lookup import PreallocationPlan, PreallocationStrategy

        for gi, (dcol, n, members) in enumerate(self._groups):
            tabs = [piece_tables[m] for m in members]
            idx = [piece_idx[m] for m in members]
            key = (gi, b0, b1, tuple((id(t), t.device_table()) for t in tabs),
                   tuple((i.data_ptr(), tuple(i.shape), tuple(i.stride())) for i in idx))
            plan = self._plans.get(key)
            if plan is None:
                if len(self._plans) >= 64:
                    self._plans.clear()
                plan = PreallocationPlan(PreallocationStrategy(0), self.out[b0:b1, dcol:dcol + n],
                                         tabs, [i[b0:b1] for i in idx])
                self._plans[key] = plan
            plan()

    def _call_p2p(self, piece_tables, piece_idx, dst):
        if dst is not None and dst.data_ptr() != self.out.data_ptr():
            raise ValueError("the p2p exchange writes into ShardedMapLookup.out (pass it, or None)")
        main = torch.cuda.current_stream(self.device)
        # the peers must be done with the previous step's `out` before pushes land in it:
        # that barrier runs on the exchange stream, beside the first chunk's lookups
        self._comm.wait_stream(main)
        with torch.cuda.stream(self._comm):
            self._p2p_barrier()
        for c in range(self.chunks):
            b0, b1 = self.bounds[c], self.bounds[c + 1]
            self._lookup_p2p(piece_tables, piece_idx, b0, b1)
            ev = torch.cuda.Event()
            ev.record(main)
            self._comm.wait_event(ev)
            with torch.cuda.stream(self._comm):
                self.push_chunk(b0, b1)
        main.wait_stream(self._comm)
        self._p2p_barrier()  # every peer's pushes into this rank's `out` have landed
        return self.out

    # --- the exchange -------------------------------------------------------------------
    def _all_ranks_ok(self, ok: bool) -> bool:
        """MIN over the ranks of `ok` (a collective of the process group)."""
        import torch.distributed as dist

        dev = self.device if self._nccl_group() else torch.device("cpu")
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        return bool(flag.item())

    def _nccl_group(self) -> bool:
        import torch.distributed as dist

        return dist.is_available() and dist.is_initialized() and \
            dist.get_backend(self.group) == "nccl"

    def _gloo(self) -> bool:
        import torch.distributed as dist

        return dist.get_backend(self.group) == "gloo"

    def _all_gather(self, out: torch.Tensor, inp: torch.Tensor):
        import torch.distributed as dist

        if self.world == 1:
            out[0].copy_(inp)
        elif self._gloo():
            # CPU rehearsal (gloo has no all_gather_into_tensor; device tensors are
            # staged through the host so that several ranks can share one GPU)
            host = torch.empty(out.shape, dtype=out.dtype)
            dist.all_gather(list(host.unbind(0)), inp.cpu().contiguous(), group=self.group)
            out.copy_(host)
        else:
            dist.all_gather_into_tensor(out.view(-1), inp.reshape(-1), group=self.group)

    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor):
        import torch.distributed as dist

        if self.world == 1:
            out[0].copy_(inp)
            return
        sizes_in = [(self.split[j + 1] - self.split[j]) * self.plan.slab_ld
                    for j in range(self.world)]
        sizes_out = [self.mine * self.plan.slab_ld] * self.world
        if self._gloo():
            host = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(host.view(-1), inp.cpu().reshape(-1), sizes_out, sizes_in,
                                   group=self.group)
            out.copy_(host)
        else:
            dist.all_to_all_single(out.view(-1), inp.reshape(-1), output_split_sizes=sizes_out,
                                   input_split_sizes=sizes_in, group=self.group)

    def __call__(self, piece_tables, piece_idx, dst: torch.Tensor) -> torch.Tensor:
        """Run the sharded step; ``dst`` is ``(B, k + sum D)`` (allgather) or this
        rank's ``(B_r, k + sum D)`` batch slice (alltoall); p2p returns ``self.out``."""
        if self._native is not None:
            return self._native(piece_tables, piece_idx, dst)
        if self.exchange_kind == "p2p":
            return self._call_p2p(piece_tables, piece_idx, dst)
        if self.exchange_kind == "alltoall":
            self.lookup_chunk(piece_tables, piece_idx, 0, self.batch)
            self._all_to_all(self.gathered[0], self.slab)
            self.assemble_chunk(self.gathered[0], dst)
            return dst
        if self._comm is None:
            for c in range(self.chunks):
                b0, b1 = self.bounds[c], self.bounds[c + 1]
                self.lookup_chunk(piece_tables, piece_idx, b0, b1)
                self._all_gather(self.gathered[c], self.slab[b0:b1])
                self.assemble_chunk(self.gathered[c], dst[b0:b1])
            return dst
        # pipelined: lookups on the caller's stream, exchange + assembly on _comm
        main = torch.cuda.current_stream(self.device)
        self._comm.wait_stream(main)  # dst / slab reuse across steps
        for c in range(self.chunks):
            b0, b1 = self.bounds[c], self.bounds[c + 1]
            self.lookup_chunk(piece_tables, piece_idx, b0, b1)
            ev = torch.cuda.Event()
            ev.record(main)
            self._comm.wait_event(ev)
            with torch.cuda.stream(self._comm):
                self._all_gather(self.gathered[c], self.slab[b0:b1])
                self.assemble_chunk(self.gathered[c], dst[b0:b1])
        main.wait_stream(self._comm)
        return dst


    # --- backward: the gradients of this rank's pieces --------------------------------
    def split_rows(self, delta_local: torch.Tensor, send: torch.Tensor):
        """et_split_slabs: the columns of every rank's pieces out of this rank's batch
        slice of the gradient, into ``send[rank]`` (the inverse of assemble_chunk)."""
        L = _lib.load()
        nb = delta_local.shape[0]
        for shift, rows, offs in self.launches:
            rr = (ctypes.c_int32 * self.world)(*rows)
            oo = (ctypes.c_int64 * self.world)(*offs)
            base = send.data_ptr() + shift * send.element_size()
            _lib.check(L.et_split_slabs(
                _lib.et_dtype(delta_local), delta_local.data_ptr(), _ld(delta_local), nb,
                self.world, ctypes.addressof(rr), ctypes.addressof(oo), base, self.plan.slab_ld,
                _lib.stream_handle(delta_local.device)))

    def piece_grads(self, piece_tables, piece_idx, delta: torch.Tensor):
        """The SparseEmbeddingUpdate of each of this rank's pieces (rrule of the sharded
        maplookup, src/lookup.jl:374-389 with the intended Slicer advance).

        All-gather layout: ``delta`` is the whole ``(B, k + sum D)`` gradient, present on
        every rank, and a piece's gradient is a column view of it (no communication).
        All-to-all layout: ``delta`` is this rank's ``(B_r, k + sum D)`` batch slice; the
        columns of every rank's pieces are cut out (et_split_slabs) and exchanged with
        one all-to-all, giving the ``(B, slab)`` gradient of this rank's features.
        The update itself is then purely local: ``update_(opt, piece_tables, grads, ...)``.
        """
        from .update import SparseEmbeddingUpdate

        ps = self.plan.pieces[self.rank]
        if self._native is not None and self.exchange_kind == "alltoall":
            recv = self._native.piece_grads(delta)
            views, s = [], 0
            for p in ps:
                views.append(recv[:, s:s + p.dim])
                s += p.dim
        elif self.exchange_kind in ("allgather", "p2p"):
            views = [delta[:, p.col:p.col + p.dim] for p in ps]
        else:
            import torch.distributed as dist

            ld = self.plan.slab_ld
            send = torch.zeros((self.world, self.mine, ld), dtype=delta.dtype, device=delta.device)
            self.split_rows(delta, send)
            recv = torch.empty((self.batch, ld), dtype=delta.dtype, device=delta.device)
            sizes_out = [(self.split[j + 1] - self.split[j]) * ld for j in range(self.world)]
            sizes_in = [self.mine * ld] * self.world
            if self.world == 1:
                recv.copy_(send[0])
            elif self._gloo():
                host = torch.empty(recv.shape, dtype=recv.dtype)
                dist.all_to_all_single(host.view(-1), send.cpu().reshape(-1), sizes_out,
                                       sizes_in, group=self.group)
                recv.copy_(host)
            else:
                dist.all_to_all_single(recv.view(-1), send.view(-1), output_split_sizes=sizes_out,
                                       input_split_sizes=sizes_in, group=self.group)
            views, s = [], 0
            for p in ps:
                views.append(recv[:, s:s + p.dim])
                s += p.dim
        return [SparseEmbeddingUpdate(t.lookup_type, v, i)
                for t, v, i in zip(piece_tables, views, piece_idx)]


class NativeShardedStep:
    """The sharded step through the C ABI (et_sharded_create / et_sharded_maplookup /
    et_sharded_piece_grads, csrc/et_shard.cpp): plan, pipelined lookup -> RCCL exchange ->
    assembly, all native; Python only hands over pointers.  The RCCL communicator is made
    with et_comm_unique_id / et_comm_init, the id broadcast over ``group``."""

    def __init__(self, plan: ShardPlan, rank: int, world: int, batch: int, dtype, device,
                 group=None, exchange: str = "allgather", chunks: int = 1, rccl: bool = True,
                 comm=None):
        self.plan, self.rank, self.world, self.batch = plan, rank, world, batch
        self.device, self.exchange = device, exchange
        self.L = L = _lib.load()
        self._et_dtype = _lib.TORCH_TO_ET[dtype]
        self.comm = ctypes.c_void_p(None)  # owned by this object (made here), else:
        self._ext_comm = comm              # a caller-owned communicator, never destroyed here
        self.h = None
        with torch.cuda.device(device):
            if comm is None and rccl:
                self.comm = make_comm(group, rank, world)
            try:
                flat = [p for r in range(world) for p in plan.pieces[r]]
                arr = (_lib.ShardPiece * max(1, len(flat)))()
                for i, (r, p) in enumerate((r, p) for r in range(world) for p in plan.pieces[r]):
                    arr[i] = _lib.ShardPiece(r, p.table, p.f0, p.dim, p.col)
                h = ctypes.c_void_p()
                kind = (_lib.ET_EXCHANGE_ALLTOALL if exchange == "alltoall"
                        else _lib.ET_EXCHANGE_ALLGATHER)
                _lib.check(L.et_sharded_create(ctypes.byref(h), comm if comm is not None
                                               else self.comm, world, rank, self._et_dtype,
                                               ctypes.addressof(arr), len(flat),
                                               plan.prependrows, plan.ld, batch, chunks, kind))
                self.h = h
                ld, ws, lo, hi = (ctypes.c_int64() for _ in range(4))
                _lib.check(L.et_sharded_info(h, ctypes.byref(ld), ctypes.byref(ws),
                                             ctypes.byref(lo), ctypes.byref(hi)))
                self.slab_ld, self.lo, self.hi = ld.value, lo.value, hi.value
                self.workspace = torch.empty(ws.value, dtype=torch.uint8, device=device)
            except BaseException:
                # never leak the communicator (or the handle) of a half-made step
                self.close()
                raise
        self._descs = {}

    def _local_descs(self, piece_tables, piece_idx):
        key = (tuple((id(t), t.device_table()) for t in piece_tables),
               tuple((i.data_ptr(), tuple(i.shape), tuple(i.stride())) for i in piece_idx))
        hit = self._descs.get(key)
        if hit is not None:
            return hit
        from .lookup import _check_idx, _check_table, _ld

        n = len(piece_tables)
        descs = (_lib.LookupDesc * max(1, n))()
        for j, (A, i) in enumerate(zip(piece_tables, piece_idx)):
            _check_table(A)
            _check_idx(i)
            D, R = A.size()
            table, cpp = A.device_table()
            pool = 1 if i.dim() == 1 else int(i.shape[1])
            descs[j] = _lib.LookupDesc(table, A.ld, R, D, pool, i.data_ptr(),
                                       1 if i.dim() == 1 else _ld(i), 0, cpp)
        if len(self._descs) >= 64:
            self._descs.clear()
        self._descs[key] = (descs, n, (piece_tables, piece_idx))
        return self._descs[key]

    def __call__(self, piece_tables, piece_idx, dst):
        descs, n, _ = self._local_descs(piece_tables, piece_idx)
        _lib.check(self.L.et_sharded_maplookup(
            self.h, ctypes.addressof(descs), n, dst.data_ptr(), _ld(dst),
            self.workspace.data_ptr(), self.workspace.numel(), _lib.ET_FLAG_NONTEMPORAL,
            _lib.stream_handle(dst.device)))
        return dst

    def piece_grads(self, delta):
        recv = torch.empty((self.batch, self.slab_ld), dtype=delta.dtype, device=delta.device)
        _lib.check(self.L.et_sharded_piece_grads(
            self.h, delta.data_ptr(), _ld(delta), recv.data_ptr(), self.workspace.data_ptr(),
            self.workspace.numel(), _lib.stream_handle(delta.device)))
        return recv

    def close(self):
        if getattr(self, "h", None):
            _lib.check(self.L.et_sharded_destroy(self.h))
            self.h = None
        if self.comm:
            _lib.check(self.L.et_comm_destroy(self.comm))
            self.comm = ctypes.c_void_p(None)


def loopback_comms(world: int) -> list:
    """et_comm_loopback: ``world`` simulated ranks of this process (rank r = item r), all
    on the current device, for running the world > 1 native step without ``world`` GPUs:
    drive each rank from its own host thread and stream (ctypes releases the GIL during
    the calls, so the ranks' collectives rendezvous inside the library).  Free each with
    ``_lib.load().et_comm_destroy``."""
    L = _lib.load()
    arr = (ctypes.c_void_p * world)()
    _lib.check(L.et_comm_loopback(ctypes.addressof(arr), world))
    return [ctypes.c_void_p(arr[r]) for r in range(world)]


def make_comm(group, rank: int, world: int) -> ctypes.c_void_p:
    """An RCCL communicator over the ranks of ``group`` through the C ABI: rank 0's
    et_comm_unique_id, broadcast by torch.distributed, then et_comm_init on every rank
    (on the current device).  World 1 needs no broadcast."""
    L = _lib.load()
    idbuf = (ctypes.c_char * _lib.ET_COMM_ID_BYTES)()
    err = None
    if rank == 0:
        try:
            _lib.check(L.et_comm_unique_id(ctypes.addressof(idbuf)))
        except _lib.EmbtabError as e:
            if world == 1:
                raise
            err = e
    if world > 1:
        import torch.distributed as dist

        # rank 0 always broadcasts (an empty id if it failed), so no rank is left
        # waiting for an id that never comes
        obj = [(b"" if err else bytes(idbuf)) if rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group)
        if err is not None:
            raise err
        if not obj[0]:
            raise _lib.EmbtabError("rank 0 could not make an RCCL unique id")
        idbuf = (ctypes.c_char * _lib.ET_COMM_ID_BYTES).from_buffer_copy(obj[0])
    comm = ctypes.c_void_p()
    _lib.check(L.et_comm_init(ctypes.byref(comm), world, ctypes.addressof(idbuf), rank))
    return comm


class ShardedPreallocation(ShardedMapLookup):
    """Round-1 name: table-wise plan, all-gather exchange, one chunk."""

    def __init__(self, plan: ShardPlan, rank: int, world: int, batch: int, dtype, device,
                 group=None):
        super().__init__(plan, rank, world, batch, dtype, device, group, "allgather", 1)
