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


def plan_tables(ntables: int, world: int, sizes=None) -> list[list[int]]:
    """Balance whole tables over ranks by COUNT (every table costs B*P*D*4 bytes per
    lookup whatever its cardinality), contiguous groups, the largest tables spread
    over distinct ranks when ``sizes`` is given (26 tables on 8 GPUs
    -> 4,4,3,3,3,3,3,3)."""
    if world <= 0:
        raise ValueError("world must be positive")
    base, extra = divmod(ntables, world)
    counts = [base + (1 if r < extra else 0) for r in range(world)]
    if sizes is None:
        out, t = [], 0
        for c in counts:
            out.append(list(range(t, t + c)))
            t += c
        return out
    # deal tables in descending size round-robin, respecting the counts
    order = sorted(range(ntables), key=lambda t: -sizes[t])
    out = [[] for _ in range(world)]
    r = 0
    for t in order:
        while len(out[r]) >= counts[r]:
            r = (r + 1) % world
        out[r].append(t)
        r = (r + 1) % world
    return [sorted(o) for o in out]


@dataclass(frozen=True)
class Piece:
    """Features ``[f0, f0 + dim)`` of global table ``table``; its columns of the
    destination start at ``col`` (prependrows included)."""

    table: int
    f0: int
    dim: int
    col: int


def _vec_split(t: int, f0: int, dim: int, col: int, es: int = 4) -> list[Piece]:
    """Cut a feature range into vector-kernel widths where alignment allows (96 ->
    64 + 32); anything else stays one piece (the generic kernel takes it)."""
    out = []
    while dim > 0:
        w = next((v for v in VEC_DIMS if v <= dim and (f0 * es) % 16 == 0), None)
        if w is None or (dim not in VEC_DIMS and dim % 16 != 0):
            out.append(Piece(t, f0, dim, col))
            break
        out.append(Piece(t, f0, w, col))
        f0, dim, col = f0 + w, dim - w, col + w
    return out


def plan_features(dims, world: int, granule: int = 32) -> list[tuple[int, int]]:
    """Feature ranges ``[lo, hi)`` of the concatenated feature axis, one per rank:
    cut points are table edges or multiples of ``granule`` inside a table, each
    chosen nearest to an equal split."""
    if world <= 0:
        raise ValueError("world must be positive")
    cuts, start = {0}, 0
    for d in dims:
        for f in range(granule, d, granule):
            cuts.add(start + f)
        start += d
        cuts.add(start)
    F = start
    cands = sorted(cuts)
    bounds = [0]
    for r in range(1, world):
        target = F * r / world
        best = min((c for c in cands if c >= bounds[-1]), key=lambda c: (abs(c - target), c))
        bounds.append(best)
    bounds.append(F)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


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
        offs = _table_cols(dims, prependrows)
        return cls(dims, prependrows,
                   [[Piece(t, 0, dims[t], offs[t]) for t in ts]
                    for ts in plan_tables(len(dims), world, sizes)])

    @classmethod
    def featurewise(cls, dims, world: int, prependrows: int = 0,
                    granule: int = 32) -> "ShardPlan":
        offs = _table_cols(dims, prependrows)
        starts = [o - prependrows for o in offs]
        pieces = []
        for lo, hi in plan_features(dims, world, granule):
            mine = []
            for t, d in enumerate(dims):
                a, b = max(lo, starts[t]), min(hi, starts[t] + d)
                if a < b:
                    mine += _vec_split(t, a - starts[t], b - a, prependrows + a)
            pieces.append(mine)
        return cls(dims, prependrows, pieces)

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


def _table_cols(dims, prependrows):
    offs, c = [], prependrows
    for d in dims:
        offs.append(c)
        c += d
    return offs


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


class ShardedMapLookup:
    """``maplookup!(PreallocationStrategy(k), dst, tables, I)`` over the ranks of
    ``group`` (RCCL on ROCm; gloo for CPU rehearsal).

    ``piece_tables`` / ``piece_idx`` are this rank's pieces (``piece_table``) and
    their index arrays, in ``plan.pieces[rank]`` order."""

    def __init__(self, plan: ShardPlan, rank: int, world: int, batch: int, dtype, device,
                 group=None, exchange: str = "allgather", chunks: int = 1):
        if plan.world != world:
            raise ValueError("plan and world size differ")
        if exchange not in ("allgather", "alltoall", "p2p"):
            raise ValueError(f"unknown exchange {exchange!r}")
        self.plan, self.rank, self.world, self.batch = plan, rank, world, batch
        self.device, self.group, self.exchange_kind = torch.device(device), group, exchange
        self.chunks = max(1, min(chunks, batch)) if exchange != "alltoall" else 1
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
        """Unmap the peers' destinations (p2p exchange)."""
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
        if self.exchange_kind in ("allgather", "p2p"):
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


class ShardedPreallocation(ShardedMapLookup):
    """Round-1 name: table-wise plan, all-gather exchange, one chunk."""

    def __init__(self, plan: ShardPlan, rank: int, world: int, batch: int, dtype, device,
                 group=None):
        super().__init__(plan, rank, world, batch, dtype, device, group, "allgather", 1)
