"""Table-wise sharding of a PreallocationStrategy maplookup across the GPUs of a node.

No counterpart exists in the single-process reference: tables
are independent, so each rank owns whole tables, looks them up for the full batch
into a local slab with ONE fused launch, and the concat of the reference's
PreallocationStrategy (src/lookup.jl:334-340) becomes an RCCL all-gather of the
slabs over xGMI plus one assembly kernel (et_concat_slabs) into the
``(B, prependrows + sum D)`` destination.

The data path is: et_maplookup_prealloc (local tables -> slab) ->
all_gather_into_tensor (slabs, RCCL) -> et_concat_slabs (slabs -> dst).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import torch

from . import _lib
from .lookup import _ld


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


@dataclass
class ShardLayout:
    """Where every rank's tables land in the concat destination."""

    dims: list[int]
    prependrows: int
    assignment: list[list[int]]
    offsets: list[int] = field(init=False)  # dst row of each global table
    rank_rows: list[int] = field(init=False)
    slab_ld: int = field(init=False)

    def __post_init__(self):
        off = self.prependrows
        self.offsets = []
        for d in self.dims:
            self.offsets.append(off)
            off += d
        self.ld = off
        self.rank_rows = [sum(self.dims[t] for t in ts) for ts in self.assignment]
        # pad the slab to a multiple of 4 elements so 16-B vector stores stay aligned
        self.slab_ld = max(4, (max(self.rank_rows) + 3) // 4 * 4)

    def rank_segments(self, r: int):
        """Contiguous (slab_row, dst_row, rows) runs of rank r's tables."""
        segs = []
        srow = 0
        for t in self.assignment[r]:
            d = self.dims[t]
            if segs and segs[-1][1] + segs[-1][2] == self.offsets[t] and \
                    segs[-1][0] + segs[-1][2] == srow:
                segs[-1] = (segs[-1][0], segs[-1][1], segs[-1][2] + d)
            else:
                segs.append((srow, self.offsets[t], d))
            srow += d
        return segs


class ShardedPreallocation:
    """maplookup(PreallocationStrategy(k), tables, I) with the tables split over ranks.

    ``local_tables`` / ``local_idx`` are this rank's tables (in assignment order) and
    their index arrays.  ``group`` is a torch.distributed process group (RCCL on
    ROCm)."""

    def __init__(self, layout: ShardLayout, rank: int, world: int, batch: int, dtype, device,
                 group=None):
        self.layout, self.rank, self.world, self.batch = layout, rank, world, batch
        self.device = device
        self.group = group
        self.slab = torch.empty((batch, layout.slab_ld), dtype=dtype, device=device)
        self.gathered = torch.empty((world, batch, layout.slab_ld), dtype=dtype, device=device)
        # Per-rank contiguous segments -> et_concat_slabs requires one run per rank, so
        # assignments are contiguous table ranges (plan_tables without sizes) or the
        # concat is issued once per run.
        self.runs = [layout.rank_segments(r) for r in range(world)]

    def local_lookup(self, local_tables, local_idx, nontemporal=True):
        """One fused launch: this rank's tables -> its slab."""
        from .lookup import PreallocationStrategy, maplookup_

        maplookup_(PreallocationStrategy(0), self.slab, local_tables, local_idx, nontemporal)
        return self.slab

    def exchange(self):
        import torch.distributed as dist

        if self.world == 1:
            self.gathered[0].copy_(self.slab)
            return self.gathered
        if dist.get_backend(self.group) == "gloo":  # CPU rehearsal: no all_gather_into_tensor
            dist.all_gather(list(self.gathered.unbind(0)), self.slab, group=self.group)
        else:
            dist.all_gather_into_tensor(self.gathered.view(-1), self.slab.view(-1),
                                        group=self.group)
        return self.gathered

    def assembly_launches(self):
        """The et_concat_slabs launches that assemble the destination: a list of
        ``(slab_row_shift, rows[rank], dst_row_off[rank])``.  With contiguous table
        ranges per rank (plan_tables without sizes) this is one launch."""
        launches = []
        max_runs = max(len(r) for r in self.runs)
        for k in range(max_runs):
            per = {}
            for r in range(self.world):
                if k < len(self.runs[r]):
                    srow, drow, n = self.runs[r][k]
                    rows, offs = per.setdefault(srow, ([0] * self.world, [0] * self.world))
                    rows[r], offs[r] = n, drow
            for shift in sorted(per):
                launches.append((shift, per[shift][0], per[shift][1]))
        return launches

    def assemble(self, dst: torch.Tensor):
        """et_concat_slabs: every rank's slab rows into their dst rows."""
        L = _lib.load()
        for shift, rows, offs in self.assembly_launches():
            rr = (ctypes.c_int32 * self.world)(*rows)
            oo = (ctypes.c_int64 * self.world)(*offs)
            base = self.gathered.data_ptr() + shift * self.gathered.element_size()
            _lib.check(L.et_concat_slabs(
                _lib.et_dtype(dst), base, self.world, self.layout.slab_ld, self.batch,
                ctypes.addressof(rr), ctypes.addressof(oo), dst.data_ptr(), _ld(dst),
                _lib.stream_handle(dst.device)))
        return dst

    def __call__(self, local_tables, local_idx, dst: torch.Tensor):
        self.local_lookup(local_tables, local_idx)
        self.exchange()
        return self.assemble(dst)
