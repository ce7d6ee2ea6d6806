"""The native sharded step (csrc/et_shard.cpp) at world > 1 on one GPU.

et_comm_loopback makes N simulated ranks of this process; each rank is driven by its
own host thread and stream, so the world > 1 code of et_sharded_maplookup and
et_sharded_piece_grads runs unchanged: gathered-chunk offsets, the all-to-all split
arithmetic, the side-stream event pipeline, the multi-launch assembly of a size-dealt
table-wise plan.  Every rank's result must equal the unsharded PreallocationStrategy
concat (reference src/lookup.jl:316-371, the row-block views at :334-340) bit for bit,
and the all-to-all backward must hand every rank exactly its pieces' gradient rows."""
import threading

import numpy as np
import pytest
import torch

import embtab as et
from embtab import _lib
from embtab.sharding import ShardedMapLookup, ShardPlan, loopback_comms, piece_table

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


def run_ranks(world, fn):
    """fn(rank) on `world` threads, each with its own stream; re-raises the first error."""
    errs = [None] * world

    def body(r):
        try:
            s = torch.cuda.Stream(DEV)
            with torch.cuda.stream(s):
                fn(r)
            s.synchronize()
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    for e in errs:
        if e is not None:
            raise e
    assert not any(t.is_alive() for t in th), "a rank hung"


class Ranks:
    """World simulated ranks of one plan: their ShardedMapLookup steps on loopback comms."""

    def __init__(self, plan, world, B, exchange, chunks, dtype=torch.float32):
        self.comms = loopback_comms(world)
        self.steps = [ShardedMapLookup(plan, r, world, B, dtype, DEV, exchange=exchange,
                                       chunks=chunks, comm=self.comms[r])
                      for r in range(world)]
        assert all(s._native is not None for s in self.steps)

    def close(self):
        for s in self.steps:
            s.close()
        L = _lib.load()
        for c in self.comms:
            _lib.check(L.et_comm_destroy(c))


def _setup(seed, dims, rows, B, P=20):
    rng = np.random.default_rng(seed)
    hs = [rng.random((r, d), dtype=np.float32) for r, d in zip(rows, dims)]
    hidx = [rng.integers(1, r + 1, (B, P)) for r in rows]
    full = [et.SimpleEmbedding(dev(h), et.Static(h.shape[1])) for h in hs]
    didx = [dev(i) for i in hidx]
    return rng, hs, hidx, full, didx


DIMS = [128] * 5 + [64, 256, 48, 128, 32, 96]
ROWS = [300, 5000, 20, 800, 64, 1000, 77, 129, 40000, 5, 610]


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("planner", ["tablewise_sizes", "tablewise", "featurewise"])
@pytest.mark.parametrize("exchange,chunks", [("allgather", 1), ("allgather", 4),
                                             ("alltoall", 1)])
def test_native_step_loopback(oracle, world, planner, exchange, chunks):
    B, k = 1003, 5  # odd batch: uneven chunks and all-to-all slices
    rng, hs, hidx, full, didx = _setup(world * 31 + len(planner), DIMS, ROWS, B)
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=k)
    if planner == "featurewise":
        plan = ShardPlan.featurewise(DIMS, world, k)
    else:
        plan = ShardPlan.tablewise(DIMS, world, k,
                                   sizes=ROWS if planner == "tablewise_sizes" else None)
    ranks = Ranks(plan, world, B, exchange, chunks)
    try:
        outs = []
        for r, st in enumerate(ranks.steps):
            lo, hi = (st._native.lo, st._native.hi)
            outs.append(torch.full((hi - lo, plan.ld), -3.0, dtype=torch.float32, device=DEV))
        tabs = [[piece_table(full[p.table], p) for p in plan.pieces[r]] for r in range(world)]
        idxs = [[didx[p.table] for p in plan.pieces[r]] for r in range(world)]
        for _ in range(2):  # twice: the second step reuses slabs, events and the group
            run_ranks(world, lambda r: ranks.steps[r](tabs[r], idxs[r], outs[r]))
        torch.cuda.synchronize()
        for r, st in enumerate(ranks.steps):
            lo, hi = st._native.lo, st._native.hi
            got = outs[r].cpu().numpy()
            assert got[:, k:].tobytes() == np.ascontiguousarray(ref[lo:hi, k:]).tobytes(), r
            assert (got[:, :k] == -3.0).all()  # prepended rows untouched
        if exchange == "alltoall":
            delta = torch.empty((B, plan.ld), dtype=torch.float32, device=DEV)
            _lib.check(_lib.load().et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(),
                                                   77, 0, -1.0, 1.0, _lib.stream_handle()))
            torch.cuda.synchronize()
            grads = [None] * world

            def bwd(r):
                lo, hi = ranks.steps[r]._native.lo, ranks.steps[r]._native.hi
                grads[r] = ranks.steps[r].piece_grads(tabs[r], idxs[r], delta[lo:hi])

            run_ranks(world, bwd)
            torch.cuda.synchronize()
            for r in range(world):
                for p, g in zip(plan.pieces[r], grads[r]):
                    assert torch.equal(g.delta, delta[:, p.col:p.col + p.dim]), (r, p)
    finally:
        ranks.close()


def test_allgather_concat_loopback(oracle):
    """et_allgather_concat on a 3-rank loopback group: rank r's slab lands in every
    rank's gathered buffer at slot r, then in its destination rows."""
    world, B, slab_ld, ld = 3, 500, 24, 80
    L = _lib.load()
    comms = loopback_comms(world)
    rng = np.random.default_rng(9)
    slabs = [dev(rng.standard_normal((B, slab_ld)).astype(np.float32)) for _ in range(world)]
    rows = np.array([24, 20, 17], np.int32)
    offs = np.array([3, 27, 50], np.int64)
    gathered = [torch.empty((world, B, slab_ld), dtype=torch.float32, device=DEV)
                for _ in range(world)]
    dsts = [torch.zeros((B, ld), dtype=torch.float32, device=DEV) for _ in range(world)]
    torch.cuda.synchronize()
    try:
        def one(r):
            _lib.check(L.et_allgather_concat(comms[r], _lib.ET_F32, slabs[r].data_ptr(), slab_ld,
                                             B, gathered[r].data_ptr(), world, rows.ctypes.data,
                                             offs.ctypes.data, dsts[r].data_ptr(), ld,
                                             _lib.stream_handle()))

        run_ranks(world, one)
        torch.cuda.synchronize()
        for r in range(world):
            for p in range(world):
                assert torch.equal(gathered[r][p], slabs[p])
                assert torch.equal(dsts[r][:, offs[p]:offs[p] + rows[p]], slabs[p][:, :rows[p]])
        # a wrong nranks for the group is refused, before any collective
        rc = L.et_allgather_concat(comms[0], _lib.ET_F32, slabs[0].data_ptr(), slab_ld, B,
                                   gathered[0].data_ptr(), 2, rows.ctypes.data, offs.ctypes.data,
                                   dsts[0].data_ptr(), ld, _lib.stream_handle())
        assert rc != 0
    finally:
        for c in comms:
            _lib.check(L.et_comm_destroy(c))


@pytest.mark.parametrize("planner", ["tablewise_sizes", "featurewise"])
def test_config5_native_step_loopback_8_ranks(oracle, planner):
    """BASELINE config 5 at full size through the native world-8 step: the 26 Criteo
    tables, B = 131072, pool 20, 8 loopback ranks on one GPU (table-wise with the sizes
    dealt so the 5 largest tables land on distinct ranks, and feature-wise), all-gather
    in 4 pipelined chunks.  Every rank's destination equals the unsharded lookup bit for
    bit (which is itself checked against the oracle on sampled bags)."""
    from test_gpu_fullsize import ROWS as CRITEO, _sample_check

    Bc, D, P, world = 131072, 128, 20, 8
    L = _lib.load()
    s = _lib.stream_handle()
    tabs, idx = [], []
    for t, R in enumerate(CRITEO):
        x = torch.empty((R, D), dtype=torch.float32, device=DEV)
        _lib.check(L.et_fill_uniform(_lib.ET_F32, x.data_ptr(), x.numel(), 1000 + t, 0, 0.0, 1.0,
                                     s))
        I = torch.empty((Bc, P), dtype=torch.int64, device=DEV)
        _lib.check(L.et_fill_index_uniform(I.data_ptr(), I.numel(), R, 5000 + t, 0, s))
        tabs.append(et.SimpleEmbedding(x, et.Static(D)))
        idx.append(I)
    base = et.maplookup(et.PreallocationStrategy(), tabs, idx)
    g = torch.Generator().manual_seed(7)
    _sample_check(oracle, tabs, idx, base, torch.randint(0, Bc, (128,), generator=g).to(DEV))
    dims = [D] * len(CRITEO)
    plan = (ShardPlan.tablewise(dims, world, sizes=CRITEO) if planner == "tablewise_sizes"
            else ShardPlan.featurewise(dims, world))
    if planner == "tablewise_sizes":
        big = [sum(1 for p in plan.pieces[r] if CRITEO[p.table] * D * 4 > (256 << 20))
               for r in range(world)]
        assert max(big) <= 1, big  # the 5 tables above 256 MiB on distinct ranks
    ranks = Ranks(plan, world, Bc, "allgather", 4)
    try:
        ptabs = [[piece_table(tabs[p.table], p) for p in plan.pieces[r]] for r in range(world)]
        pidx = [[idx[p.table] for p in plan.pieces[r]] for r in range(world)]
        # all ranks write their own full destination in one step (8 x 1.74 GB)
        dsts = [torch.empty_like(base) for _ in range(world)]
        run_ranks(world, lambda q: ranks.steps[q](ptabs[q], pidx[q], dsts[q]))
        torch.cuda.synchronize()
        for q in range(world):
            assert torch.equal(dsts[q], base), q
    finally:
        ranks.close()
        del tabs, idx, base
        torch.cuda.empty_cache()


def test_loopback_rank_failing_before_collective_aborts_group():
    """A loopback rank whose step fails before its collective (here: a wrong descriptor
    count, refused by the argument check) aborts the group, so its peer's pending
    all-gather returns an error at once instead of after the 120 s rendezvous timeout
    (et_shard.cpp loop_abort)."""
    import time

    world, B, k = 2, 257, 0
    rng, hs, hidx, full, didx = _setup(5, DIMS, ROWS, B)
    plan = ShardPlan.tablewise(DIMS, world, k)
    ranks = Ranks(plan, world, B, "allgather", 1)
    try:
        outs = [torch.empty((B, plan.ld), dtype=torch.float32, device=DEV) for _ in range(world)]
        tabs = [[piece_table(full[p.table], p) for p in plan.pieces[r]] for r in range(world)]
        idxs = [[didx[p.table] for p in plan.pieces[r]] for r in range(world)]
        assert len(tabs[1]) >= 2
        errs = [None] * world

        def body(r):
            try:
                if r == 1:  # one descriptor short: fails before joining the all-gather
                    ranks.steps[r](tabs[r][:-1], idxs[r][:-1], outs[r])
                else:
                    ranks.steps[r](tabs[r], idxs[r], outs[r])
            except _lib.EmbtabError as e:
                errs[r] = e

        t0 = time.monotonic()
        th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=150)
        elapsed = time.monotonic() - t0
        assert not any(t.is_alive() for t in th), "a rank hung"
        assert errs[1] is not None and "descriptors given" in str(errs[1])
        assert errs[0] is not None and "did not join" in str(errs[0])
        assert elapsed < 30, f"peer waited {elapsed:.1f} s"
        torch.cuda.synchronize()
    finally:
        ranks.close()
