"""Sharded Preallocation maplookup on 2 and 3 CPU ranks (gloo): the real plans,
piece decomposition, chunked all-gather / all-to-all exchange and assembly plan of
embtab.sharding, with the oracle standing in for the two device kernels
(et_maplookup_prealloc into the slab and et_concat_slabs), checked against the
single-process Preallocation result."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from embtab.sharding import ShardedMapLookup, ShardPlan, plan_features, plan_tables

CRITEO = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194,
          27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572]


def test_plan_tables_counts():
    a = plan_tables(26, 8)
    assert [len(x) for x in a] == [4, 4, 3, 3, 3, 3, 3, 3]
    assert sorted(t for x in a for t in x) == list(range(26))
    b = plan_tables(26, 8, sizes=CRITEO)
    big5 = sorted(range(26), key=lambda t: -CRITEO[t])[:5]
    owners = [next(r for r, x in enumerate(b) if t in x) for t in big5]
    assert len(set(owners)) == 5  # the five largest tables on distinct GPUs
    assert [len(x) for x in b] == [4, 4, 3, 3, 3, 3, 3, 3]
    assert plan_tables(26, 2) == [list(range(13)), list(range(13, 26))]


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_featurewise_plan_covers_every_feature_once(world):
    dims = [128] * 26
    plan = ShardPlan.featurewise(dims, world, prependrows=16)
    seen = np.zeros((26, 128), np.int32)
    for r, ps in enumerate(plan.pieces):
        col = None
        for p in ps:
            seen[p.table, p.f0:p.f0 + p.dim] += 1
            assert p.col == 16 + 128 * p.table + p.f0
            assert col is None or p.col == col  # one contiguous run of dst columns
            col = p.col + p.dim
            assert p.dim in (16, 32, 64, 128, 256, 512) and p.f0 % 4 == 0
        assert len(plan.runs(r)) == 1
    assert (seen == 1).all()
    if world in (1, 2, 4, 8):  # 3328 features cut into equal slabs: no padding
        assert plan.widths == [3328 // world] * world and plan.slab_ld == 3328 // world
    assert len(plan.assembly_launches()) == 1
    assert plan_features([5, 7], 2) == [(0, 5), (5, 12)]  # unsplittable tables


class _Tab:
    """Stand-in piece table for the gradient plumbing (only the lookup type is read)."""

    lookup_type = None


def _worker(rank, world, port, sizes, result_q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import oracle as orc

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(0)
    dims = [16, 32, 16, 48, 16, 128, 96]
    B, P, k = 41, 6, 3
    tabs = [rng.random((r, d), dtype=np.float32) for r, d in zip(sizes, dims)]
    idx = [rng.integers(1, r + 1, (B, P)) for r in sizes]
    ref = orc.maplookup_prealloc(tabs, idx, prependrows=k)

    class OracleShard(ShardedMapLookup):
        """Device kernels replaced by the oracle / numpy (same semantics)."""

        def lookup_chunk(self, piece_tables, piece_idx, b0, b1):
            if piece_tables:
                s = orc.maplookup_prealloc(piece_tables, [i[b0:b1] for i in piece_idx])
                self.slab[b0:b1, :s.shape[1]] = torch.from_numpy(s)

        def assemble_chunk(self, gathered, dst):
            g = gathered.numpy()
            for shift, rows, offs in self.launches:
                for r, (n, o) in enumerate(zip(rows, offs)):
                    if n:
                        dst[:, o:o + n] = torch.from_numpy(g[r][:, shift:shift + n])

        def split_rows(self, delta_local, send):
            for shift, rows, offs in self.launches:
                for r, (n, o) in enumerate(zip(rows, offs)):
                    if n:
                        send[r][:, shift:shift + n] = delta_local[:, o:o + n]

    plans = {"table": ShardPlan.tablewise(dims, world, k),
             "table_spread": ShardPlan.tablewise(dims, world, k, sizes=sizes),
             "feature": ShardPlan.featurewise(dims, world, k, granule=16)}
    for name, plan in plans.items():
        ps = plan.pieces[rank]
        ptabs = [np.ascontiguousarray(tabs[p.table][:, p.f0:p.f0 + p.dim]) for p in ps]
        pidx = [idx[p.table] for p in ps]
        for exchange, chunks in (("allgather", 1), ("allgather", 3), ("alltoall", 1)):
            sm = OracleShard(plan, rank, world, B, torch.float32, torch.device("cpu"),
                             exchange=exchange, chunks=chunks)
            if exchange == "allgather":
                dst = torch.zeros((B, plan.ld))
                sm(ptabs, pidx, dst)
                ok = np.array_equal(dst.numpy()[:, k:], ref[:, k:])
            else:
                dst = torch.zeros((sm.mine, plan.ld))
                sm(ptabs, pidx, dst)
                lo, hi = sm.split[rank], sm.split[rank + 1]
                ok = np.array_equal(dst.numpy()[:, k:], ref[lo:hi, k:])
            # backward: the gradient columns of this rank's pieces, for every bag
            full = torch.from_numpy(np.random.default_rng(9).standard_normal(
                (B, plan.ld)).astype(np.float32))
            local = full if exchange == "allgather" else full[sm.split[rank]:sm.split[rank + 1]]
            grads = sm.piece_grads([_Tab() for _ in ps], pidx, local.contiguous())
            for p, g in zip(ps, grads):
                ok = ok and torch.equal(g.delta, full[:, p.col:p.col + p.dim])
            result_q.put((rank, name, exchange, chunks, bool(ok)))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_prealloc_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    sizes = [50, 400, 30, 70, 1000, 20, 333]
    procs = [ctx.Process(target=_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    n = world * 3 * 3
    res = [q.get(timeout=5) for _ in range(n)]
    assert len(res) == n and all(r[-1] for r in res), [r for r in res if not r[-1]]


def test_compact_piece_tables_hold_only_the_slice():
    """Feature-wise ranks keep their slice as its own (R, dim) table (ld = dim), not a
    view of the full table: values equal the slice, memory is the slice's."""
    import torch

    import embtab as et
    from embtab.sharding import Piece, compact_piece_table

    full = et.SimpleEmbedding(torch.arange(40 * 128, dtype=torch.float32).view(40, 128),
                              et.Static(128))
    p = Piece(3, 32, 64, 7)
    c = compact_piece_table(full, p)
    assert c.data.shape == (40, 64) and c.ld == 64 and c.data.is_contiguous()
    assert torch.equal(c.data, full.data[:, 32:96])
    assert c.data.untyped_storage().nbytes() == 40 * 64 * 4
    assert c.lookup_type == et.Static(64)
    assert compact_piece_table(full, Piece(3, 0, 128, 7)) is full


def _comm_fail_worker(rank, world, port, result_q):
    import embtab.sharding as sh
    from embtab import _lib

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class FailingL:
        """Library stand-in whose et_comm_unique_id fails (rank 0 only calls it)."""

        def et_comm_unique_id(self, buf):
            return 5

        def et_last_error(self):
            return b"no RCCL here"

        def et_comm_init(self, *a):
            raise AssertionError("et_comm_init reached after a failed unique id")

    real = _lib.load
    _lib.load = lambda: FailingL()
    try:
        sh.make_comm(None, rank, world)
        raised = False
    except _lib.EmbtabError:
        raised = True
    finally:
        _lib.load = real
    sm = sh.ShardedMapLookup.__new__(sh.ShardedMapLookup)
    sm.device, sm.group = torch.device("cpu"), None
    agree_fail = sm._all_ranks_ok(rank != 1)  # one rank failed -> every rank sees False
    agree_ok = sm._all_ranks_ok(True)
    result_q.put((rank, raised, agree_fail, agree_ok))
    dist.destroy_process_group()


def test_native_step_fallback_is_collective():
    """A failed RCCL unique id on rank 0 raises on every rank (rank 0 broadcasts an empty
    id instead of leaving the others blocked), and the auto fallback is decided by a MIN
    over the ranks, so every rank takes the same exchange."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert res == [(0, True, False, True), (1, True, False, True)], res
