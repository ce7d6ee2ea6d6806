"""A seeded random sweep of the lookup paths against the oracle: `lookup` (vector gather and
matrix pooled sum, src/lookup.jl:51-165) and the Preallocation `maplookup` (:305-371) over
random tables — storage (contiguous, paged with a random page size, device column pointers),
element type (Float32, Float64, Float16 in Julia's arithmetic or with Float32 sums, BFloat16,
Int32, Int64), rows, dims (vector-path and odd ones), pools, batches, prepended rows — every
output bit-identical to the oracle, every case an independent draw."""
import numpy as np
import pytest
import torch

import embtab as et
from embtab.tables import AbstractEmbeddingTable, Static

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
KINDS = ["f32", "f64", "f16", "f16acc", "bf16", "i32", "i64"]


class _ColPtr(AbstractEmbeddingTable):
    def __init__(self, dense, rng):
        R, D = dense.shape
        self.R, self.D = R, D
        es = dense.element_size()
        self.pitch = D + 16 // es
        self.perm = torch.from_numpy(rng.permutation(R)).to(DEV)
        self.pool = torch.zeros((R, self.pitch), dtype=dense.dtype, device=DEV)
        self.pool[self.perm, :D] = dense
        self.lookup_type = Static(D)

    def size(self):
        return (self.D, self.R)

    def columnpointers(self):
        es = self.pool.element_size()
        return self.pool.data_ptr() + self.perm.cpu().numpy().astype(np.int64) * self.pitch * es

    def example(self):
        return self.pool[0:1, :self.D]


def _host_table(rng, kind, R, D):
    from oracle import f32_to_bf16

    if kind in ("i32", "i64"):
        return rng.integers(-1000, 1000, (R, D)).astype(np.int32 if kind == "i32" else np.int64)
    x = rng.standard_normal((R, D)).astype(np.float32)
    if kind == "bf16":
        return f32_to_bf16(x)
    return x.astype({"f32": np.float32, "f64": np.float64, "f16": np.float16,
                     "f16acc": np.float16}[kind])


def _dev_table(h, kind, storage, rng):
    x = torch.from_numpy(h).to(DEV)
    if kind == "bf16":
        x = x.view(torch.bfloat16)
    D = h.shape[1]
    if storage == "simple":
        return et.SimpleEmbedding(x, Static(D))
    if storage == "paged":
        return et.SplitEmbedding(x, int(rng.integers(1, h.shape[0] + 1)))
    return _ColPtr(x, rng)


def _bits(t, kind):
    if kind in ("bf16", "f16", "f16acc"):
        t = t.view(torch.int16)
    return t.cpu().numpy().tobytes()


@pytest.mark.parametrize("seed", range(40))
def test_random_lookup_and_maplookup_vs_oracle(oracle, seed):
    rng = np.random.default_rng(1000 + seed)
    kind = KINDS[seed % len(KINDS)]
    bf16, acc = kind == "bf16", kind == "f16acc"
    n = int(rng.integers(1, 5))
    B = int(rng.choice([1, 7, 128, 1000, 4097]))
    P = int(rng.choice([1, 3, 20, 33]))
    k = int(rng.choice([0, 1, 16]))
    rows = [int(rng.choice([1, 5, 300, 3000])) for _ in range(n)]
    dims = [int(rng.choice([5, 16, 20, 64, 96, 128, 256])) for _ in range(n)]
    hs = [_host_table(rng, kind, r, d) for r, d in zip(rows, dims)]
    tabs = [_dev_table(h, kind, ["simple", "paged", "colptr"][int(rng.integers(0, 3))], rng)
            for h in hs]
    hidx = [rng.integers(1, r + 1, (B, P)) for r in rows]
    tdt = tabs[0].dtype

    def guarded(rows_, cols_):
        """A (rows_, cols_) destination inside a canary-filled buffer: one guard row above and
        below, 7 guard columns on each side (row stride cols_ + 14), so any write outside
        the destination shows up as a changed canary."""
        buf = torch.full((rows_ + 2, cols_ + 14), 0, dtype=tdt, device=DEV)
        buf.view(torch.uint8).fill_(0xA5)
        return buf, buf[1:rows_ + 1, 7:7 + cols_]

    def canaries_intact(buf, rows_, cols_):
        b = buf.view(torch.uint8).view(rows_ + 2, -1)
        es = buf.element_size()
        inner = torch.zeros_like(b, dtype=torch.bool)
        inner[1:rows_ + 1, 7 * es:(7 + cols_) * es] = True
        return bool((b[~inner] == 0xA5).all())

    # lookup: pooled sum of table 0 (matrix indices) and the gather (vector indices)
    # (lookup sums Float16 in Julia's Float16 arithmetic; maplookup below takes the option)
    buf, dst = guarded(B, dims[0])
    got = et.lookup_(dst, tabs[0], torch.from_numpy(hidx[0]).to(DEV))
    ref = oracle.pooled_sum(hs[0], hidx[0], bf16=bf16)
    assert _bits(got.contiguous(), kind) == np.ascontiguousarray(ref).view(ref.dtype).tobytes(), "pooled"
    assert canaries_intact(buf, B, dims[0]), "pooled: write outside the destination"
    v = hidx[0][:, 0].copy()
    buf, dst = guarded(B, dims[0])
    got = et.lookup_(dst, tabs[0], torch.from_numpy(v).to(DEV))
    assert _bits(got.contiguous(), kind) == np.ascontiguousarray(
        oracle.gather(hs[0], v, bf16=bf16)).tobytes()
    assert canaries_intact(buf, B, dims[0]), "gather: write outside the destination"
    # the Preallocation maplookup over every table (one fused launch)
    ld = k + sum(dims)
    buf, dst = guarded(B, ld)
    y = et.maplookup_(et.PreallocationStrategy(k), dst, tabs,
                      [torch.from_numpy(i).to(DEV) for i in hidx], f16_fp32_acc=acc)
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=k, f16_fp32_acc=acc, bf16=bf16)
    got = y.contiguous()
    got = got.view(torch.int16) if kind in ("bf16", "f16", "f16acc") else got
    got = got.cpu().numpy()[:, k:]
    assert got.tobytes() == np.ascontiguousarray(ref[:, k:]).view(got.dtype).tobytes(), "maplookup"
    assert canaries_intact(buf, B, ld), "maplookup: write outside the destination"
    assert et.check_errors() == 0


@pytest.mark.parametrize("seed", range(12))
def test_random_sharded_step_loopback_vs_oracle(oracle, seed):
    """The native sharded Preallocation step (csrc/et_shard.cpp) on N loopback ranks of one
    process, random shapes: 2-8 ranks, table-wise (count- or size-dealt) or feature-wise
    plans, all-gather in 1-5 pipelined chunks or all-to-all, odd batches, prepended rows —
    every rank's rows equal the unsharded oracle concat (src/lookup.jl:316-371)."""
    from test_gpu_loopback import Ranks, run_ranks

    from embtab.sharding import ShardPlan, piece_table

    rng = np.random.default_rng(2000 + seed)
    world = int(rng.integers(2, 9))
    n = int(rng.integers(world, 3 * world + 1))
    dims = [int(rng.choice([32, 64, 96, 128])) for _ in range(n)]
    rows = [int(rng.choice([3, 100, 2000, 30000])) for _ in range(n)]
    B = int(rng.integers(world, 3000))
    P = int(rng.choice([1, 8, 20]))
    k = int(rng.choice([0, 3]))
    planner = ["tablewise", "tablewise_sizes", "featurewise"][seed % 3]
    exchange = "alltoall" if seed % 4 == 3 else "allgather"
    chunks = 1 if exchange == "alltoall" else int(rng.integers(1, 6))
    hs = [rng.random((r, d), dtype=np.float32) for r, d in zip(rows, dims)]
    hidx = [rng.integers(1, r + 1, (B, P)) for r in rows]
    full = [et.SimpleEmbedding(torch.from_numpy(h).to(DEV), Static(h.shape[1])) for h in hs]
    didx = [torch.from_numpy(i).to(DEV) for i in hidx]
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=k)
    plan = (ShardPlan.featurewise(dims, world, k) if planner == "featurewise" else
            ShardPlan.tablewise(dims, world, k, sizes=rows if planner == "tablewise_sizes" else None))
    ranks = Ranks(plan, world, B, exchange, chunks)
    try:
        outs = []
        for st in ranks.steps:
            lo, hi = st._native.lo, st._native.hi
            outs.append(torch.full((hi - lo, plan.ld), -3.0, dtype=torch.float32, device=DEV))
        tabs = [[piece_table(full[p.table], p) for p in plan.pieces[r]] for r in range(world)]
        idxs = [[didx[p.table] for p in plan.pieces[r]] for r in range(world)]
        run_ranks(world, lambda r: ranks.steps[r](tabs[r], idxs[r], outs[r]))
        torch.cuda.synchronize()
        for r, st in enumerate(ranks.steps):
            lo, hi = st._native.lo, st._native.hi
            got = outs[r].cpu().numpy()
            assert got[:, k:].tobytes() == np.ascontiguousarray(ref[lo:hi, k:]).tobytes(), (
                seed, r, world, planner, exchange, chunks)
    finally:
        ranks.close()
