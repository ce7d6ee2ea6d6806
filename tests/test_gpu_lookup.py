"""Parity of the HIP forward path with the oracle (bit-exact), through the C ABI.

Mirrors test/lookup.jl (dims 32..1504, permutations / repeats, 12 lookups per
output), test/map.jl (strategy equivalence over every index container) and the
README KATs, plus the engine's own edge cases (dtypes, strided destinations,
empty inputs, out-of-range indices)."""
import numpy as np
import pytest
import torch

import embtab as et

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


def host(x):
    return x.cpu().numpy()


def table(h, static=True):
    return et.SimpleEmbedding(dev(h), et.Static(h.shape[1]) if static else et.Dynamic)


def bits_equal(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


def test_readme_kats(kat):
    k = kat["readme_lookup"]
    A = table(np.asarray(k["table_columns"], np.int64), static=False)
    got = et.lookup(A, dev(np.array(k["vector_indices"])))
    assert host(got).tolist() == k["vector_expected_columns"]
    got = et.lookup(A, dev(np.array(k["matrix_indices_bags"])))
    assert host(got).tolist() == k["matrix_expected_columns"]
    m = kat["readme_maplookup"]
    tabs = [table(np.asarray(m["A_columns"], np.int64), False),
            table(np.asarray(m["B_columns"], np.int64), False)]
    idx = [dev(np.array(m["iA"])), dev(np.array(m["iB"]))]
    res = et.maplookup(tabs, idx)
    assert host(res[0]).tolist() == m["expected_A_columns"]
    assert host(res[1]).tolist() == m["expected_B_columns"]
    comb = torch.stack(idx)  # Julia hcat(iA, iB): 3 x 2 -> torch (2, 3)
    res2 = et.maplookup(tabs, comb)
    assert all(torch.equal(a, b) for a, b in zip(res, res2))
    cat = et.maplookup(et.PreallocationStrategy(), tabs, idx)
    assert torch.equal(cat, torch.cat(res, 1))


DIMS = [16, 32, 64, 128, 256, 512, 1024, 1504]


@pytest.mark.parametrize("dim", DIMS)
@pytest.mark.parametrize("static", [True, False])
def test_lookup_parity(oracle, dim, static):
    rng = np.random.default_rng(dim)
    ncols = 1000
    h = rng.random((ncols, dim), dtype=np.float32)
    A = table(h, static)
    for I in (rng.permutation(ncols) + 1, rng.integers(1, ncols + 1, ncols)):
        assert bits_equal(host(et.lookup(A, dev(I))), oracle.lookup(h, I))
    for I in (np.stack([rng.permutation(np.arange(2, ncols + 1)) for _ in range(12)], 1),
              rng.integers(1, ncols + 1, (ncols, 12)),
              rng.integers(1, ncols + 1, (333, 20)),
              rng.integers(1, ncols + 1, (77, 45))):  # pool > 32: several index chunks
        assert bits_equal(host(et.lookup(A, dev(I))), oracle.lookup(h, I))


@pytest.mark.parametrize("dim", [20, 24, 36, 48, 96, 200, 384, 1000, 2048])
def test_masked_vector_dims(oracle, dim):
    """Dims that are a multiple of 16 bytes but not a power-of-two vector width run the
    masked vector kernel (next power-of-two capacity): bit-identical to the oracle for
    pooled sums (pool 1, 12, 45), gathers, a strided destination and bad indices."""
    rng = np.random.default_rng(dim)
    h = rng.standard_normal((700, dim)).astype(np.float32)
    A = table(h)
    for I in (rng.integers(1, 701, (300, 12)), rng.integers(1, 701, (77, 45)),
              rng.integers(1, 701, (64, 1))):
        assert bits_equal(host(et.lookup(A, dev(I))), oracle.pooled_sum(h, I))
    v = rng.integers(1, 701, 257)
    assert bits_equal(host(et.lookup(A, dev(v))), oracle.gather(h, v))
    I = rng.integers(1, 701, (100, 20))
    big = torch.full((100, dim + 12), -3.0, dtype=torch.float32, device=DEV)
    et.lookup_(big[:, 4:4 + dim], A, dev(I))
    got = host(big)
    assert bits_equal(got[:, 4:4 + dim], oracle.pooled_sum(h, I))
    assert (got[:, :4] == -3.0).all() and (got[:, 4 + dim:] == -3.0).all()
    et.check_errors()
    bad = I.copy()
    bad[3, 5] = 701
    out = host(et.lookup(A, dev(bad)))
    assert et.check_errors() == 1
    ref = oracle.pooled_sum(h, I)
    ref[3] = oracle.pooled_sum(h, np.delete(I[3:4], 5, axis=1))[0]
    assert bits_equal(out, ref)


@pytest.mark.parametrize("dtype", [np.float64, np.float16, np.int64, "bf16"])
def test_masked_dims_other_types_and_mixed_launch(oracle, dtype):
    rng = np.random.default_rng(5)
    dims = [24, 40, 200, 128, 96]
    hs = []
    for d in dims:
        x = rng.standard_normal((300, d)) * 50
        hs.append(oracle.f32_to_bf16(x.astype(np.float32)) if dtype == "bf16"
                  else x.astype(dtype))
    hidx = [rng.integers(1, 301, (150, 16)) for _ in dims]
    tabs = [et.SimpleEmbedding(dev(h).view(torch.bfloat16) if dtype == "bf16" else dev(h))
            for h in hs]
    out = et.maplookup(et.PreallocationStrategy(1), tabs, [dev(i) for i in hidx])
    got = host(out.view(torch.int16)).view(np.uint16) if dtype == "bf16" else host(out)
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=1, bf16=dtype == "bf16")
    assert bits_equal(got[:, 1:], ref[:, 1:])


@pytest.mark.parametrize("dtype", [np.float64, np.int32, np.int64, np.float16])
@pytest.mark.parametrize("dim", [16, 128, 40])
def test_lookup_dtypes(oracle, dtype, dim):
    rng = np.random.default_rng(1)
    h = (rng.standard_normal((500, dim)) * 100).astype(dtype)
    A = table(h)
    I = rng.integers(1, 501, (200, 20))
    assert bits_equal(host(et.lookup(A, dev(I))), oracle.pooled_sum(h, I))
    v = rng.integers(1, 501, 300)
    assert bits_equal(host(et.lookup(A, dev(v))), oracle.gather(h, v))


@pytest.mark.parametrize("dim", [16, 128, 512, 40])
def test_bf16_tables(oracle, dim):
    """bfloat16 tables (fp32 accumulation, one rounding): pooled sums, gathers, the
    fused Preallocation launch and the fill are bit-identical to the oracle."""
    rng = np.random.default_rng(dim)
    h = oracle.f32_to_bf16(rng.standard_normal((600, dim)).astype(np.float32))
    A = et.SimpleEmbedding(dev(h).view(torch.bfloat16))
    assert A.dtype == torch.bfloat16
    I = rng.integers(1, 601, (300, 20))
    got = et.lookup(A, dev(I))
    assert got.dtype == torch.bfloat16
    assert bits_equal(host(got.view(torch.int16)).view(np.uint16),
                      oracle.pooled_sum(h, I, bf16=True))
    v = rng.integers(1, 601, 333)
    assert bits_equal(host(et.lookup(A, dev(v)).view(torch.int16)).view(np.uint16),
                      oracle.gather(h, v, bf16=True))
    hs = [h, oracle.f32_to_bf16(rng.random((50, dim), dtype=np.float32))]
    idx = [I, rng.integers(1, 51, (300, 7))]
    tabs = [A, et.SimpleEmbedding(dev(hs[1]).view(torch.bfloat16))]
    out = et.maplookup(et.PreallocationStrategy(2), tabs, [dev(i) for i in idx])
    ref = oracle.maplookup_prealloc(hs, idx, prependrows=2, bf16=True)
    assert bits_equal(host(out.view(torch.int16)).view(np.uint16)[:, 2:], ref[:, 2:])
    from embtab import _lib

    buf = torch.empty(5000, dtype=torch.bfloat16, device=DEV)
    _lib.check(_lib.load().et_fill_uniform(_lib.ET_BF16, buf.data_ptr(), 5000, 9, 3, -2.0, 2.0,
                                           _lib.stream_handle()))
    assert bits_equal(host(buf.view(torch.int16)).view(np.uint16),
                      oracle.fill_uniform((5000,), "bf16", 9, 3, -2.0, 2.0))


@pytest.mark.parametrize("dim", [16, 128, 24])
def test_f16_fp32_accumulate_mode(oracle, dim):
    from embtab import _lib

    rng = np.random.default_rng(2)
    h = rng.standard_normal((400, dim)).astype(np.float16)
    I = rng.integers(1, 401, (150, 20))
    out = torch.empty((150, dim), dtype=torch.float16, device=DEV)
    A = table(h)
    _lib.check(_lib.load().et_pooled_sum(
        _lib.ET_F16, A.columnpointer(1), A.ld, 400, dim, dev(I).data_ptr(), 20, 20, 150,
        out.data_ptr(), dim, _lib.ET_FLAG_F16_FP32_ACC, _lib.stream_handle()))
    assert bits_equal(host(out), oracle.pooled_sum(h, I, f16_fp32_acc=True))


def test_strided_destination_and_table(oracle):
    """lookup! into a column block of a wider matrix and from a padded table (ld > D)."""
    rng = np.random.default_rng(3)
    big = rng.random((300, 160), dtype=np.float32)
    h = big[:, :128]  # ld 160
    A = et.SimpleEmbedding(dev(big)[:, :128], et.Static(128))
    I = rng.integers(1, 301, (64, 20))
    dst = torch.zeros((64, 200), dtype=torch.float32, device=DEV)
    et.lookup_(dst[:, 36:164], A, dev(I))
    got = host(dst)
    assert bits_equal(got[:, 36:164], oracle.pooled_sum(np.ascontiguousarray(h), I))
    assert not got[:, :36].any() and not got[:, 164:].any()


def test_empty_and_pool_zero():
    A = table(np.ones((10, 128), np.float32))
    assert et.lookup(A, torch.zeros(0, dtype=torch.int64, device=DEV)).shape == (0, 128)
    out = et.lookup(A, torch.zeros((7, 0), dtype=torch.int64, device=DEV))
    assert out.shape == (7, 128) and not out.any()


def test_out_of_range_indices_are_counted_not_faulted():
    et.check_errors()
    A = table(np.ones((10, 128), np.float32))
    I = torch.tensor([[1, 11], [0, 3], [2, -5]], dtype=torch.int64, device=DEV)
    out = host(et.lookup(A, I))
    assert et.check_errors() == 3
    assert out[0].tolist() == [1.0] * 128  # bad rows contribute zero
    assert et.check_errors() == 0


@pytest.mark.parametrize("dim", [16, 64, 512])
def test_maplookup_strategies(oracle, dim):
    """test/map.jl:32-103 — every strategy equals reduce(vcat, map(lookup, ...)) for
    vector-of-vectors, matrix, vector-of-matrices and 3-D index containers."""
    rng = np.random.default_rng(dim)
    ntables, ncols, B, P = 10, 100, 64, 10
    hs = [rng.standard_normal((ncols, dim)).astype(np.float32) for _ in range(ntables)]
    tabs = [table(h) for h in hs]
    for shape in ((B,), (B, P)):
        hidx = [rng.integers(1, ncols + 1, shape) for _ in range(ntables)]
        ref = np.concatenate([oracle.lookup(h, i) for h, i in zip(hs, hidx)], 1)
        vec = [dev(i) for i in hidx]
        stacked = dev(np.stack(hidx))  # Julia B x T / P x B x T
        for I in (vec, stacked):
            for s in (et.DefaultStrategy(), et.SimpleParallelStrategy()):
                assert bits_equal(np.concatenate([host(o) for o in et.maplookup(s, tabs, I)], 1),
                                  ref)
            assert bits_equal(host(et.maplookup(et.PreallocationStrategy(), tabs, I)), ref)
            got = host(et.maplookup(et.PreallocationStrategy(20), tabs, I))
            assert bits_equal(got[:, 20:], ref)


def test_prealloc_mixed_dims_and_pools(oracle):
    """Tables with different dims (vector + generic kernels in one call) and pools."""
    rng = np.random.default_rng(9)
    dims = [128, 5, 128, 64, 37, 128]
    pools = [20, 3, 1, 20, 7, 0]
    hs = [rng.random((50 + 10 * t, d), dtype=np.float32) for t, d in enumerate(dims)]
    B = 100
    hidx = [rng.integers(1, h.shape[0] + 1, (B, p)) for h, p in zip(hs, pools)]
    got = host(et.maplookup(et.PreallocationStrategy(3), [table(h) for h in hs],
                            [dev(i) for i in hidx]))
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=3)
    assert bits_equal(got[:, 3:], ref[:, 3:])


def test_many_tables_split_launches(oracle):
    """More tables than fit one kernel-argument pack (32)."""
    rng = np.random.default_rng(4)
    hs = [rng.random((20, 16), dtype=np.float32) for _ in range(40)]
    hidx = [rng.integers(1, 21, (33, 4)) for _ in hs]
    got = host(et.maplookup(et.PreallocationStrategy(), [table(h) for h in hs],
                            [dev(i) for i in hidx]))
    assert bits_equal(got, oracle.maplookup_prealloc(hs, hidx))


def test_criteo_shaped_sample(oracle):
    """Config-3 shape (26 tables x 128, pool 20) at a small batch, with tables of the
    small Criteo cardinalities so the oracle check is exact and fast."""
    rng = np.random.default_rng(26)
    card = [1460, 583, 305, 24, 12517, 633, 3, 5683, 3194, 27, 14992, 10, 5652, 2173, 4,
            18, 15, 105, 1460, 583, 305, 24, 633, 3, 27, 10]
    hs = [rng.random((r, 128), dtype=np.float32) for r in card]
    hidx = [rng.integers(1, r + 1, (1000, 20)) for r in card]
    got = host(et.maplookup(et.PreallocationStrategy(), [table(h) for h in hs],
                            [dev(i) for i in hidx]))
    assert bits_equal(got, oracle.maplookup_prealloc(hs, hidx, nthreads=8))


@pytest.mark.parametrize("dtype", [np.float32, np.float16, np.float64, np.int32])
def test_tiny_tables_in_striped_launch(oracle, dtype):
    """Tiny (L1-resident) tables beside larger ones in one striped multi-table launch:
    tables around 16 KiB, a strided (ld > D) tiny table, out-of-range indices counted
    and contributing zero — all bit-identical to the oracle."""
    rng = np.random.default_rng(77)
    es = np.dtype(dtype).itemsize
    D = 64
    lim = (16 << 10) // (D * es)  # rows that fit the LDS stage
    card = [3, lim, lim + 1, 1, 700, 5, 2000]
    mk = (lambda r: rng.integers(-9, 9, (r, D)).astype(dtype)) if dtype == np.int32 else \
        (lambda r: rng.standard_normal((r, D)).astype(dtype))
    hs = [mk(r) for r in card]
    B, P = 300, 20
    hidx = [rng.integers(1, r + 1, (B, P)) for r in card]
    tabs = [table(h) for h in hs]
    wide = np.zeros((5, D + 8), dtype)  # table 5 with ld = D + 8
    wide[:, :D] = hs[5]
    tabs[5] = et.SimpleEmbedding(dev(wide)[:, :D])
    assert tabs[5].ld == D + 8
    et.check_errors()
    got = host(et.maplookup(et.PreallocationStrategy(), tabs, [dev(i) for i in hidx]))
    assert et.check_errors() == 0
    assert bits_equal(got, oracle.maplookup_prealloc(hs, hidx))
    bad = [i.copy() for i in hidx]
    bad[0][7, 3] = 4  # one past the 3-row table
    bad[1][0, 0] = 0
    got = host(et.maplookup(et.PreallocationStrategy(), tabs, [dev(i) for i in bad]))
    assert et.check_errors() == 2
    ref = oracle.maplookup_prealloc(hs, hidx)
    # a bad index contributes a zero row (x + 0 == x): its bag equals the bag without it
    for t, (j, k) in ((0, (7, 3)), (1, (0, 0))):
        bag = np.delete(hidx[t][j:j + 1], k, axis=1)
        ref[j, D * t:D * (t + 1)] = oracle.pooled_sum(hs[t], bag)[0]
    assert bits_equal(got, ref)


def test_fill_matches_oracle(oracle):
    from embtab import _lib

    L = _lib.load()
    for dtype, tdt in ((np.float32, torch.float32), (np.float16, torch.float16),
                       (np.float64, torch.float64)):
        x = torch.empty(100000, dtype=tdt, device=DEV)
        _lib.check(L.et_fill_uniform(_lib.et_dtype(x), x.data_ptr(), x.numel(), 7, 123, -1.0,
                                     1.0, _lib.stream_handle()))
        ref = oracle.fill_uniform((100000,), dtype, 7, 123, -1.0, 1.0)
        assert bits_equal(host(x), ref)
    i = torch.empty(100000, dtype=torch.int64, device=DEV)
    _lib.check(L.et_fill_index_uniform(i.data_ptr(), i.numel(), 10131227, 9, 0,
                                       _lib.stream_handle()))
    assert bits_equal(host(i), oracle.fill_index_uniform((100000,), 10131227, 9))


def test_concat_slabs():
    from embtab import _lib

    rng = np.random.default_rng(6)
    B, nranks, slab_ld = 50, 3, 12
    slabs = rng.random((nranks, B, slab_ld), dtype=np.float32)
    rows = np.array([12, 8, 4], np.int32)
    offs = np.array([2, 14, 22], np.int64)
    dst = torch.zeros((B, 26), dtype=torch.float32, device=DEV)
    _lib.check(_lib.load().et_concat_slabs(
        _lib.ET_F32, dev(slabs).data_ptr(), nranks, slab_ld, B, rows.ctypes.data,
        offs.ctypes.data, dst.data_ptr(), 26, _lib.stream_handle()))
    got = host(dst)
    for r in range(nranks):
        assert np.array_equal(got[:, offs[r]:offs[r] + rows[r]], slabs[r][:, :rows[r]])


def test_sharded_prealloc_single_rank(oracle):
    """embtab.sharding end to end on one GPU (world 1, 4 pipelined chunks on a second
    stream): fused lookup into the slab, exchange, et_concat_slabs assembly — equals
    the unsharded Preallocation."""
    from embtab.sharding import ShardedMapLookup, ShardPlan

    rng = np.random.default_rng(8)
    dims = [128] * 6
    rows = [300, 5000, 20, 800, 64, 1000]
    hs = [rng.random((r, d), dtype=np.float32) for r, d in zip(rows, dims)]
    hidx = [rng.integers(1, r + 1, (256, 20)) for r in rows]
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=4)
    for plan in (ShardPlan.tablewise(dims, 1, 4), ShardPlan.featurewise(dims, 1, 4)):
        for chunks in (1, 4):
            sp = ShardedMapLookup(plan, 0, 1, 256, torch.float32, DEV, chunks=chunks)
            dst = torch.zeros((256, plan.ld), dtype=torch.float32, device=DEV)
            sp([table(h) for h in hs], [dev(i) for i in hidx], dst)
            torch.cuda.synchronize()
            assert bits_equal(host(dst)[:, 4:], ref[:, 4:])


@pytest.mark.parametrize("exchange,chunks", [("allgather", 1), ("allgather", 4),
                                             ("alltoall", 1)])
def test_native_sharded_step_rccl_world1(oracle, exchange, chunks):
    """The C-ABI sharded step (et_sharded_create / et_sharded_maplookup, csrc/et_shard.cpp)
    with a real RCCL communicator of one rank (et_comm_unique_id / et_comm_init), so the
    ncclAllGather / ncclSend-ncclRecv calls execute: equals the unsharded Preallocation
    (src/lookup.jl:316-371) bit for bit; the all-to-all backward returns the gradient rows
    of the rank's pieces."""
    from embtab.sharding import ShardedMapLookup, ShardPlan

    rng = np.random.default_rng(81)
    dims = [128, 64, 128, 96]
    rows = [300, 5000, 20, 800]
    B, k = 300, 4
    hs = [rng.random((r, d), dtype=np.float32) for r, d in zip(rows, dims)]
    hidx = [rng.integers(1, r + 1, (B, 20)) for r in rows]
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=k)
    for plan in (ShardPlan.tablewise(dims, 1, k), ShardPlan.featurewise(dims, 1, k)):
        sm = ShardedMapLookup(plan, 0, 1, B, torch.float32, DEV, exchange=exchange,
                              chunks=chunks, rccl=True)
        assert sm._native is not None and sm._native.comm
        try:
            dst = torch.zeros((B, plan.ld), dtype=torch.float32, device=DEV)
            from embtab.sharding import piece_table
            full = [table(h) for h in hs]
            ps = plan.pieces[0]
            sm([piece_table(full[p.table], p) for p in ps], [dev(hidx[p.table]) for p in ps], dst)
            torch.cuda.synchronize()
            assert bits_equal(host(dst)[:, k:], ref[:, k:])
            if exchange == "alltoall":
                delta = dev(rng.standard_normal((B, plan.ld)).astype(np.float32))
                grads = sm.piece_grads([piece_table(full[p.table], p) for p in ps],
                                       [dev(hidx[p.table]) for p in ps], delta)
                for p, g in zip(ps, grads):
                    assert torch.equal(g.delta, delta[:, p.col:p.col + p.dim])
        finally:
            sm.close()


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float64])
def test_native_sharded_step_other_types(oracle, dtype):
    """The C-ABI sharded step exchanges bytes, so every element type goes through it:
    Float16 (Julia Float16 sums), BFloat16 and Float64 tables, feature-wise plan with
    prepended rows, 3 pipelined chunks, one-rank RCCL communicator."""
    from embtab.sharding import ShardedMapLookup, ShardPlan, piece_table

    rng = np.random.default_rng(5)
    dims, rows, B, k = [64, 128, 32], [200, 3000, 50], 257, 3
    raw = [rng.standard_normal((r, d)).astype(np.float32) for r, d in zip(rows, dims)]
    hidx = [rng.integers(1, r + 1, (B, 12)) for r in rows]
    if dtype == torch.bfloat16:
        hs = [oracle.f32_to_bf16(x) for x in raw]
        full = [et.SimpleEmbedding(dev(h).view(torch.bfloat16), et.Static(h.shape[1])) for h in hs]
    else:
        hs = [x.astype(np.float16 if dtype == torch.float16 else np.float64) for x in raw]
        full = [table(h) for h in hs]
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=k, bf16=dtype == torch.bfloat16)
    plan = ShardPlan.featurewise(dims, 1, k, elsize=torch.empty((), dtype=dtype).element_size())
    sm = ShardedMapLookup(plan, 0, 1, B, dtype, DEV, chunks=3, rccl=True)
    try:
        assert sm._native is not None
        dst = torch.zeros((B, plan.ld), dtype=dtype, device=DEV)
        ps = plan.pieces[0]
        sm([piece_table(full[p.table], p) for p in ps], [dev(hidx[p.table]) for p in ps], dst)
        torch.cuda.synchronize()
        got = host(dst.view(torch.int16)).view(np.uint16) if dtype == torch.bfloat16 else host(dst)
        assert bits_equal(got[:, k:], ref[:, k:])
    finally:
        sm.close()


def test_allgather_concat_rccl_world1():
    """et_allgather_concat on a one-rank RCCL communicator: ncclAllGather + assembly."""
    import ctypes

    from embtab import _lib

    L = _lib.load()
    idb = (ctypes.c_char * _lib.ET_COMM_ID_BYTES)()
    _lib.check(L.et_comm_unique_id(ctypes.addressof(idb)))
    comm = ctypes.c_void_p()
    _lib.check(L.et_comm_init(ctypes.byref(comm), 1, ctypes.addressof(idb), 0))
    try:
        rng = np.random.default_rng(3)
        B, slab_ld, ld = 1000, 40, 50
        slab = dev(rng.standard_normal((B, slab_ld)).astype(np.float32))
        gathered = torch.empty_like(slab)
        dst = torch.zeros((B, ld), dtype=torch.float32, device=DEV)
        rows = np.array([37], np.int32)
        offs = np.array([9], np.int64)
        _lib.check(L.et_allgather_concat(comm, _lib.ET_F32, slab.data_ptr(), slab_ld, B,
                                         gathered.data_ptr(), 1, rows.ctypes.data,
                                         offs.ctypes.data, dst.data_ptr(), ld,
                                         _lib.stream_handle()))
        torch.cuda.synchronize()
        assert torch.equal(gathered, slab)
        assert torch.equal(dst[:, 9:46], slab[:, :37])
        assert not dst[:, :9].any() and not dst[:, 46:].any()
    finally:
        _lib.check(L.et_comm_destroy(comm))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_pieces_simulated_ranks(oracle, world):
    """Feature-sharded plans on the real kernels: every simulated rank looks up its
    pieces (column-slice views, widths 32/64/96/128...) into its slab; the stacked
    slabs are assembled by et_concat_slabs — bit-identical to the unsharded lookup."""
    from embtab.sharding import ShardedMapLookup, ShardPlan, piece_table

    rng = np.random.default_rng(world)
    dims = [128] * 5 + [64, 256, 48]
    rows = [300, 5000, 20, 800, 64, 1000, 77, 129]
    B, k = 200, 3
    hs = [rng.random((r, d), dtype=np.float32) for r, d in zip(rows, dims)]
    hidx = [rng.integers(1, r + 1, (B, 20)) for r in rows]
    full = [table(h) for h in hs]
    didx = [dev(i) for i in hidx]
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=k)
    for plan in (ShardPlan.featurewise(dims, world, k),
                 ShardPlan.tablewise(dims, world, k, sizes=rows)):
        slabs = []
        for r in range(world):
            sm = ShardedMapLookup(plan, r, world, B, torch.float32, DEV)
            ps = plan.pieces[r]
            sm.lookup_chunk([piece_table(full[p.table], p) for p in ps],
                            [didx[p.table] for p in ps], 0, B)
            slabs.append(sm.slab)
        dst = torch.zeros((B, plan.ld), dtype=torch.float32, device=DEV)
        sm.assemble_chunk(torch.stack(slabs), dst)
        torch.cuda.synchronize()
        assert bits_equal(host(dst)[:, k:], ref[:, k:])


def test_split_slabs_inverts_concat():
    """et_split_slabs(et_concat_slabs(slabs)) == slabs on the covered columns."""
    from embtab import _lib
    import ctypes

    rng = np.random.default_rng(12)
    B, nranks, slab_ld, ld = 77, 3, 12, 30
    rows = np.array([12, 7, 5], np.int32)
    offs = np.array([1, 13, 22], np.int64)
    mat = dev(rng.standard_normal((B, ld)).astype(np.float32))
    slabs = torch.zeros((nranks, B, slab_ld), dtype=torch.float32, device=DEV)
    L = _lib.load()
    _lib.check(L.et_split_slabs(_lib.ET_F32, mat.data_ptr(), ld, B, nranks, rows.ctypes.data,
                                offs.ctypes.data, slabs.data_ptr(), slab_ld,
                                _lib.stream_handle()))
    for r in range(nranks):
        assert torch.equal(slabs[r, :, :rows[r]], mat[:, offs[r]:offs[r] + rows[r]])
    back = torch.zeros_like(mat)
    _lib.check(L.et_concat_slabs(_lib.ET_F32, slabs.data_ptr(), nranks, slab_ld, B,
                                 rows.ctypes.data, offs.ctypes.data, back.data_ptr(), ld,
                                 _lib.stream_handle()))
    cov = np.zeros(ld, bool)
    for r in range(nranks):
        cov[offs[r]:offs[r] + rows[r]] = True
    assert torch.equal(back[:, torch.from_numpy(cov).to(DEV)], mat[:, torch.from_numpy(cov).to(DEV)])


@pytest.mark.parametrize("exact", [True, False])
def test_sharded_training_step_simulated_ranks(oracle, exact):
    """Forward on 4 simulated feature-sharded ranks, then every rank's local update of
    its pieces from the gradient's column views: the union equals the unsharded
    multi-table update bit for bit (a feature slice's SGD is independent of the others)."""
    from embtab.sharding import ShardedMapLookup, ShardPlan, piece_table

    rng = np.random.default_rng(44)
    # dim 50 (not a multiple of 4) takes the generic kernels as a whole table, while its
    # 32-feature slice takes the vector ones: both combine > 8 partials identically
    dims, rows, B, P = [128, 128, 64, 128, 50], [3000, 40, 700, 9000, 900], 512, 20
    hs = [rng.standard_normal((r, d)).astype(np.float32) for r, d in zip(rows, dims)]
    hidx = [rng.integers(1, r + 1, (B, P)) for r in rows]
    hidx[1][:, :5] = 2  # a hot column (2560 occurrences)
    hidx[4][:, :5] = 3  # and one in the generic-path table
    didx = [dev(i) for i in hidx]
    delta = dev(rng.standard_normal((B, sum(dims))).astype(np.float32))
    ref = [et.SimpleEmbedding(dev(h), et.Static(h.shape[1])) for h in hs]
    offs = np.cumsum([0] + dims[:-1])
    et.update_(et.Descent(0.1), ref, [et.SparseEmbeddingUpdate(t.lookup_type,
                                                               delta[:, o:o + d], i)
                                      for t, o, d, i in zip(ref, offs, dims, didx)],
               [et.Indexer() for _ in ref], exact=exact)
    full = [et.SimpleEmbedding(dev(h), et.Static(h.shape[1])) for h in hs]
    world = 4
    plan = ShardPlan.featurewise(dims, world)
    for r in range(world):
        sm = ShardedMapLookup(plan, r, world, B, torch.float32, DEV)
        ps = plan.pieces[r]
        ptabs = [piece_table(full[p.table], p) for p in ps]
        pidx = [didx[p.table] for p in ps]
        grads = sm.piece_grads(ptabs, pidx, delta)
        et.update_(et.Descent(0.1), ptabs, grads, [et.Indexer() for _ in ptabs], exact=exact)
    for a, b in zip(full, ref):
        assert torch.equal(a.data, b.data)


@pytest.mark.parametrize("src,dst", [("f16", torch.float32), ("f32", torch.float16),
                                     ("bf16", torch.float32), ("f32", torch.bfloat16),
                                     ("f64", torch.float32)])
def test_preallocation_eltype_conversion(oracle, src, dst):
    """PreallocationStrategy{U} (src/lookup.jl:284-315): sums in the table type, then
    one conversion to the destination type U on the store."""
    rng = np.random.default_rng(17)
    dims, rows, B, P, k = [64, 40, 128], [300, 50, 1000], 200, 12, 3
    raw = [rng.standard_normal((r, d)).astype(np.float32) for r, d in zip(rows, dims)]
    if src == "bf16":
        hs = [oracle.f32_to_bf16(x) for x in raw]
        tabs = [et.SimpleEmbedding(dev(h).view(torch.bfloat16)) for h in hs]
    else:
        npt = {"f16": np.float16, "f32": np.float32, "f64": np.float64}[src]
        hs = [x.astype(npt) for x in raw]
        tabs = [et.SimpleEmbedding(dev(h)) for h in hs]
    hidx = [rng.integers(1, r + 1, (B, P)) for r in rows]
    out = et.maplookup(et.PreallocationStrategy(k, eltype=dst), tabs, [dev(i) for i in hidx])
    assert out.dtype == dst and out.shape == (B, k + sum(dims))
    ref_t = oracle.maplookup_prealloc(hs, hidx, prependrows=k, bf16=src == "bf16")[:, k:]
    as32 = oracle.bf16_to_f32(ref_t) if src == "bf16" else ref_t.astype(np.float64)
    if dst == torch.float32:
        ref = np.asarray(as32, np.float32)
        got = host(out[:, k:])
    elif dst == torch.float16:
        ref = np.asarray(as32, np.float32).astype(np.float16).view(np.uint16)
        got = host(out[:, k:].view(torch.int16)).view(np.uint16)
    else:
        ref = oracle.f32_to_bf16(np.asarray(as32, np.float32))
        got = host(out[:, k:].view(torch.int16)).view(np.uint16)
    assert bits_equal(got, ref)


def test_preallocation_plan_reuse(oracle):
    """PreallocationPlan: descriptors built once; refilling the index buffers in place
    and calling again gives the new result (same kernels as maplookup!)."""
    rng = np.random.default_rng(23)
    dims, rows, B, P, k = [128, 64, 40, 128], [5000, 300, 77, 1000], 256, 20, 2
    hs = [rng.standard_normal((r, d)).astype(np.float32) for r, d in zip(rows, dims)]
    tabs = [et.SimpleEmbedding(dev(h), et.Static(h.shape[1])) for h in hs]
    tabs[3] = et.SplitEmbedding(dev(hs[3]), 100)
    idx = [dev(rng.integers(1, r + 1, (B, P))) for r in rows]
    dst = torch.zeros((B, k + sum(dims)), dtype=torch.float32, device=DEV)
    plan = et.PreallocationPlan(et.PreallocationStrategy(k), dst, tabs, idx)
    for it in range(3):
        hidx = [rng.integers(1, r + 1, (B, P)) for r in rows]
        for d, h in zip(idx, hidx):
            d.copy_(torch.from_numpy(h))
        assert plan() is dst
        ref = oracle.maplookup_prealloc(hs, hidx, prependrows=k)
        assert bits_equal(host(dst[:, k:]), ref[:, k:])
    # graph-captured plan replay sees refilled indices too
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        plan()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        plan()
    hidx = [rng.integers(1, r + 1, (B, P)) for r in rows]
    for d, h in zip(idx, hidx):
        d.copy_(torch.from_numpy(h))
    g.replay()
    torch.cuda.synchronize()
    assert bits_equal(host(dst[:, k:]), oracle.maplookup_prealloc(hs, hidx, prependrows=k)[:, k:])
    # a half-precision destination through the same plan type
    dst16 = torch.zeros((B, k + sum(dims)), dtype=torch.float16, device=DEV)
    et.PreallocationPlan(et.PreallocationStrategy(k), dst16, tabs, idx)()
    ref16 = oracle.maplookup_prealloc(hs, hidx, prependrows=k)[:, k:].astype(np.float16)
    assert bits_equal(host(dst16[:, k:]), ref16)
    with pytest.raises(et.ArgumentError):
        et.PreallocationPlan(et.PreallocationStrategy(k), dst[:, :100], tabs, idx)


@pytest.mark.parametrize("dtype,dim", [(np.float32, 128), (np.float16, 256), (np.float64, 64),
                                       (np.int64, 64), (np.float32, 64), (np.float16, 128),
                                       (np.float64, 32)])
def test_scalar_addressed_rows(oracle, dtype, dim):
    """512-byte rows take the scalar-addressed kernel (two bags per wave, index lists read
    with scalar loads, row addresses on the scalar ALU); 256-byte rows the per-lane loop
    beside it.  Batches that are not a multiple of the bags per wave (the last wave
    re-runs its first bag in the spare groups), pools that exercise every batch size,
    single-table and striped multi-table launches, and out-of-range indices —
    including one whose low word is in range (2^32 + 1) — must match the oracle bit
    for bit, with bad indices counted and contributing zero rows."""
    rng = np.random.default_rng(512 + dim)
    mk = (lambda r: rng.integers(-99, 99, (r, dim)).astype(dtype)) if dtype == np.int64 else \
        (lambda r: rng.standard_normal((r, dim)).astype(dtype))
    card = [7, 300, 1, 4099, 50]
    pools = [1, 2, 13, 20, 33]
    hs = [mk(r) for r in card]
    tabs = [table(h) for h in hs]
    for B in (1, 3, 6, 257):
        hidx = [rng.integers(1, r + 1, (B, p)) for r, p in zip(card, pools)]
        et.check_errors()
        got = host(et.maplookup(et.PreallocationStrategy(5), tabs, [dev(i) for i in hidx]))
        assert et.check_errors() == 0
        assert bits_equal(got[:, 5:], oracle.maplookup_prealloc(hs, hidx, prependrows=5)[:, 5:])
        for h, A, i in zip(hs, tabs, hidx):  # single-table launches (k_pooled_vec)
            assert bits_equal(host(et.lookup(A, dev(i))), oracle.lookup(h, i))
    # out-of-range indices: first entry of a bag, mid-batch, in the second bag of a wave,
    # and a value whose low 32 bits alone would look valid
    B = 9
    hidx = [rng.integers(1, r + 1, (B, p)) for r, p in zip(card, pools)]
    bad = [i.copy() for i in hidx]
    edits = [(2, 0, 0, 0), (3, 4, 9, card[3] + 1), (4, 1, 20, -3), (3, 7, 0, (1 << 32) + 1),
             (1, 8, 1, 301)]
    for t, j, k, v in edits:
        bad[t][j, k] = v
    et.check_errors()
    got = host(et.maplookup(et.PreallocationStrategy(), tabs, [dev(i) for i in bad]))
    assert et.check_errors() == len(edits)
    ref = oracle.maplookup_prealloc(hs, hidx)
    for t, j, k, _ in edits:
        keep = np.delete(hidx[t][j:j + 1], k, axis=1)
        ref[j, dim * t:dim * (t + 1)] = (oracle.pooled_sum(hs[t], keep)[0] if keep.size
                                         else np.zeros(dim, dtype))
    assert bits_equal(got, ref)


@pytest.mark.parametrize("B", [1, 3, 257, 2000])
def test_striped_heavy_and_light_tables(oracle, B):
    """Heavy tables (> 4 MiB, one above the 256 MiB non-temporal threshold) beside light
    ones in one striped scalar-addressed launch, odd batches (the last chunk of every
    table ends early), out-of-range indices counted — bit-identical to the oracle."""
    rng = np.random.default_rng(1000 + B)
    card = [530_000, 9000, 7, 300, 1, 4099, 50, 20_000, 3]
    hs = [rng.random((r, 128), dtype=np.float32) for r in card]
    tabs = [table(h) for h in hs]
    P = 13
    hidx = [rng.integers(1, r + 1, (B, P)) for r in card]
    et.check_errors()
    got = host(et.maplookup(et.PreallocationStrategy(2), tabs, [dev(i) for i in hidx]))
    assert et.check_errors() == 0
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=2, nthreads=8)
    assert bits_equal(got[:, 2:], ref[:, 2:])
    bad = [i.copy() for i in hidx]
    edits = [(0, B - 1, 12, card[0] + 1), (2, 0, 0, 0), (7, B // 2, 5, -1)]
    for t, j, k, v in edits:
        bad[t][j, k] = v
    got = host(et.maplookup(et.PreallocationStrategy(2), tabs, [dev(i) for i in bad]))
    assert et.check_errors() == len(edits)
    for t, j, k, _ in edits:
        keep = np.delete(hidx[t][j:j + 1], k, axis=1)
        ref[j, 2 + 128 * t:2 + 128 * (t + 1)] = oracle.pooled_sum(hs[t], keep)[0]
    assert bits_equal(got[:, 2:], ref[:, 2:])
