"""Paged tables (the reference's SplitEmbedding, src/split.jl) on the HIP path.

Mirrors test/lookup.jl:110-139 ("Testing Standard Split" / "Testing Reducing Split":
dims 32..1504, 1000 columns, chunk sizes 10..50, permutations and repeats, 12 lookups
per output): every result is bit-identical to the oracle run on the dense table.
The update cases check that a paged table receives exactly the dense update."""
import numpy as np
import pytest
import torch

import embtab as et
from embtab.tables import fused_update_path

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
NROWS = [32, 64, 128, 256, 512, 1024, 1504]  # test/lookup.jl:66
CHUNKS = [10, 20, 30, 40, 50]                 # test/lookup.jl:111


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


def host(x):
    return x.cpu().numpy()


def bits_equal(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


@pytest.mark.parametrize("dim", NROWS)
def test_split_lookup_parity(oracle, dim):
    rng = np.random.default_rng(1000 + dim)
    ncols = 1000
    base = rng.random((ncols, dim), dtype=np.float32)
    for cps in CHUNKS:
        A = et.SplitEmbedding(dev(np.zeros_like(base)), cps)
        A.copy_(dev(base))                       # table .= base
        assert A.size() == (dim, ncols) and len(A) == dim * ncols
        assert bits_equal(host(A.to_dense()), base)  # table == baseline
        # non_reducing_lookup: permutation, then repeats
        for I in (rng.permutation(ncols) + 1, rng.integers(1, ncols + 1, ncols)):
            assert bits_equal(host(et.lookup(A, dev(I))), oracle.lookup(base, I))
        # reducing_lookup: 12 lookups per output, no repeats within a row, then repeats
        for I in (np.stack([rng.permutation(np.arange(2, ncols + 1)) for _ in range(12)], 1),
                  rng.integers(1, ncols + 1, (ncols, 12))):
            assert bits_equal(host(et.lookup(A, dev(I))), oracle.lookup(base, I))


def test_split_ragged_last_page_and_dtypes(oracle):
    rng = np.random.default_rng(3)
    for dtype, dim in ((np.float64, 24), (np.int64, 16), (np.float16, 40), (np.float32, 7)):
        ncols = 101  # 101 = 3 pages of 33 + one page of 2
        base = (rng.integers(-50, 50, (ncols, dim)).astype(dtype) if dtype == np.int64
                else rng.standard_normal((ncols, dim)).astype(dtype))
        A = et.SplitEmbedding(dev(base), 33)
        assert len(A.pages) == 4 and A.pages[-1].shape[0] == 2
        I = rng.integers(1, ncols + 1, (64, 9))
        assert bits_equal(host(et.lookup(A, dev(I))), oracle.pooled_sum(base, I))
        v = rng.integers(1, ncols + 1, 77)
        assert bits_equal(host(et.lookup(A, dev(v))), oracle.gather(base, v))


def test_split_in_preallocation(oracle):
    """A paged table among contiguous ones in one fused PreallocationStrategy launch."""
    rng = np.random.default_rng(5)
    B, P, k = 300, 20, 2
    hs = [rng.standard_normal((r, d)).astype(np.float32)
          for r, d in ((500, 128), (900, 128), (77, 64), (300, 40))]
    tabs = [et.SimpleEmbedding(dev(hs[0]), et.Static(128)), et.SplitEmbedding(dev(hs[1]), 50),
            et.SplitEmbedding(dev(hs[2]), 10), et.SimpleEmbedding(dev(hs[3]))]
    hidx = [rng.integers(1, h.shape[0] + 1, (B, P)) for h in hs]
    got = host(et.maplookup(et.PreallocationStrategy(k), tabs, [dev(i) for i in hidx]))
    ref = oracle.maplookup_prealloc(hs, hidx, prependrows=k)
    assert bits_equal(got[:, k:], ref[:, k:])


@pytest.mark.parametrize("dim,cps", [(64, 10), (128, 37), (256, 50), (80, 20)])
@pytest.mark.parametrize("exact", [True, False])
def test_split_update_vs_oracle(oracle, dim, cps, exact):
    """update!(Descent) on a paged table == the oracle's update of the dense table
    (SplitEmbedding is Static{D}: fused path when D*4 <= 512, generic otherwise)."""
    rng = np.random.default_rng(dim + cps)
    ncols, B, P = 1000, 512, 10
    base = rng.standard_normal((ncols, dim)).astype(np.float32)
    I = rng.integers(1, ncols + 1, (B, P))
    delta = rng.standard_normal((B, dim)).astype(np.float32)
    A = et.SplitEmbedding(dev(base), cps)
    g = et.SparseEmbeddingUpdate(A.lookup_type, dev(delta), dev(I))
    et.update_(et.Descent(0.5), A, g, exact=exact)
    ref = base.copy()
    oracle.sgd(ref, delta, I, 0.5, fused=fused_update_path(A))
    assert bits_equal(host(A.to_dense()), ref)  # no column has > ET_SGD_CHUNK occurrences here


def test_split_update_dynamic_and_indexer_view(oracle):
    rng = np.random.default_rng(9)
    ncols, dim = 200, 48
    base = rng.standard_normal((ncols, dim)).astype(np.float32)
    delta = rng.standard_normal((256, dim)).astype(np.float32)
    I = rng.integers(1, ncols + 1, 256)
    # undef constructor with a Dynamic lookup type -> the generic (unfused) update
    A = et.SplitEmbedding.undef(dim, ncols, 30, torch.float32, DEV, et.Dynamic)
    A.copy_(dev(base))
    et.update_(et.Descent(0.25), A, et.SparseEmbeddingUpdate(A.lookup_type, dev(delta), dev(I)))
    ref = base.copy()
    oracle.sgd(ref, delta, I, 0.25, fused=False)
    assert bits_equal(host(A.to_dense()), ref)
    # 4 IndexerView splits on a paged table == the unsplit update (test/update.jl:90-120)
    A = et.SplitEmbedding(dev(base), 30)
    g = et.SparseEmbeddingUpdate(A.lookup_type, dev(delta), dev(I))
    ix = et.index_(et.Indexer(), g.indices, ncols)
    for s in range(1, 5):
        et.update_(A, g, et.IndexerView(ix, 4, s), 1.0)
    ref = base.copy()
    oracle.sgd(ref, delta, I, 1.0, fused=True)
    assert bits_equal(host(A.to_dense()), ref)


def test_split_multi_table_update(oracle):
    """Multi-table update! with paged and contiguous tables in one pipeline."""
    rng = np.random.default_rng(21)
    k, B, P = 4, 256, 20
    dims, rows = (128, 128, 64), (300, 1000, 50)
    hs = [rng.standard_normal((r, d)).astype(np.float32) for r, d in zip(rows, dims)]
    tabs = [et.SplitEmbedding(dev(hs[0]), 40), et.SimpleEmbedding(dev(hs[1]), et.Static(128)),
            et.SplitEmbedding(dev(hs[2]), 10)]
    hidx = [rng.integers(1, r + 1, (B, P)) for r in rows]
    y, back = et.rrule(et.maplookup, et.PreallocationStrategy(k), tabs, [dev(i) for i in hidx])
    delta = rng.standard_normal(tuple(y.shape)).astype(np.float32)
    grads = back(dev(delta))[2]
    et.update_(et.Descent(0.1), tabs, grads, [et.Indexer() for _ in tabs])
    refs = [h.copy() for h in hs]
    offs = np.cumsum([k] + list(dims[:-1]))
    oracle.sgd_multi(refs, delta, hidx, 0.1, [fused_update_path(t) for t in tabs], num_splits=4,
                     nthreads=4, delta_offsets=offs)
    got = [host(tabs[0].to_dense()), host(tabs[1].data), host(tabs[2].to_dense())]
    for t in range(3):
        assert bits_equal(got[t], refs[t])
