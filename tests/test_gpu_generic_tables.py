"""User-defined table types that implement only the reference's plug-in contract —
``size`` / ``columnpointer`` / ``example`` (README.md:288-307) — on the HIP path.

Mirrors test/constructors.jl:34-54 (DummyEmbedding: a wrapper whose columnpointer
forwards to a plain matrix) and goes further: tables whose columns sit in arbitrary
order and at arbitrary (element-aligned) addresses, which the engine describes as a
device array of column pointers (``cols_per_page = 1``).  Every lookup, Preallocation
maplookup and Descent update is bit-identical to the oracle run on the dense table."""
import numpy as np
import pytest
import torch

import embtab as et
from embtab.tables import AbstractEmbeddingTable, Dynamic, Static

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


def host(x):
    return x.cpu().numpy()


def bits_equal(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


class DummyEmbedding(AbstractEmbeddingTable):
    """test/constructors.jl:34-45: size / columnpointer / example forwarded to a matrix."""

    def __init__(self, data, lookup_type=Dynamic):
        self.data = data
        self.lookup_type = lookup_type

    def size(self):
        return (int(self.data.shape[1]), int(self.data.shape[0]))

    def columnpointer(self, i, ctx=None):
        return et.columnpointer(self.data, i)

    def example(self):
        return self.data


class ScatteredEmbedding(AbstractEmbeddingTable):
    """Column i lives at slot perm[i] of a pool whose slots are `pitch` bytes apart —
    no uniform spacing, so the engine needs the column-pointer form."""

    def __init__(self, cols: np.ndarray, pitch_elems: int, rng, lookup_type=Dynamic):
        R, D = cols.shape
        self.R, self.D = R, D
        self.perm = rng.permutation(R)
        pool = np.zeros((R, pitch_elems), cols.dtype)
        pool[self.perm, :D] = cols
        self.pool = dev(pool.reshape(-1))  # flat buffer: slot k at k * pitch_elems
        self.pitch = pitch_elems
        self.lookup_type = lookup_type

    def size(self):
        return (self.D, self.R)

    def columnpointer(self, i, ctx=None):
        es = self.pool.element_size()
        return self.pool.data_ptr() + int(self.perm[i - 1]) * self.pitch * es

    def example(self):
        return self.pool[:self.D].view(1, self.D)

    def dense(self):
        flat = host(self.pool).reshape(self.R, self.pitch)
        return flat[self.perm, :self.D]


def test_dummy_embedding_constructors_jl(oracle):
    """test/constructors.jl:47-54: a 10 x 10 Float32 DummyEmbedding, lookup with a
    10 x 10 index matrix (and a vector) — equal to the oracle on its matrix."""
    rng = np.random.default_rng(47)
    h = rng.standard_normal((10, 10)).astype(np.float32)
    A = DummyEmbedding(dev(h))
    I = rng.integers(1, 11, (10, 10))
    assert A.device_table()[1] == 0 and A.ld == 10  # equally spaced: contiguous form
    assert bits_equal(host(et.lookup(A, dev(I))), oracle.lookup(h, I))
    v = rng.integers(1, 11, 25)
    assert bits_equal(host(et.lookup(A, dev(v))), oracle.lookup(h, v))


@pytest.mark.parametrize("dim,pitch", [(128, 128 + 4), (128, 128 + 1), (50, 53), (16, 20)])
def test_scattered_columns_lookup_and_update(oracle, dim, pitch):
    """Arbitrary column addresses: 16-byte aligned pointers (pitch 132 fp32) keep the
    vector kernels, unaligned ones (pitch 129, 53) take the generic ones; lookups,
    a Preallocation maplookup mixed with SimpleEmbeddings, and multi-table / single-table
    Descent updates are bit-identical to the oracle on the dense tables."""
    rng = np.random.default_rng(dim * 1000 + pitch)
    R, B, P = 700, 256, 20
    cols = rng.standard_normal((R, dim)).astype(np.float32)
    S = ScatteredEmbedding(cols, pitch, rng, Static(dim))
    assert S.device_table()[1] == 1  # column-pointer form
    assert bits_equal(S.dense(), cols)
    I = rng.integers(1, R + 1, (B, P))
    assert bits_equal(host(et.lookup(S, dev(I))), oracle.pooled_sum(cols, I))
    v = rng.integers(1, R + 1, 300)
    assert bits_equal(host(et.lookup(S, dev(v))), oracle.gather(cols, v))
    # Preallocation over [Simple, Scattered, Simple]
    h0 = rng.standard_normal((300, 64)).astype(np.float32)
    h2 = rng.standard_normal((90, dim)).astype(np.float32)
    tabs = [et.SimpleEmbedding(dev(h0), Static(64)), S, et.SimpleEmbedding(dev(h2), Static(dim))]
    hidx = [rng.integers(1, 301, (B, P)), I, rng.integers(1, 91, (B, P))]
    y, back = et.rrule(et.maplookup, et.PreallocationStrategy(3), tabs, [dev(i) for i in hidx])
    ref = oracle.maplookup_prealloc([h0, cols, h2], hidx, prependrows=3)
    assert bits_equal(host(y)[:, 3:], ref[:, 3:])
    # multi-table update (the scattered table in the middle of the pipeline)
    delta = rng.standard_normal(tuple(y.shape)).astype(np.float32)
    grads = back(dev(delta))[2]
    et.update_(et.Descent(0.1), tabs, grads, [et.Indexer() for _ in tabs])
    refs = [h0.copy(), cols.copy(), h2.copy()]
    offs = [3, 3 + 64, 3 + 64 + dim]
    for r, i, o, d in zip(refs, hidx, offs, (64, dim, dim)):
        oracle.sgd(r, np.ascontiguousarray(delta[:, o:o + d]), i, 0.1, fused=True)
    assert bits_equal(host(tabs[0].data), refs[0])
    assert bits_equal(S.dense(), refs[1])
    assert bits_equal(host(tabs[2].data), refs[2])
    # single-table update and an IndexerView update on the same table
    d1 = rng.standard_normal((300, dim)).astype(np.float32)
    g = et.SparseEmbeddingUpdate(S.lookup_type, dev(d1), dev(v))
    et.update_(et.Descent(0.5), S, g)
    oracle.sgd(refs[1], d1, v, 0.5, fused=True)
    assert bits_equal(S.dense(), refs[1])
    ix = et.index_(et.Indexer(), g.indices, R)
    for s in range(1, 5):
        et.update_(S, g, et.IndexerView(ix, 4, s), 0.25)
    oracle.sgd(refs[1], d1, v, 0.25, fused=True)
    assert bits_equal(S.dense(), refs[1])
    assert et.check_errors() == 0
