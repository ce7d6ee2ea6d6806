"""Host-side mirror of the reference API that runs without a GPU: constructors
(test/constructors.jl), dispatch rules, index containers, IndexerView ranges, and
that the product path refuses to compute on the CPU (no silent fallback)."""
import collections
import pytest
import torch

import embtab as et


def test_constructors():
    """test/constructors.jl:1-25."""
    even = torch.rand(10, 64)  # Julia 64 x 10
    odd = torch.rand(10, 65)
    x = et.SimpleEmbedding(even, et.Static(64))
    assert x.size() == (64, 10)
    with pytest.raises(et.ArgumentError):
        et.SimpleEmbedding(even, et.Static(32))
    with pytest.raises(et.ArgumentError):
        et.Static(64.0)
    x = et.SimpleEmbedding(odd)
    assert x.size() == (65, 10) and x.lookup_type is et.Dynamic
    x = et.SimpleEmbedding(odd, et.Static(65))
    assert x.lookup_type == et.Static(65)


def test_columnpointer_and_example():
    data = torch.rand(10, 16)
    A = et.SimpleEmbedding(data, et.Static(16))
    assert A.columnpointer(1) == data.data_ptr()
    assert A.columnpointer(3) == data.data_ptr() + 2 * 16 * 4
    assert et.example(A) is data and et.featuresize(A) == 16
    assert et.example([A]) is data
    assert A[2, 3] == pytest.approx(float(data[2, 1]))
    A[2, 3] = 5.0
    assert float(data[2, 1]) == 5.0


def test_fused_path_dispatch_rule():
    """src/sparseupdate.jl:131-154: specialized iff Static and N*sizeof(T) <= 512."""
    from embtab.tables import fused_update_path

    assert fused_update_path(et.SimpleEmbedding(torch.rand(3, 128), et.Static(128)))
    assert not fused_update_path(et.SimpleEmbedding(torch.rand(3, 256), et.Static(256)))
    assert not fused_update_path(et.SimpleEmbedding(torch.rand(3, 128)))


def test_colwrap():
    I = torch.arange(2 * 5 * 3).reshape(3, 5, 2)  # Julia 2 x 5 x 3
    parts = et.colwrap(I)
    assert len(parts) == 3 and parts[1].shape == (5, 2)
    assert et.colwrap([I[0], I[1]])[1] is I[1] or torch.equal(et.colwrap([I[0], I[1]])[1], I[1])


def test_indexer_view_ranges():
    """src/utils.jl:325-333 on an Indexer with U = 6 distinct columns (7 cumulative)."""
    ix = et.Indexer()
    ix.cumulative = torch.zeros((7, 2), dtype=torch.int64)
    ranges = [et.IndexerView(ix, 4, s).entries() for s in range(1, 5)]
    assert ranges == [(0, 2), (2, 4), (4, 6), (6, 6)]
    covered = [e for b, f in ranges for e in range(b, f)]
    assert covered == list(range(6))


def test_no_cpu_fallback():
    """The product path computes on the GPU only: CPU tensors are refused loudly."""
    A = et.SimpleEmbedding(torch.rand(10, 16), et.Static(16))
    with pytest.raises(et.ArgumentError):
        et.lookup(A, torch.tensor([1, 2, 3]))


def test_split_embedding_host_logic():
    """src/split.jl:11-86: pages of cols_per_shard columns (last one short), Static{D},
    size, columnpointer through _divrem_index, getindex/setindex!, undef constructor."""
    data = torch.rand(23, 8)  # Julia 8 x 23
    A = et.SplitEmbedding(data, 5)
    assert [p.shape[0] for p in A.pages] == [5, 5, 5, 5, 3]
    assert A.size() == (8, 23) and len(A) == 8 * 23
    assert A.lookup_type == et.Static(8) and A.ld == 8 and A.cols_per_page == 5
    assert torch.equal(A.to_dense(), data)
    assert all(p.data_ptr() != data.data_ptr() for p in A.pages)  # copies, like the reference
    # column 12 -> page 3, column 2 (1-based): _divrem_index(12, 5) == (3, 2)
    assert A.columnpointer(12) == A.pages[2].data_ptr() + 1 * 8 * 4
    assert A.columnpointer(23) == A.pages[4].data_ptr() + 2 * 8 * 4
    with pytest.raises(IndexError):
        A.columnpointer(26)
    assert A[3, 12] == pytest.approx(float(data[11, 2]))
    A[3, 12] = -7.0
    assert float(A.pages[2][1, 2]) == -7.0
    table, cpp = A.device_table()
    assert table == A.page_table.data_ptr() and cpp == 5
    assert A.page_table.tolist() == [p.data_ptr() for p in A.pages]
    assert et.SimpleEmbedding(data).device_table() == (data.data_ptr(), 0)
    U = et.SplitEmbedding.undef(16, 10, 4, torch.float32, "cpu", et.Dynamic)
    assert U.size() == (16, 10) and U.lookup_type is et.Dynamic
    assert [p.shape for p in U.pages] == [(4, 16), (4, 16), (2, 16)]
    with pytest.raises(et.ArgumentError):
        et.SplitEmbedding.undef(16, 10, 4, lookup_type=et.Static(8))
    with pytest.raises(et.ArgumentError):
        et.SplitEmbedding(data, 0)
    with pytest.raises(et.ArgumentError):
        et.lookup(A, torch.tensor([1, 2, 3]))  # no CPU fallback for paged tables either


def test_update_workspaces_are_per_stream(monkeypatch):
    """Round 6: the update's cached workspace is per (key, device, stream) — two streams never
    share one (concurrent updates on two streams corrupted a shared one), one stream reuses its
    own, and a larger request replaces it (CPU stand-in for the device and the streams)."""
    from embtab import _lib, update

    cur = {"s": 1}
    monkeypatch.setattr(_lib, "stream_handle", lambda device=None: cur["s"])
    monkeypatch.setattr(update, "_ws_cache", collections.OrderedDict())
    dev = torch.device("cpu")
    a = update._workspace(1000, dev, "sgd")
    assert update._workspace(900, dev, "sgd") is a
    cur["s"] = 2
    b = update._workspace(1000, dev, "sgd")
    assert b is not a and b.data_ptr() != a.data_ptr()
    cur["s"] = 1
    assert update._workspace(1000, dev, "sgd") is a
    c = update._workspace(5000, dev, "sgd")
    assert c is not a and c.numel() >= 5000
    assert update._workspace(1000, dev, "index") is not c
    # bounded: only the _WS_STREAMS most recently used streams per (key, device) keep theirs
    for st in range(10, 10 + update._WS_STREAMS):
        cur["s"] = st
        update._workspace(1000, dev, "sgd")
    sgd = [k for k in update._ws_cache if k[0] == "sgd"]
    assert len(sgd) == update._WS_STREAMS and (("sgd", "cpu", 1)) not in sgd
    assert ("index", "cpu", 1) in update._ws_cache  # another key keeps its own
