"""The CPU oracle pinned against the reference's own known-answer tests, and its
algorithms cross-checked against the naive restatement (CPU only).

KATs: README.md:32-73, README.md:115-159, README.md:191-228, test/misc.jl:2-110.
Property tests mirror test/lookup.jl, test/map.jl and test/update.jl.
"""
import numpy as np
import pytest


def cols_to_rows(cols, dtype):
    """Julia column list -> (N, D) row-per-column array (our layout)."""
    return np.asarray(cols, dtype=dtype)


# --- KATs ----------------------------------------------------------------------------

def test_readme_lookup_kat(oracle, kat):
    k = kat["readme_lookup"]
    A = cols_to_rows(k["table_columns"], np.int64)
    got = oracle.lookup(A, np.array(k["vector_indices"]))
    assert np.array_equal(got, cols_to_rows(k["vector_expected_columns"], np.int64))
    got = oracle.lookup(A, np.array(k["matrix_indices_bags"]))
    assert np.array_equal(got, cols_to_rows(k["matrix_expected_columns"], np.int64))


def test_readme_maplookup_kat(oracle, kat):
    k = kat["readme_maplookup"]
    A = cols_to_rows(k["A_columns"], np.int64)
    B = cols_to_rows(k["B_columns"], np.int64)
    iA, iB = np.array(k["iA"]), np.array(k["iB"])
    assert np.array_equal(oracle.lookup(A, iA), cols_to_rows(k["expected_A_columns"], np.int64))
    assert np.array_equal(oracle.lookup(B, iB), cols_to_rows(k["expected_B_columns"], np.int64))
    # PreallocationStrategy == reduce(vcat, maplookup(...)) (README.md:165-167)
    cat = oracle.maplookup_prealloc([A, B], [iA, iB])
    assert np.array_equal(cat, np.concatenate([oracle.lookup(A, iA), oracle.lookup(B, iB)], 1))


@pytest.mark.parametrize("fused", [False, True])
def test_readme_update_kat(oracle, kat, fused):
    k = kat["readme_update"]
    t = np.zeros((k["ncols"], k["nrows"]), np.float32)
    delta = cols_to_rows(k["delta_columns"], np.float32)
    oracle.sgd(t, delta, np.array(k["indices"]), k["eta"], fused=fused)
    exp = cols_to_rows(k["expected_columns_as_printed"], np.float32)
    assert np.allclose(t, exp, rtol=1e-6, atol=0)
    # exact Float32 arithmetic: -Float32(0.1) * delta (one rounding, acc = 0 + d)
    e32 = np.float32(k["eta"])
    exact = np.zeros_like(t)
    for c, j in zip(k["indices"], range(3)):
        exact[c - 1] = np.float32(0) - e32 * delta[j]
    assert np.array_equal(t, exact)


@pytest.mark.parametrize("dense", [False, True])
def test_histogram_kat(oracle, kat, dense):
    k = kat["misc_histogram"]
    for _ in range(2):  # run twice: shallow_empty! semantics (test/misc.jl:57-71)
        keys, order, count = oracle.histogram(np.array(k["A"]), k["maxindex"], dense)
        assert keys.tolist() == k["expected_keys_in_order"]
        for key, o, c in zip(keys, order, count):
            assert [o, c] == k["expected_order_count"][str(key)]


@pytest.mark.parametrize("dense", [False, True])
def test_indexer_kat(oracle, kat, dense):
    k = kat["misc_indexer"]
    A = np.array(k["A"])
    for _ in range(2):
        cum, mp = oracle.index_build(A, int(A.max()), dense)
        assert cum.tolist() == k["expected_cumulative"]
        assert mp.tolist() == k["expected_map"]


def test_columns_order_kat(oracle, kat):
    """`columns(A)` (test/misc.jl:2-11): a matrix's occurrences go down each column, and
    an occurrence's gradient column is its Julia column — the map of a P x B index."""
    k = kat["misc_columns"]
    rows = np.array(k["matrix_rows"])  # Julia [1 2; 3 4]
    bags = rows.T.copy()  # our (B, P) layout: bag j = Julia column j
    cum, mp = oracle.index_build(bags, 4)
    # the occurrence sequence (col, item) of columns(y) is [(1,1),(1,3),(2,2),(2,4)]
    seq = [(int(mp[p]), int(cum[u][0])) for u in range(len(cum) - 1)
           for p in range(cum[u][1] - 1, cum[u + 1][1] - 1)]
    assert sorted(seq) == sorted(tuple(x) for x in k["matrix_expected"])


# --- properties (test/lookup.jl, test/map.jl, test/update.jl) -------------------------------

DIMS = [32, 64, 128, 256, 512, 1024, 1504]


@pytest.mark.parametrize("dim", DIMS)
def test_lookup_vs_naive(oracle, dim):
    rng = np.random.default_rng(dim)
    ncols = 1000
    A = rng.random((ncols, dim), dtype=np.float32)
    perm = rng.permutation(ncols) + 1
    assert np.array_equal(oracle.lookup(A, perm), oracle.naive_lookup(A, perm))
    rep = rng.integers(1, ncols + 1, ncols)
    assert np.array_equal(oracle.lookup(A, rep), oracle.naive_lookup(A, rep))
    # reducing: 12 lookups per output (test/lookup.jl:42), no repeats then repeats
    I = np.stack([rng.permutation(np.arange(2, ncols + 1)) for _ in range(12)], 1)
    assert np.array_equal(oracle.lookup(A, I), oracle.naive_lookup(A, I))
    I = rng.integers(1, ncols + 1, (ncols, 12))
    assert np.array_equal(oracle.lookup(A, I), oracle.naive_lookup(A, I))


@pytest.mark.parametrize("dtype", [np.float64, np.int32, np.int64])
def test_lookup_dtypes_vs_naive(oracle, dtype):
    rng = np.random.default_rng(7)
    A = (rng.random((300, 48)) * 1000).astype(dtype)
    I = rng.integers(1, 301, (64, 20))
    assert np.array_equal(oracle.lookup(A, I), oracle.naive_lookup(A, I))


def test_f16_per_add_rounding(oracle):
    """Julia Float16 `+` rounds after every add; the fp32-accumulate mode rounds once."""
    rng = np.random.default_rng(3)
    A = rng.standard_normal((100, 16)).astype(np.float16)
    I = rng.integers(1, 101, (32, 20))
    got = oracle.pooled_sum(A, I)
    ref = A[I[:, 0] - 1].copy()
    for i in range(1, 20):
        ref = (ref.astype(np.float32) + A[I[:, i] - 1].astype(np.float32)).astype(np.float16)
    assert np.array_equal(got.view(np.uint16), ref.view(np.uint16))
    acc = oracle.pooled_sum(A, I, f16_fp32_acc=True)
    ref32 = A[I - 1].astype(np.float32)
    s = ref32[:, 0].copy()
    for i in range(1, 20):
        s += ref32[:, i]
    assert np.array_equal(acc.view(np.uint16), s.astype(np.float16).view(np.uint16))


def test_bf16_fp32_accumulation(oracle):
    """bfloat16 (not a reference type): fp32 sum in pool order, one RNE rounding."""
    x = np.array([1.0, 1.00390625, 1.005859375, -3.14159, np.inf, 3.3895e38], np.float32)
    assert oracle.f32_to_bf16(x).tolist() == [16256, 16256, 16257, 49225, 32640, 32639]
    rng = np.random.default_rng(4)
    A = oracle.f32_to_bf16(rng.standard_normal((100, 24)).astype(np.float32))
    I = rng.integers(1, 101, (32, 20))
    f = oracle.bf16_to_f32(A)[I - 1]
    s = f[:, 0].copy()
    for i in range(1, 20):
        s += f[:, i]
    assert np.array_equal(oracle.pooled_sum(A, I, bf16=True), oracle.f32_to_bf16(s))
    assert np.array_equal(oracle.gather(A, I[:, 0], bf16=True), A[I[:, 0] - 1])
    u = oracle.fill_uniform((1000,), "bf16", 5, 0, -1.0, 1.0)
    assert np.array_equal(u, oracle.f32_to_bf16(oracle.fill_uniform((1000,), np.float32, 5, 0,
                                                                     -1.0, 1.0)))


def test_pool_zero_and_empty(oracle):
    A = np.ones((10, 16), np.float32)
    assert np.array_equal(oracle.pooled_sum(A, np.zeros((5, 0), np.int64)), np.zeros((5, 16)))
    assert oracle.lookup(A, np.zeros(0, np.int64)).shape == (0, 16)


@pytest.mark.parametrize("nthreads", [1, 4])
@pytest.mark.parametrize("dim", [16, 64, 512])
def test_prealloc_strategy_equivalence(oracle, nthreads, dim):
    """test/map.jl:32-103: Preallocation == reduce(vcat, map(lookup, ...))."""
    rng = np.random.default_rng(dim + nthreads)
    ntables, ncols, B, P = 10, 100, 64, 10
    tables = [rng.standard_normal((ncols, dim)).astype(np.float32) for _ in range(ntables)]
    for pool in (None, P):
        shape = (B,) if pool is None else (B, pool)
        idx = [rng.integers(1, ncols + 1, shape) for _ in range(ntables)]
        ref = np.concatenate([oracle.naive_lookup(t, i) for t, i in zip(tables, idx)], 1)
        got = oracle.maplookup_prealloc(tables, idx, nthreads=nthreads)
        assert np.array_equal(got, ref)
        got = oracle.maplookup_prealloc(tables, idx, prependrows=20, nthreads=nthreads)
        assert np.array_equal(got[:, 20:], ref)


def _dense_sgd(table, delta, I, eta, fused):
    """Dense Flux reference: table -= eta * uncompress(grad), sequential in occurrence
    order per column (test/update.jl:55-61 compares with isapprox)."""
    I = I.reshape(I.shape[0], -1)
    acc = np.zeros_like(table)
    touched = np.zeros(table.shape[0], bool)
    for j in range(I.shape[0]):
        for i in range(I.shape[1]):
            acc[I[j, i] - 1] += delta[j]
            touched[I[j, i] - 1] = True
    e = np.float32(eta)
    out = table.copy()
    if fused:
        out[touched] = (table[touched].astype(np.float64) - np.float64(e) * acc[touched]).astype(
            np.float32)
    else:
        out[touched] = table[touched] - e * acc[touched]
    return out


@pytest.mark.parametrize("dim", [64, 80, 256])
@pytest.mark.parametrize("reducing", [False, True])
def test_update_vs_dense(oracle, dim, reducing):
    rng = np.random.default_rng(dim)
    ncols = 100
    base = rng.standard_normal((ncols, dim)).astype(np.float32)
    I = rng.integers(1, ncols + 1, (ncols, 10) if reducing else (ncols,))
    delta = rng.standard_normal((ncols, dim)).astype(np.float32)
    for fused in (True, False):
        t = base.copy()
        oracle.sgd(t, delta, I, 10.0, fused=fused)
        assert np.allclose(t, _dense_sgd(base, delta, I, 10.0, fused), rtol=3.45e-4, atol=1e-4)


@pytest.mark.parametrize("dense", [False, True])
def test_update_partitions_exact(oracle, dense):
    """test/update.jl:90-120: the 4-way IndexerView split equals the unsplit update
    exactly — here through the multi-table queue with num_splits 4 vs 1."""
    rng = np.random.default_rng(11)
    base = rng.standard_normal((100, 16)).astype(np.float32)
    delta = rng.standard_normal((512, 16)).astype(np.float32)
    I = rng.integers(1, 101, 512)
    a = base.copy()
    oracle.sgd(a, delta, I, 1.0, fused=True, dense_indexer=dense)
    b = base.copy()
    oracle.sgd_multi([b], [delta], [I], 1.0, [True], num_splits=4, nthreads=4)
    assert np.array_equal(a, b)


def test_multi_table_generic_uses_f64_eta(oracle):
    """Quirk: the multi-table generic path evaluates x - eta*y with the
    Float64 eta; the single-table path converts eta to Float32 first."""
    rng = np.random.default_rng(5)
    base = rng.standard_normal((50, 40)).astype(np.float32)
    delta = rng.standard_normal((256, 40)).astype(np.float32)
    I = rng.integers(1, 51, 256)
    a = base.copy()
    oracle.sgd_multi([a], [delta], [I], 0.1, [False], num_splits=4, nthreads=2)
    acc = np.zeros_like(base)
    for j, c in enumerate(I):
        acc[c - 1] += delta[j]
    touched = np.bincount(I - 1, minlength=50) > 0
    exp = base.copy()
    exp[touched] = (base[touched].astype(np.float64) - 0.1 * acc[touched].astype(np.float64)
                    ).astype(np.float32)
    assert np.array_equal(a, exp)


def test_fill_is_deterministic(oracle):
    a = oracle.fill_uniform((1000,), np.float32, 42, nthreads=1)
    b = oracle.fill_uniform((1000,), np.float32, 42, nthreads=4)
    assert np.array_equal(a, b) and a.min() >= 0 and a.max() < 1
    i = oracle.fill_index_uniform((5000,), 7, 3)
    assert i.min() == 1 and i.max() == 7
