"""A seeded random sweep of the default (exact) update against the oracle: table storage
(contiguous, paged with a random page size, device column pointers), element type (Float32,
Float64, Float16 with Julia's Float16 arithmetic or Float32 sums, BFloat16), rows, dim, pool,
batch and Zipf or uniform indices drawn at random per case — every table bit-identical to the
oracle's model of src/sparseupdate.jl:97-129 (single-table update!) after one update, every
case an independent draw.  Complements the targeted tests (chain paths, sizes, layouts)
with shapes nobody picked by hand: batches at and around the chunk (256) and tile (4,096)
boundaries, pools of 1, rows of 1."""
import numpy as np
import pytest
import torch

import embtab as et
from embtab.tables import AbstractEmbeddingTable, Static, fused_update_path

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


class _ColPtr(AbstractEmbeddingTable):
    def __init__(self, dense, rng):
        R, D = dense.shape
        self.R, self.D = R, D
        self.pitch = D + 16 // dense.element_size()
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

    def dense(self):
        return self.pool[self.perm, :self.D]


def _case(seed):
    rng = np.random.default_rng(seed)
    kind = ["f32", "f64", "f16", "f16acc", "bf16"][seed % 5]
    storage = ["simple", "paged", "colptr"][(seed // 5) % 3]
    R = int(rng.choice([1, 3, 17, 128, 129, 1000, 5000]))
    D = int(rng.choice([16, 64, 128]))
    P = int(rng.choice([1, 2, 7, 20]))
    B = int(rng.choice([1, 255, 256, 257, 4095, 4096, 4097, 20000]))
    zipf = bool(rng.integers(0, 2))
    return rng, kind, storage, R, D, P, B, zipf


@pytest.mark.parametrize("seed", range(30))
def test_random_default_update_vs_oracle(oracle, seed):
    from oracle import f32_to_bf16

    rng, kind, storage, R, D, P, B, zipf = _case(seed)
    x = rng.standard_normal((R, D)).astype(np.float32)
    d = rng.standard_normal((B, D)).astype(np.float32)
    if kind == "bf16":
        base, delta = f32_to_bf16(x), f32_to_bf16(d)
    else:
        dt = {"f32": np.float32, "f64": np.float64, "f16": np.float16, "f16acc": np.float16}[kind]
        base, delta = x.astype(dt), d.astype(dt)
    if zipf and R > 1:
        u = rng.random((B, P))
        a1 = 1.0 - 1.05
        I = np.floor(((float(R) ** a1 - 1.0) * u + 1.0) ** (1.0 / a1)).clip(1, R).astype(np.int64)
        I = rng.permutation(R)[I - 1] + 1
    else:
        I = rng.integers(1, R + 1, (B, P))
    if P == 1 and seed % 2:
        I = I[:, 0].copy()  # vector indices
    tdev = torch.from_numpy(base).to(DEV)
    ddev = torch.from_numpy(delta).to(DEV)
    if kind == "bf16":
        tdev, ddev = tdev.view(torch.bfloat16), ddev.view(torch.bfloat16)
    if storage == "simple":
        A = et.SimpleEmbedding(tdev, Static(D))
    elif storage == "paged":
        A = et.SplitEmbedding(tdev, int(rng.integers(1, max(2, R) + 1)))
    else:
        A = _ColPtr(tdev, rng)
    g = et.SparseEmbeddingUpdate(A.lookup_type, ddev, torch.from_numpy(I).to(DEV))
    et.update_(et.Descent(0.1), A, g, f16_fp32_acc=kind == "f16acc")
    ref = base.copy()
    oracle.sgd(ref, delta, I, 0.1, fused=fused_update_path(A), bf16=kind == "bf16",
               f16_fp32_acc=kind == "f16acc")
    got = A.data if storage == "simple" else (A.to_dense() if storage == "paged" else A.dense())
    got = (got.view(torch.int16) if kind in ("bf16", "f16", "f16acc") else got).cpu().numpy()
    assert got.tobytes() == ref.view(got.dtype).tobytes(), (kind, storage, R, D, P, B, zipf)
    assert et.check_errors() == 0


@pytest.mark.parametrize("seed", range(100, 120))
def test_random_multi_table_update_vs_oracle(oracle, seed):
    """The multi-table update! (src/sparseupdate.jl:199-238) over 2-6 tables of one element
    type with random storages, rows, dims and pools, sharing one Preallocation-strided gradient
    (k prepended rows), in one pipeline; indexers filled; every table bit-identical to the
    oracle's per-table update of its slice (fused path: Float32 eta; tables whose column
    exceeds 512 bytes take the generic path with the Float64 eta, as the reference)."""
    from oracle import f32_to_bf16

    rng = np.random.default_rng(seed)
    kind = ["f32", "f64", "f16", "bf16"][seed % 4]
    n = int(rng.integers(2, 7))
    B = int(rng.choice([300, 4097, 30000]))
    k = int(rng.choice([0, 1, 4]))
    rows = [int(rng.choice([2, 50, 128, 900, 6000])) for _ in range(n)]
    dims = [int(rng.choice([32, 64, 128])) for _ in range(n)]
    pools = [int(rng.choice([1, 5, 20])) for _ in range(n)]
    ld = k + sum(dims)
    dt = {"f32": np.float32, "f64": np.float64, "f16": np.float16}.get(kind)
    conv = (lambda a: f32_to_bf16(a)) if kind == "bf16" else (lambda a: a.astype(dt))
    hs = [conv(rng.standard_normal((r, d)).astype(np.float32)) for r, d in zip(rows, dims)]
    delta = conv(rng.standard_normal((B, ld)).astype(np.float32))
    hidx = [rng.integers(1, r + 1, (B, p)) for r, p in zip(rows, pools)]
    for t in range(n):  # a hot column in some tables (a chain)
        if rng.integers(0, 2):
            hidx[t][:, 0] = 1
    ddev = torch.from_numpy(delta).to(DEV)
    if kind == "bf16":
        ddev = ddev.view(torch.bfloat16)
    tabs = []
    for t in range(n):
        x = torch.from_numpy(hs[t]).to(DEV)
        if kind == "bf16":
            x = x.view(torch.bfloat16)
        st = int(rng.integers(0, 3))
        tabs.append(et.SimpleEmbedding(x, Static(dims[t])) if st == 0 else
                    et.SplitEmbedding(x, int(rng.integers(1, rows[t] + 1))) if st == 1 else
                    _ColPtr(x, rng))
    offs = np.cumsum([k] + dims[:-1]).tolist()
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, ddev[:, o:o + d], torch.from_numpy(i).to(DEV))
             for A, o, d, i in zip(tabs, offs, dims, hidx)]
    ixs = [et.Indexer() for _ in tabs]
    et.update_(et.Descent(0.1), tabs, grads, ixs)
    refs = [h.copy() for h in hs]
    oracle.sgd_multi(refs, delta, hidx, 0.1, [fused_update_path(A) for A in tabs], num_splits=4,
                     nthreads=4, delta_offsets=offs, bf16=kind == "bf16")
    for t, A in enumerate(tabs):
        got = A.data if isinstance(A, et.SimpleEmbedding) else (
            A.to_dense() if isinstance(A, et.SplitEmbedding) else A.dense())
        got = (got.view(torch.int16) if kind in ("bf16", "f16") else got).cpu().numpy()
        assert got.tobytes() == refs[t].view(got.dtype).tobytes(), (kind, t, rows, dims, pools, B)
        cum, mp = oracle.index_build(hidx[t], rows[t])
        assert np.array_equal(ixs[t].cumulative.cpu().numpy(), cum)
        assert np.array_equal(ixs[t].map.cpu().numpy(), mp)
    assert et.check_errors() == 0


@pytest.mark.parametrize("seed", range(200, 212))
def test_random_indexer_views_and_phased_update_vs_oracle(oracle, seed):
    """Random shapes through the reference's lower-level entry points: index!(Indexer, ...)
    then update!(table, grad, IndexerView(ix, num_splits, s), alpha) for every split
    (src/utils.jl:320-338, src/sparseupdate.jl:46-154; partition exactness as
    test/update.jl:90-120), and the two-phase multi-table update (PhasedUpdate: index while
    the gradient is produced, then apply) — both equal to the oracle, bit for bit."""
    rng = np.random.default_rng(seed)
    R = int(rng.choice([2, 40, 700, 5000]))
    D = int(rng.choice([16, 64, 128, 200]))
    B = int(rng.choice([1, 100, 4096, 9000]))
    P = int(rng.choice([1, 6, 20]))
    dtype = np.float64 if seed % 3 == 0 else np.float32
    h = rng.standard_normal((R, D)).astype(dtype)
    delta = rng.standard_normal((B, D)).astype(dtype)
    I = rng.integers(1, R + 1, (B, P))
    if rng.integers(0, 2):
        I[:, 0] = 1  # a hot column
    storage = ["simple", "paged", "colptr"][seed % 3]
    x = torch.from_numpy(h).to(DEV)
    A = (et.SimpleEmbedding(x, Static(D)) if storage == "simple" else
         et.SplitEmbedding(x, int(rng.integers(1, R + 1))) if storage == "paged" else
         _ColPtr(x, rng))
    g = et.SparseEmbeddingUpdate(A.lookup_type, torch.from_numpy(delta).to(DEV),
                                 torch.from_numpy(I).to(DEV))
    ix = et.index_(et.Indexer(), g.indices, R)
    ns = int(rng.integers(1, 6))
    alpha = float(rng.choice([0.1, 0.5, 1.0]))
    for s in range(1, ns + 1):
        et.update_(A, g, et.IndexerView(ix, ns, s), alpha)
    ref = h.copy()
    oracle.sgd(ref, delta, I, alpha, fused=fused_update_path(A))

    def dense(T):
        return (T.data if isinstance(T, et.SimpleEmbedding) else
                T.to_dense() if isinstance(T, et.SplitEmbedding) else T.dense())

    assert dense(A).cpu().numpy().tobytes() == ref.tobytes(), ("views", R, D, B, P, ns, storage)
    # the phased multi-table update of this table and a second one
    h2 = rng.standard_normal((int(rng.choice([3, 900])), D)).astype(dtype)
    I2 = rng.integers(1, h2.shape[0] + 1, (B, P))
    A2 = et.SimpleEmbedding(torch.from_numpy(h2).to(DEV), Static(D))
    dd = torch.zeros((B, 2 * D), dtype=torch.float64 if dtype == np.float64 else torch.float32,
                     device=DEV)
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, dd[:, :D], g.indices),
             et.SparseEmbeddingUpdate(A2.lookup_type, dd[:, D:], torch.from_numpy(I2).to(DEV))]
    pu = et.PhasedUpdate([A, A2], grads)
    pu.index_()
    d2 = rng.standard_normal((B, 2 * D)).astype(dtype)
    dd.copy_(torch.from_numpy(d2))  # the gradient arrives after the index phase
    pu.update_(et.Descent(0.1))
    refs = [ref, h2.copy()]
    oracle.sgd_multi(refs, d2, [I, I2], 0.1, [fused_update_path(A), fused_update_path(A2)],
                     delta_offsets=[0, D])
    assert dense(A).cpu().numpy().tobytes() == refs[0].tobytes(), "phased 0"
    assert A2.data.cpu().numpy().tobytes() == refs[1].tobytes(), "phased 1"
    assert et.check_errors() == 0


@pytest.mark.parametrize("seed", range(300, 306))
def test_random_step_captured_in_a_graph_replays_eager_bits(oracle, seed):
    """A random training step — Preallocation maplookup of 2-5 tables of mixed storage, the
    rrule pullback, the multi-table default (exact) update with indexers — captured once in a
    HIP graph after an eager warm-up and replayed twice on fresh tables: bit-identical to the
    same two steps run eagerly (every launch stream-ordered, no host synchronisation inside)."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 6))
    B = int(rng.choice([64, 1000, 4096]))
    P = int(rng.choice([1, 8, 20]))
    rows = [int(rng.choice([3, 128, 2000])) for _ in range(n)]
    dims = [int(rng.choice([32, 64, 128])) for _ in range(n)]
    kinds = [int(rng.integers(0, 3)) for _ in range(n)]
    hs = [rng.standard_normal((r, d)).astype(np.float32) for r, d in zip(rows, dims)]
    idx = [torch.from_numpy(rng.integers(1, r + 1, (B, P))).to(DEV) for r in rows]
    dy = torch.from_numpy(rng.standard_normal((B, sum(dims))).astype(np.float32)).to(DEV)

    def make():
        out = []
        for h, kd in zip(hs, kinds):
            x = torch.from_numpy(h).to(DEV)
            out.append(et.SimpleEmbedding(x, Static(x.shape[1])) if kd == 0 else
                       et.SplitEmbedding(x, int(rng.integers(1, x.shape[0] + 1))) if kd == 1 else
                       _ColPtr(x, np.random.default_rng(seed)))
        return out

    def dense(T):
        return (T.data if isinstance(T, et.SimpleEmbedding) else
                T.to_dense() if isinstance(T, et.SplitEmbedding) else T.dense())

    def step(tabs, dst):
        et.maplookup_(et.PreallocationStrategy(0), dst, tabs, idx)
        offs = np.cumsum([0] + dims[:-1]).tolist()
        grads = [et.SparseEmbeddingUpdate(t.lookup_type, dy[:, o:o + d], i)
                 for t, o, d, i in zip(tabs, offs, dims, idx)]
        et.update_(et.Descent(0.05), tabs, grads, [et.Indexer() for _ in tabs])

    eager = make()
    out_e = torch.empty((B, sum(dims)), dtype=torch.float32, device=DEV)
    step(eager, out_e)
    step(eager, out_e)
    graphed = make()
    for t in graphed:  # a column-pointer table's device pointer array is built (and uploaded)
        t.device_table()  # on first use: outside the capture, as any host-to-device copy
    out_g = torch.empty_like(out_e)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up outside the capture (workspaces)
        step(make(), torch.empty_like(out_e))
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step(graphed, out_g)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out_g, out_e)
    for a, b in zip(graphed, eager):
        assert torch.equal(dense(a), dense(b))
    assert et.check_errors() == 0


def test_concurrent_exact_updates_from_two_threads(oracle):
    """Two host threads, each with its own stream and tables, run default (exact) multi-table
    updates 6 times at once: the library's shared side streams and fork/join events serialise
    the calls' side work correctly, and every table equals the oracle's six serial updates."""
    import threading

    rng = np.random.default_rng(400)
    B, P, D = 2048, 20, 64
    cases = []
    for _ in range(2):
        rows = [3, 500, 20000]
        hs = [rng.standard_normal((r, D)).astype(np.float32) for r in rows]
        hidx = [rng.integers(1, r + 1, (B, P)) for r in rows]
        for i in hidx:
            i[:, :2] = 1  # a chain in every table
        delta = rng.standard_normal((B, 3 * D)).astype(np.float32)
        cases.append((rows, hs, hidx, delta))
    results, errs = [None, None], []

    def body(c):
        try:
            rows, hs, hidx, delta = cases[c]
            st = torch.cuda.Stream(DEV)
            with torch.cuda.stream(st):
                tabs = [et.SimpleEmbedding(torch.from_numpy(h).to(DEV), Static(D)) for h in hs]
                dd = torch.from_numpy(delta).to(DEV)
                grads = [et.SparseEmbeddingUpdate(t.lookup_type, dd[:, k * D:(k + 1) * D],
                                                  torch.from_numpy(i).to(DEV))
                         for k, (t, i) in enumerate(zip(tabs, hidx))]
                for _ in range(6):
                    et.update_(et.Descent(0.1), tabs, grads, None)
                results[c] = [t.data.cpu().numpy() for t in tabs]
            st.synchronize()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=body, args=(c,)) for c in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=180)
    assert not errs, errs
    assert not any(t.is_alive() for t in th)
    for c in range(2):
        rows, hs, hidx, delta = cases[c]
        for k in range(3):
            w = hs[k].copy()
            for _ in range(6):
                oracle.sgd(w, np.ascontiguousarray(delta[:, k * D:(k + 1) * D]), hidx[k], 0.1,
                           fused=True)
            assert results[c][k].tobytes() == w.tobytes(), (c, k)


def test_empty_batches_through_every_entry_point(oracle):
    """Batches of zero bags (and pools of zero) through maplookup (Preallocation), the rrule
    pullback, the single- and multi-table update with indexers, and the phased update: no launch
    faults, outputs have the right (empty) shapes, tables are unchanged, and the indexers are
    the reference's empty Indexer (cumulative = [(0, 1)])."""
    rng = np.random.default_rng(500)
    hs = [rng.standard_normal((r, 64)).astype(np.float32) for r in (5, 300)]
    tabs = [et.SimpleEmbedding(torch.from_numpy(h).to(DEV), Static(64)) for h in hs]
    for shape in ((0, 20), (0,), (7, 0)):
        I = [torch.zeros(shape, dtype=torch.int64, device=DEV) for _ in tabs]
        y, back = et.rrule(et.maplookup, et.PreallocationStrategy(2), tabs, I)
        assert tuple(y.shape) == (shape[0], 2 + 128)
        grads = back(torch.zeros_like(y))[2]
        ixs = [et.Indexer(), et.Indexer()]
        et.update_(et.Descent(0.1), tabs, grads, ixs)
        for k in range(2):
            et.update_(et.Descent(0.1), tabs[k], grads[k], et.Indexer())
        pu = et.PhasedUpdate(tabs, grads)
        pu.index_()
        pu.update_(et.Descent(0.1))
        torch.cuda.synchronize()
        for A, h, ix in zip(tabs, hs, ixs):
            assert A.data.cpu().numpy().tobytes() == h.tobytes()
            assert ix.cumulative.cpu().numpy().tolist() == [[0, 1]]
    assert et.check_errors() == 0


def test_concurrent_lookups_and_updates_on_three_streams(oracle):
    """Three host threads at once, each on its own stream and tables: Preallocation maplookups
    (per-XCD queue blocks), multi-table exact updates with indexers (side streams, snapshots),
    single-table lookups + updates of a paged table — each thread's results equal the oracle's
    serial model of its own calls."""
    import threading

    rng = np.random.default_rng(600)
    B, P, D = 1024, 20, 64
    # thread 0: maplookups
    hA = [rng.standard_normal((r, D)).astype(np.float32) for r in (7, 900, 5000)]
    iA = [rng.integers(1, r + 1, (B, P)) for r in (7, 900, 5000)]
    # thread 1: multi-table updates
    hB = [rng.standard_normal((r, D)).astype(np.float32) for r in (3, 2000)]
    iB = [rng.integers(1, r + 1, (B, P)) for r in (3, 2000)]
    dB = rng.standard_normal((B, 2 * D)).astype(np.float32)
    # thread 2: lookups + single-table updates of a paged table
    hC = rng.standard_normal((777, D)).astype(np.float32)
    iC = rng.integers(1, 778, (B, P))
    dC = rng.standard_normal((B, D)).astype(np.float32)
    out, errs = {}, []

    def t0():
        tabs = [et.SimpleEmbedding(torch.from_numpy(h).to(DEV), Static(D)) for h in hA]
        idx = [torch.from_numpy(i).to(DEV) for i in iA]
        ys = [et.maplookup(et.PreallocationStrategy(0), tabs, idx) for _ in range(8)]
        out[0] = [y.cpu().numpy() for y in ys]

    def t1():
        tabs = [et.SimpleEmbedding(torch.from_numpy(h).to(DEV), Static(D)) for h in hB]
        dd = torch.from_numpy(dB).to(DEV)
        grads = [et.SparseEmbeddingUpdate(t.lookup_type, dd[:, k * D:(k + 1) * D],
                                          torch.from_numpy(i).to(DEV))
                 for k, (t, i) in enumerate(zip(tabs, iB))]
        ixs = [et.Indexer(), et.Indexer()]
        for _ in range(4):
            et.update_(et.Descent(0.1), tabs, grads, ixs)
        out[1] = ([t.data.cpu().numpy() for t in tabs], [ix.map.cpu().numpy() for ix in ixs])

    def t2():
        A = et.SplitEmbedding(torch.from_numpy(hC).to(DEV), 50)
        I = torch.from_numpy(iC).to(DEV)
        g = et.SparseEmbeddingUpdate(A.lookup_type, torch.from_numpy(dC).to(DEV), I)
        ys = []
        for _ in range(4):
            ys.append(et.lookup(A, I).cpu().numpy())
            et.update_(et.Descent(0.1), A, g)
        out[2] = (ys, A.to_dense().cpu().numpy())

    def run(fn):
        try:
            st = torch.cuda.Stream(DEV)
            with torch.cuda.stream(st):
                fn()
            st.synchronize()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(f,)) for f in (t0, t1, t2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=180)
    assert not errs, errs
    assert not any(t.is_alive() for t in th)
    ref = np.ascontiguousarray(oracle.maplookup_prealloc(hA, iA, prependrows=0)).tobytes()
    assert all(y.tobytes() == ref for y in out[0])
    w = [h.copy() for h in hB]
    for _ in range(4):
        for k in range(2):
            oracle.sgd(w[k], np.ascontiguousarray(dB[:, k * D:(k + 1) * D]), iB[k], 0.1, fused=True)
    for k in range(2):
        assert out[1][0][k].tobytes() == w[k].tobytes()
        assert np.array_equal(out[1][1][k], oracle.index_build(iB[k], hB[k].shape[0])[1])
    wc = hC.copy()
    for it in range(4):
        assert out[2][0][it].tobytes() == oracle.pooled_sum(wc, iC).tobytes()
        oracle.sgd(wc, dC, iC, 0.1, fused=True)
    assert out[2][1].tobytes() == wc.tobytes()


def test_captured_update_survives_workspace_eviction(oracle):
    """The host caches update workspaces for the 4 most recently used streams per key and
    releases older ones; a workspace a HIP graph captured is pinned instead — the graph replays
    into it.  Capture an exact update, then run eager updates from 6 other streams (evicting
    every cached workspace) and churn the allocator, then replay: bit-identical to the oracle's
    two serial updates."""
    rng = np.random.default_rng(700)
    B, P, D, R = 4096, 20, 64, 300
    h = rng.standard_normal((R, D)).astype(np.float32)
    hi = rng.integers(1, R + 1, (B, P))
    hd = rng.standard_normal((B, D)).astype(np.float32)
    A = et.SimpleEmbedding(torch.from_numpy(h).to(DEV), Static(D))
    g_up = et.SparseEmbeddingUpdate(A.lookup_type, torch.from_numpy(hd).to(DEV),
                                    torch.from_numpy(hi).to(DEV))
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up outside the capture
        W = et.SimpleEmbedding(torch.from_numpy(h).to(DEV), Static(D))
        et.update_(et.Descent(0.1), W, g_up)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        et.update_(et.Descent(0.1), A, g_up)
    torch.cuda.synchronize()
    other = et.SimpleEmbedding(torch.from_numpy(h).to(DEV), Static(D))
    for _ in range(6):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            et.update_(et.Descent(0.1), other, g_up)
            junk = torch.full((B * P * 16,), 7, dtype=torch.int32, device=DEV)  # reuse freed blocks
            del junk
        st.synchronize()
    A.data.copy_(torch.from_numpy(h).to(DEV))  # the capture ran nothing: start from h
    graph.replay()
    graph.replay()
    torch.cuda.synchronize()
    ref = h.copy()
    for _ in range(2):
        oracle.sgd(ref, hd, hi, 0.1, fused=True)
    assert A.data.cpu().numpy().tobytes() == ref.tobytes()
    assert et.check_errors() == 0
