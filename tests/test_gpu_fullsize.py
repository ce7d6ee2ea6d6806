"""Parity at BASELINE.json's full sizes (configs 2-4 on one MI355X).

The oracle cannot redo a 17 GB step in seconds, so each test checks (a) a random
sample of outputs bit-for-bit against the oracle run on exactly the rows they read
(gathered from the device tables), and (b) size-independent properties over the
whole output: linearity of the pooled sum (sum over all bags == sum over all
occurrences of the row sums, in fp64) and, for the update, that untouched columns
are bit-unchanged.  Tables come from the engine's counter-hash fill, which
tests/test_gpu_lookup.py::test_fill_matches_oracle pins to the oracle's fill."""
import numpy as np
import pytest
import torch

import embtab as et
from embtab import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
ROWS = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194, 27,
        14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572]
B, P, D = 65536, 20, 128


def _fill_tables(seed0=1000):
    L = _lib.load()
    s = _lib.stream_handle()
    tabs, idx = [], []
    for t, R in enumerate(ROWS):
        x = torch.empty((R, D), dtype=torch.float32, device=DEV)
        _lib.check(L.et_fill_uniform(_lib.ET_F32, x.data_ptr(), x.numel(), seed0 + t, 0, 0.0, 1.0,
                                     s))
        I = torch.empty((B, P), dtype=torch.int64, device=DEV)
        _lib.check(L.et_fill_index_uniform(I.data_ptr(), I.numel(), R, 2000 + t, 0, s))
        tabs.append(et.SimpleEmbedding(x, et.Static(D)))
        idx.append(I)
    return tabs, idx


@pytest.fixture(scope="module")
def criteo():
    tabs, idx = _fill_tables()
    yield tabs, idx
    del tabs, idx
    torch.cuda.empty_cache()


def _sample_check(oracle, tabs, idx, out, bags, k=0):
    """Oracle pooled sums of the sampled bags from the rows they read."""
    off = k
    for A, I in zip(tabs, idx):
        Ib = I[bags]                                   # (nb, P) 1-based
        uniq, inv = torch.unique(Ib, return_inverse=True)
        rows = A.data[uniq - 1].cpu().numpy()          # the rows these bags read
        local = (inv + 1).cpu().numpy().astype(np.int64)
        ref = oracle.pooled_sum(rows, local)
        got = out[bags, off:off + D].cpu().numpy()
        assert ref.tobytes() == np.ascontiguousarray(got).tobytes()
        off += D


def test_config3_full_size(oracle, criteo):
    tabs, idx = criteo
    out = et.maplookup(et.PreallocationStrategy(), tabs, idx)
    torch.cuda.synchronize()
    assert et.check_errors() == 0
    g = torch.Generator().manual_seed(3)
    bags = torch.randint(0, B, (512,), generator=g).to(DEV)
    _sample_check(oracle, tabs, idx, out, bags)
    # linearity: sum over bags of the output == sum over occurrences of the row sums
    for t, (A, I) in enumerate(zip(tabs, idx)):
        rs = A.data.double().sum(1)
        lhs = out[:, t * D:(t + 1) * D].double().sum()
        rhs = rs[I.view(-1) - 1].sum()
        assert torch.allclose(lhs, rhs, rtol=1e-6, atol=0), t


def test_config3_prepend_and_nontemporal_variants(oracle, criteo):
    tabs, idx = criteo
    base = et.maplookup(et.PreallocationStrategy(), tabs, idx)
    k = 16
    dst = torch.full((B, k + D * len(tabs)), -7.0, dtype=torch.float32, device=DEV)
    et.maplookup_(et.PreallocationStrategy(k), dst, tabs, idx, nontemporal=False)
    assert torch.equal(dst[:, k:], base)
    assert (dst[:, :k] == -7.0).all()  # prepended rows untouched


def test_config2_full_size(oracle):
    L = _lib.load()
    R = 10_000_000
    x = torch.empty((R, D), dtype=torch.float32, device=DEV)
    _lib.check(L.et_fill_uniform(_lib.ET_F32, x.data_ptr(), x.numel(), 3000, 0, 0.0, 1.0,
                                 _lib.stream_handle()))
    I = torch.empty(B, dtype=torch.int64, device=DEV)
    _lib.check(L.et_fill_index_uniform(I.data_ptr(), B, R, 3001, 0, _lib.stream_handle()))
    A = et.SimpleEmbedding(x, et.Static(D))
    out = et.lookup(A, I)
    assert torch.equal(out, x[I - 1])          # bit copy of every row
    sample = torch.arange(0, B, 97, device=DEV)
    rows = x[I[sample] - 1].cpu().numpy()
    ref = oracle.gather(rows, np.arange(1, len(sample) + 1))
    assert ref.tobytes() == out[sample].cpu().numpy().tobytes()
    del x
    torch.cuda.empty_cache()


def _zipf(R, shape, gen):
    u = torch.rand(shape, generator=gen, device=DEV, dtype=torch.float64)
    a1 = 1.0 - 1.05
    x = torch.floor(((float(R) ** a1 - 1.0) * u + 1.0) ** (1.0 / a1)).clamp_(1, R).long()
    return torch.randperm(R, generator=gen, device=DEV)[x - 1] + 1


def test_config4_full_size(oracle, criteo):
    """Zipf(1.05) forward + fused Descent(0.1) on all 26 tables at B = 65536 in the
    split mode (exact=False: columns longer than one chunk summed as ordered partials);
    every table is checked: untouched columns unchanged, 24 sampled touched columns plus
    the hottest against the oracle's serial update (bit-identical up to one chunk, within
    the summation bound beyond).  The default (exact) mode is the next test."""
    tabs, _ = criteo
    gen = torch.Generator(device=DEV)
    gen.manual_seed(4000)
    idx = [_zipf(R, (B, P), gen) for R in ROWS]
    before = [A.data.clone() for A in tabs]
    y, back = et.rrule(et.maplookup, et.PreallocationStrategy(), tabs, idx)
    delta = torch.empty_like(y)
    _lib.check(_lib.load().et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 4001, 0,
                                           -1.0, 1.0, _lib.stream_handle()))
    grads = back(delta)[2]
    et.update_(et.Descent(0.1), tabs, grads, [et.Indexer() for _ in tabs], exact=False)
    torch.cuda.synchronize()
    assert et.check_errors() == 0
    g = torch.Generator().manual_seed(5)
    errs_chunked, errs_serial = [], []
    for t in range(len(ROWS)):
        A, I, W0 = tabs[t], idx[t], before[t]
        counts = torch.bincount(I.view(-1), minlength=ROWS[t] + 1)[1:]
        touched = torch.nonzero(counts).view(-1)
        # untouched columns are bit-unchanged
        mask = torch.ones(ROWS[t], dtype=torch.bool, device=DEV)
        mask[touched] = False
        assert torch.equal(A.data[mask], W0[mask])
        # sampled touched columns (always including the hottest) vs the oracle, serially
        pick = touched[torch.randperm(len(touched), generator=g)[:24].to(DEV)]
        pick = torch.unique(torch.cat([pick, counts.argmax().view(1)]))
        dl = grads[t].delta
        for c in pick.tolist():
            occ = torch.nonzero(I.view(-1) == c + 1).view(-1)     # occurrence order
            bags = (occ // P).cpu().numpy()
            dsub = dl[occ // P].cpu().numpy()                       # one delta row per occurrence
            w = W0[c:c + 1].cpu().numpy().copy()
            oracle.sgd(w, dsub, np.ones(len(bags), np.int64), 0.1, fused=True)
            got = A.data[c].cpu().numpy()
            n = len(bags)
            if n <= et._lib.ET_SGD_CHUNK:   # one chunk: the serial sum, bit-identical
                assert w[0].tobytes() == got.tobytes(), (t, c, n)
            else:
                # chunked: against the EXACT update, 1e-6 of |w| + eta * sum|delta| (the
                # error-bound scale; see test_gpu_update), and no worse than the serial sum
                eta = np.float64(np.float32(0.1))
                w0 = W0[c].cpu().numpy().astype(np.float64)
                exact = w0 - eta * dsub.astype(np.float64).sum(0)
                scale = np.abs(w0) + eta * np.abs(dsub).astype(np.float64).sum(0)
                err = np.abs(got.astype(np.float64) - exact)
                assert np.all(err <= 1e-6 * scale), (t, c, n, float((err / scale).max()))
                errs_chunked.append(err.max())
                errs_serial.append(np.abs(w[0].astype(np.float64) - exact).max())
    # over all sampled split columns: the chunked sums are no farther from the exact
    # update than the reference's serial fp32 sum (per column either may win by chance)
    assert errs_chunked and max(errs_chunked) <= max(errs_serial)


def test_config4_full_size_exact(oracle, criteo):
    """north_star's parity bar for the fp32 update at full size: the exact mode
    (ET_FLAG_EXACT_UPDATE: single-chunk columns in the chunk pass, every longer column a
    serial chain) on the Zipf(1.05) batch of all 26 tables at B = 65536 is bit-identical
    to the oracle's serial update (reference src/sparseupdate.jl:110-127) on sampled
    columns of every table, always including each table's three hottest columns — the
    hottest of the batch has 834,828 occurrences — and leaves untouched columns
    bit-unchanged."""
    tabs, _ = criteo
    gen = torch.Generator(device=DEV)
    gen.manual_seed(4000)
    idx = [_zipf(R, (B, P), gen) for R in ROWS]
    before = [A.data.clone() for A in tabs]
    delta = torch.empty((B, D * len(ROWS)), dtype=torch.float32, device=DEV)
    _lib.check(_lib.load().et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 4001, 0,
                                           -1.0, 1.0, _lib.stream_handle()))
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, t * D:(t + 1) * D], i)
             for t, (A, i) in enumerate(zip(tabs, idx))]
    et.update_(et.Descent(0.1), tabs, grads, [et.Indexer() for _ in tabs], exact=True)
    torch.cuda.synchronize()
    assert et.check_errors() == 0
    g = torch.Generator().manual_seed(6)
    hottest = 0
    for t in range(len(ROWS)):
        A, I, W0 = tabs[t], idx[t], before[t]
        counts = torch.bincount(I.view(-1), minlength=ROWS[t] + 1)[1:]
        touched = torch.nonzero(counts).view(-1)
        mask = torch.ones(ROWS[t], dtype=torch.bool, device=DEV)
        mask[touched] = False
        assert torch.equal(A.data[mask], W0[mask])
        pick = touched[torch.randperm(len(touched), generator=g)[:12].to(DEV)]
        top = torch.topk(counts, min(3, ROWS[t])).indices
        pick = torch.unique(torch.cat([pick, top]))
        dl = grads[t].delta
        for c in pick.tolist():
            occ = torch.nonzero(I.view(-1) == c + 1).view(-1)     # occurrence order
            n = len(occ)
            if n == 0:
                continue
            hottest = max(hottest, n)
            dsub = dl[occ // P].cpu().numpy()                       # one delta row per occurrence
            w = W0[c:c + 1].cpu().numpy().copy()
            oracle.sgd(w, dsub, np.ones(n, np.int64), 0.1, fused=True)
            assert w[0].tobytes() == A.data[c].cpu().numpy().tobytes(), (t, c, n)
            del dsub
    assert hottest >= 800_000  # the serial chain of the hottest column was checked
    del before


def test_config1_reference_plumbing(oracle):
    """BASELINE config 1: SimpleEmbedding Float32 dim 16, 1000 columns, vector indices
    B = 128 — the GPU result equals the oracle's and the reference's naive lookup."""
    rng = np.random.default_rng(0)
    h = rng.random((1000, 16), dtype=np.float32)
    I = rng.integers(1, 1001, 128)
    A = et.SimpleEmbedding(torch.from_numpy(h).to(DEV), et.Static(16))
    got = et.lookup(A, torch.from_numpy(I).to(DEV)).cpu().numpy()
    assert got.tobytes() == oracle.gather(h, I).tobytes() == oracle.naive_lookup(h, I).tobytes()


def test_config5_shape_simulated_8_ranks(oracle):
    """BASELINE config 5 shape (26 Criteo tables, B = 131072) through the 8-rank
    feature-balanced plan on one GPU: every simulated rank looks up its pieces into
    its slab with the real kernels; the stacked slabs are assembled by et_concat_slabs
    (all-gather layout) or sliced per rank (all-to-all layout).  Both equal the
    unsharded Preallocation output bit for bit."""
    from embtab.sharding import ShardedMapLookup, ShardPlan, piece_table

    Bc = 131072
    L = _lib.load()
    s = _lib.stream_handle()
    tabs, idx = [], []
    for t, R in enumerate(ROWS):
        x = torch.empty((R, D), dtype=torch.float32, device=DEV)
        _lib.check(L.et_fill_uniform(_lib.ET_F32, x.data_ptr(), x.numel(), 1000 + t, 0, 0.0, 1.0,
                                     s))
        I = torch.empty((Bc, P), dtype=torch.int64, device=DEV)
        _lib.check(L.et_fill_index_uniform(I.data_ptr(), I.numel(), R, 5000 + t, 0, s))
        tabs.append(et.SimpleEmbedding(x, et.Static(D)))
        idx.append(I)
    base = et.maplookup(et.PreallocationStrategy(), tabs, idx)
    g = torch.Generator().manual_seed(5)
    _sample_check(oracle, tabs, idx, base, torch.randint(0, Bc, (256,), generator=g).to(DEV))
    world = 8
    plan = ShardPlan.featurewise([D] * len(ROWS), world)
    slabs = []
    for r in range(world):
        sm = ShardedMapLookup(plan, r, world, Bc, torch.float32, DEV)
        ps = plan.pieces[r]
        sm.lookup_chunk([piece_table(tabs[p.table], p) for p in ps], [idx[p.table] for p in ps],
                        0, Bc)
        slabs.append(sm.slab)
    gathered = torch.stack(slabs)
    dst = torch.empty_like(base)
    sm.assemble_chunk(gathered, dst)
    assert torch.equal(dst, base)
    a2a = [ShardedMapLookup(plan, r, world, Bc, torch.float32, DEV, exchange="alltoall")
           for r in range(world)]
    for r in (0, 5):
        lo, hi = a2a[r].split[r], a2a[r].split[r + 1]
        part = torch.empty((hi - lo, plan.ld), dtype=torch.float32, device=DEV)
        a2a[r].assemble_chunk(gathered[:, lo:hi].contiguous(), part)
        assert torch.equal(part, base[lo:hi])
    del tabs, idx, base, slabs, gathered, dst
    torch.cuda.empty_cache()
