"""Early chains (exact Float32 update): the multi-chunk columns of tables with at most
128 rows are planned straight from the index arrays (k_ec_count / k_ec_plan / k_ec_emit)
and summed on a side stream from the start of the call, while every other chain is
planned from the sorted pairs.  Either way a column's gradient sum is the reference's
serial sum in occurrence order (src/sparseupdate.jl:110-127), so every test here is a
bit-for-bit comparison with the oracle.

Covered: tables of 3 / 4 / 10 / 128 rows (early) beside 129 / 1000-row ones (regular
chains) in one call; pools 1, 20 and 40 (runs of up to 40 equal bags, longer than the
largest entry of 16 adds); a batch that is not a multiple of the 256-bag blocks; a
strided index view (ld_idx > pool); generic (dim 50, Dynamic) and masked-vector (dim 80)
tables; a column with exactly 256 occurrences (one chunk: not a chain) beside one with
257; out-of-range indices (skipped, counted); the two-phase update; HIP-graph capture of
the forked side stream."""
import numpy as np
import pytest
import torch

import embtab as et
from embtab.tables import fused_update_path

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
CHUNK = et._lib.ET_SGD_CHUNK


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


def host(x):
    return x.cpu().numpy()


def _zipf(rng, R, shape, alpha=1.05):
    u = rng.random(shape)
    a1 = 1.0 - alpha
    x = np.floor(((float(R) ** a1 - 1.0) * u + 1.0) ** (1.0 / a1)).clip(1, R).astype(np.int64)
    return rng.permutation(R)[x - 1] + 1


# (rows, dim, static, pool)
MIX = [(3, 128, True, 20), (4, 64, True, 40), (10, 80, True, 20), (128, 128, True, 20),
       (129, 128, True, 20), (7, 50, False, 20), (1000, 128, True, 20), (5, 128, True, 1)]


def _mix(seed, B=1500):
    rng = np.random.default_rng(seed)
    hs = [rng.standard_normal((r, d)).astype(np.float32) for r, d, _, _ in MIX]
    idx = []
    for r, _, _, p in MIX:
        I = _zipf(rng, r, (B, p))
        idx.append(I[:, 0] if p == 1 else I)
    # table 1: long runs of one column inside bags (up to 40 equal bags in a row)
    idx[1][::3, :] = 2
    idx[1][1::7, 5:30] = 3
    # table 3 (128 rows): column 7 exactly CHUNK occurrences (one chunk, not a chain),
    # column 9 CHUNK + 1 (a chain)
    I3 = idx[3]
    I3[I3 == 7] = 1
    I3[I3 == 9] = 1
    flat = I3.reshape(-1)
    pos = rng.permutation(flat.size)
    flat[pos[:CHUNK]] = 7
    flat[pos[CHUNK:2 * CHUNK + 1]] = 9
    return hs, idx


def _tables(hs):
    return [et.SimpleEmbedding(dev(h), et.Static(h.shape[1]) if s else et.Dynamic)
            for h, (_, _, s, _) in zip(hs, MIX)]


def _grads(tabs, idx, delta, strided=False):
    offs = np.cumsum([0] + [d for _, d, _, _ in MIX[:-1]])
    out = []
    for t, (A, I, o) in enumerate(zip(tabs, idx, offs)):
        d = MIX[t][1]
        It = dev(I)
        if strided and I.ndim == 2:  # ld_idx > pool: a column block of a wider array
            wide = torch.zeros((I.shape[0], I.shape[1] + 3), dtype=torch.int64, device=DEV)
            wide[:, :I.shape[1]] = It
            It = wide[:, :I.shape[1]]
        out.append(et.SparseEmbeddingUpdate(A.lookup_type, delta[:, o:o + d], It))
    return out


def _oracle_multi(oracle, hs, idx, delta_h, tabs, eta):
    refs = [h.copy() for h in hs]
    offs = np.cumsum([0] + [d for _, d, _, _ in MIX[:-1]])
    oracle.sgd_multi(refs, delta_h, idx, eta, [fused_update_path(t) for t in tabs],
                     delta_offsets=offs)
    return refs


def test_counts_make_chains_in_every_class():
    """The fixture really exercises both planners: every table has multi-chunk columns,
    the 128-row table has a column of exactly one chunk and one just above."""
    hs, idx = _mix(1)
    for (r, _, _, _), I in zip(MIX, idx):
        c = np.bincount(I.reshape(-1), minlength=r + 1)[1:]
        assert (c > CHUNK).any(), r
    c3 = np.bincount(idx[3].reshape(-1), minlength=129)[1:]
    assert c3[6] == CHUNK and c3[8] == CHUNK + 1


@pytest.mark.parametrize("strided", [False, True])
def test_early_and_regular_chains_vs_oracle(oracle, strided):
    hs, idx = _mix(2 + strided)
    tabs = _tables(hs)
    rng = np.random.default_rng(5)
    ld = sum(d for _, d, _, _ in MIX)
    delta_h = rng.standard_normal((1500, ld)).astype(np.float32)
    grads = _grads(tabs, idx, dev(delta_h), strided)
    et.update_(et.Descent(0.1), tabs, grads, [et.Indexer() for _ in tabs], exact=True)
    torch.cuda.synchronize()
    assert et.check_errors() == 0
    refs = _oracle_multi(oracle, hs, idx, delta_h, tabs, 0.1)
    for t, (A, r) in enumerate(zip(tabs, refs)):
        assert host(A.data).tobytes() == r.tobytes(), f"table {t} ({MIX[t]})"


def test_early_chains_single_table_calls(oracle):
    """One small table per call (the single-table update!): fused for Static, unfused
    for Dynamic, each bit-identical to the oracle's single-table update."""
    hs, idx = _mix(7)
    rng = np.random.default_rng(8)
    for t in (0, 1, 2, 5, 7):
        r, d, s, _ = MIX[t]
        A = et.SimpleEmbedding(dev(hs[t]), et.Static(d) if s else et.Dynamic)
        delta = rng.standard_normal((1500, d)).astype(np.float32)
        g = et.SparseEmbeddingUpdate(A.lookup_type, dev(delta), dev(idx[t]))
        et.update_(et.Descent(0.25), A, g, exact=True)
        ref = hs[t].copy()
        oracle.sgd(ref, delta, idx[t], 0.25, fused=fused_update_path(A))
        assert host(A.data).tobytes() == ref.tobytes(), t


def test_early_chains_out_of_range_indices(oracle):
    """Out-of-range indices of a small table add nothing and are counted once; every
    in-range column is the serial sum of its own occurrences."""
    rng = np.random.default_rng(9)
    R, D, B, P = 6, 128, 700, 20
    h = rng.standard_normal((R, D)).astype(np.float32)
    I = _zipf(rng, R, (B, P))
    bad = rng.random((B, P)) < 0.01
    I[bad] = np.where(rng.random(bad.sum()) < 0.5, 0, R + 1)
    delta = rng.standard_normal((B, D)).astype(np.float32)
    et.check_errors()
    A = et.SimpleEmbedding(dev(h), et.Static(D))
    et.update_(et.Descent(0.1), A, et.SparseEmbeddingUpdate(A.lookup_type, dev(delta), dev(I)),
               exact=True)
    torch.cuda.synchronize()
    assert et.check_errors() == int(bad.sum())
    got = host(A.data)
    chains = 0
    for c in range(R):
        occ = np.nonzero(I.reshape(-1) == c + 1)[0]
        chains += len(occ) > CHUNK
        w = h[c:c + 1].copy()
        oracle.sgd(w, delta[occ // P], np.ones(len(occ), np.int64), 0.1, fused=True)
        assert got[c].tobytes() == w[0].tobytes(), c
    assert chains >= R - 1  # (the bounded Zipf never draws its last rank)


def test_early_chains_two_phases(oracle):
    """INDEX_ONLY (the early plan on the side stream) then APPLY_ONLY (the early chains):
    the same bits as the one-call update and the oracle."""
    hs, idx = _mix(11)
    rng = np.random.default_rng(12)
    ld = sum(d for _, d, _, _ in MIX)
    delta_h = rng.standard_normal((1500, ld)).astype(np.float32)
    delta = dev(delta_h)
    one = _tables(hs)
    et.update_(et.Descent(0.1), one, _grads(one, idx, delta), None, exact=True)
    two = _tables(hs)
    pu = et.PhasedUpdate(two, _grads(two, idx, delta), exact=True)
    pu.index_(torch.cuda.current_stream())
    pu.update_(et.Descent(0.1))
    torch.cuda.synchronize()
    refs = _oracle_multi(oracle, hs, idx, delta_h, one, 0.1)
    for t in range(len(MIX)):
        assert host(two[t].data).tobytes() == host(one[t].data).tobytes() == refs[t].tobytes(), t


def test_early_chains_capture_in_a_hip_graph(oracle):
    """The side-stream fork and join are captured with the caller's stream: replaying the
    graph twice equals two eager updates."""
    hs, idx = _mix(13)
    rng = np.random.default_rng(14)
    ld = sum(d for _, d, _, _ in MIX)
    delta = dev(rng.standard_normal((1500, ld)).astype(np.float32))
    eager = _tables(hs)
    for _ in range(2):
        et.update_(et.Descent(0.1), eager, _grads(eager, idx, delta), None, exact=True)
    graphed = _tables(hs)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # workspace allocation outside the capture
        scratch = _tables(hs)
        et.update_(et.Descent(0.1), scratch, _grads(scratch, idx, delta), None, exact=True)
    torch.cuda.current_stream().wait_stream(side)
    gr = _grads(graphed, idx, delta)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        et.update_(et.Descent(0.1), graphed, gr, None, exact=True)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    for a, b in zip(graphed, eager):
        assert torch.equal(a.data, b.data)
