"""Paged (SplitEmbedding) and column-pointer tables through every chain path of the DEFAULT
(exact) update.

Since ABI v9 the default update sums every column longer than one chunk (256 occurrences) as
a serial chain, and each chain path addresses the table through col_ptr(..., cols_per_page):
  * early chains (EC) — tables of at most 128 rows, planned from the index arrays
    (S = 4 / 8 / 16 entries of the hand-scheduled loop);
  * early hot columns (EH) — the sampled hottest columns of the larger tables;
  * the quad walk — Float32 S = 1 chains of at least 1,024 64-entry groups;
  * regular chains — the rest of the > 256-occurrence columns, planned after the sort.
The reference's paged `columnpointer` is src/split.jl:81-86 (`_divrem_index` into a page);
the sum it must equal is src/sparseupdate.jl:110-127 (acc from +0 in occurrence order, then
fma(-eta, acc, w)); the multi-table call is :199-238.  Every table here is paged (cols per
page 7 or 4,096) or a device column-pointer array (cols_per_page = 1), and the batches are
shaped so that every path above has work (the host recomputes the chain shapes of the checked
columns with the plan's own cost rule and asserts it).  Each table's three hottest columns,
8 sampled ones, regular-chain and chunk-pass columns are bit-identical to oracle.sgd on the
dense copy, and every untouched column is unchanged."""
import numpy as np
import pytest
import torch

import embtab as et
from embtab import _lib
from embtab.tables import AbstractEmbeddingTable, Static, fused_update_path

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
CHUNK = _lib.ET_SGD_CHUNK          # a longer column is a chain in the exact mode
EC_MAX_ROWS = 128                  # et_update.hip kEcMaxRows
QUAD_MIN_ENTRIES = 1024 * 64       # kQuadMinGroups 64-entry groups
COST2 = {0: 9, 1: 17, 2: 21, 3: 22, 4: 38}  # chain_entry_cost2(2^k)


class ColumnPointerTable(AbstractEmbeddingTable):
    """Only the reference's plug-in contract (size / columnpointer / example, README.md:288-307):
    column i sits at slot perm[i] of a pool whose slots are `pitch` elements apart, so the
    engine describes it as a device column-pointer array (cols_per_page = 1)."""

    def __init__(self, dense: torch.Tensor, pitch: int, gen: torch.Generator):
        R, D = dense.shape
        self.R, self.D, self.pitch = R, D, pitch
        self.perm = torch.randperm(R, generator=gen, device=DEV)
        self.pool = torch.zeros((R, pitch), dtype=dense.dtype, device=DEV)
        self.pool[self.perm, :D] = dense
        self.lookup_type = Static(D)

    def size(self):
        return (self.D, self.R)

    def columnpointers(self):
        es = self.pool.element_size()
        return self.pool.data_ptr() + self.perm.cpu().numpy().astype(np.int64) * self.pitch * es

    def columnpointer(self, i, ctx=None):
        return int(self.columnpointers()[i - 1])

    def example(self):
        return self.pool[0:1, :self.D]

    def dense(self) -> torch.Tensor:
        return self.pool[self.perm, :self.D]


def _dense(A) -> torch.Tensor:
    return A.to_dense() if isinstance(A, et.SplitEmbedding) else A.dense()


def _zipf(R, shape, gen):
    u = torch.rand(shape, generator=gen, device=DEV, dtype=torch.float64)
    a1 = 1.0 - 1.05
    x = torch.floor(((float(R) ** a1 - 1.0) * u + 1.0) ** (1.0 / a1)).clamp_(1, R).long()
    return torch.randperm(R, generator=gen, device=DEV)[x - 1] + 1


def _chain_shape(I: torch.Tensor, c: int):
    """(S, entries) the chain plan gives column c (1-based): runs r_b per bag, entries at S = 2^k
    are sum ceil(r_b / S), cost entries * chain_entry_cost2(S), cheapest first (k_chain_choose)."""
    r = (I == c).sum(1)
    r = r[r > 0].double()
    E = [int(torch.ceil(r / 2 ** k).sum()) for k in range(5)]
    k = min(range(5), key=lambda k: (E[k] * COST2[k], k))
    return 2 ** k, E[k]


def _check_columns(oracle, got, W0, I, dl, P, cols, feats):
    """The oracle's serial fused update of columns `cols` (0-based) on the feature subset
    `feats` (features are independent in the reference's sum), bit for bit."""
    for c in cols:
        occ = torch.nonzero(I.reshape(-1) == c + 1).view(-1)  # occurrence order
        n = len(occ)
        dsub = dl[:, feats][occ // P].cpu().numpy()
        w = W0[c:c + 1, feats].cpu().numpy().copy()
        oracle.sgd(w, dsub, np.ones(n, np.int64), 0.1, fused=True)
        assert w[0].tobytes() == got[c, feats].cpu().numpy().tobytes(), (c, n)


def test_paged_and_column_pointer_tables_every_chain_path(oracle):
    Bb, D = 262144, 128
    # (rows, pool, storage, role)
    spec = [(100, 20, 7, "EC"), (4, 20, 1, "EC"),
            (1_200_000, 5, 4096, "EH+quad"), (1_000_000, 5, 1, "EH+quad"),
            (5000, 20, 7, "regular"), (3000, 20, 1, "regular")]
    ld = D * len(spec)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(606)
    L = _lib.load()
    s = _lib.stream_handle()
    tabs, idx, before = [], [], []
    for t, (R, P, cpp, _) in enumerate(spec):
        x = torch.empty((R, D), dtype=torch.float32, device=DEV)
        _lib.check(L.et_fill_uniform(_lib.ET_F32, x.data_ptr(), x.numel(), 6060 + t, 0, -1.0, 1.0,
                                     s))
        A = et.SplitEmbedding(x, cpp) if cpp > 1 else ColumnPointerTable(x, D + 4, gen)
        assert A.device_table()[1] == cpp and fused_update_path(A)
        tabs.append(A)
        before.append(x)
        idx.append(_zipf(R, (Bb, P), gen))
    delta = torch.empty((Bb, ld), dtype=torch.float32, device=DEV)
    _lib.check(L.et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 6100, 0, -1.0, 1.0,
                                 s))
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, t * D:(t + 1) * D], i)
             for t, (A, i) in enumerate(zip(tabs, idx))]
    et.update_(et.Descent(0.1), tabs, grads, [et.Indexer() for _ in tabs])  # default mode
    torch.cuda.synchronize()
    assert et.check_errors() == 0

    g = torch.Generator().manual_seed(61)
    feats = torch.tensor([0, 1, 31, 63, 64, 100, 127], device=DEV)
    roles = {"EC": 0, "quad": 0, "EH": 0, "regular": 0, "chunk": 0, "S>1": 0}
    for t, (R, P, cpp, role) in enumerate(spec):
        A, I, W0 = tabs[t], idx[t], before[t]
        got = _dense(A)
        counts = torch.bincount(I.view(-1), minlength=R + 1)[1:]
        touched = torch.nonzero(counts).view(-1)
        mask = torch.ones(R, dtype=torch.bool, device=DEV)
        mask[touched] = False
        assert torch.equal(got[mask], W0[mask]), t  # untouched columns unchanged
        pick = touched[torch.randperm(len(touched), generator=g)[:8].to(DEV)]
        top = torch.topk(counts, min(3, R)).indices
        mid = torch.nonzero((counts > CHUNK) & (counts <= 20000)).view(-1)[:2]  # regular chains
        low = torch.nonzero((counts > 1) & (counts <= CHUNK)).view(-1)[:2]      # chunk pass
        cols = torch.unique(torch.cat([pick, top, mid, low])).tolist()
        _check_columns(oracle, got, W0, I, grads[t].delta, P, cols, feats)
        # what the checked columns exercised (the plan's own rules, recomputed on the host)
        for c in cols:
            n = int(counts[c])
            if n <= CHUNK:
                roles["chunk"] += 1
                continue
            S, E = _chain_shape(I, c + 1)
            roles["S>1"] += S > 1
            if R <= EC_MAX_ROWS:
                roles["EC"] += 1
            elif S == 1 and E >= QUAD_MIN_ENTRIES:
                roles["quad"] += 1
            elif n >= 32768:
                roles["EH"] += 1
            elif n <= 20000:
                roles["regular"] += 1
        del got
    assert all(v > 0 for v in roles.values()), roles
    del delta, grads, before, tabs, idx
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kind", ["f32", "f64", "f16", "f16acc", "bf16"])
def test_paged_and_column_pointer_early_chains_typed(oracle, kind):
    """The early chains (S = 4 / 8 / 16 entries and S = 1) of a paged (7 columns per page) and a
    column-pointer table in every element type: the whole table bit-identical to the oracle's
    typed model of the reference's update (oracle/embtab_oracle.c)."""
    from oracle import f32_to_bf16

    rng = np.random.default_rng(62)
    Bb, P, dim = 65536, 20, 64
    gen = torch.Generator(device=DEV)
    gen.manual_seed(63)
    npdt = {"f32": np.float32, "f64": np.float64, "f16": np.float16, "f16acc": np.float16}
    for R, cpp in ((100, 7), (4, 1)):
        x = rng.standard_normal((R, dim)).astype(np.float32)
        d = rng.standard_normal((Bb, dim)).astype(np.float32)
        if kind == "bf16":
            base, delta = f32_to_bf16(x), f32_to_bf16(d)
        else:
            base, delta = x.astype(npdt[kind]), d.astype(npdt[kind])
        I = _zipf(R, (Bb, P), gen)
        tdev = torch.from_numpy(base).to(DEV)
        ddev = torch.from_numpy(delta).to(DEV)
        if kind == "bf16":
            tdev, ddev = tdev.view(torch.bfloat16), ddev.view(torch.bfloat16)
        pitch = dim + 16 // tdev.element_size()  # 16-byte aligned columns
        A = et.SplitEmbedding(tdev, cpp) if cpp > 1 else ColumnPointerTable(tdev, pitch, gen)
        assert A.device_table()[1] == cpp
        g = et.SparseEmbeddingUpdate(A.lookup_type, ddev, I)
        et.update_(et.Descent(0.1), A, g, f16_fp32_acc=kind == "f16acc")  # default mode
        ref = base.copy()
        oracle.sgd(ref, delta, I.cpu().numpy(), 0.1, fused=fused_update_path(A),
                   bf16=kind == "bf16", f16_fp32_acc=kind == "f16acc")
        got = _dense(A)
        got = (got.view(torch.int16) if kind in ("bf16", "f16", "f16acc") else got).cpu().numpy()
        counts = np.bincount(I.cpu().numpy().ravel(), minlength=R + 1)[1:]
        assert counts.max() > 100_000  # early chains ran
        shapes = {_chain_shape(I, c + 1)[0] for c in np.nonzero(counts > CHUNK)[0]}
        assert shapes - {1}, shapes  # entries of several adds (S > 1) as well
        assert got.tobytes() == ref.view(got.dtype).tobytes(), (kind, R, cpp)
    assert et.check_errors() == 0


def test_exact_default_at_2_pow_24_bags(oracle):
    """ADVICE r05 (medium) / VERDICT r05 item 7: a batch of 2^24 bags, pool 1, one small hot
    table, in the DEFAULT mode.  Chain entries carry a 27-bit bag from 2^24 bags on
    (chain_shift), so the hot columns (~2 M occurrences each) still run as chains, not as one
    wave per column; the whole table is bit-identical to the oracle's serial update."""
    Bb, R, dim = 1 << 24, 1000, 16
    gen = torch.Generator(device=DEV)
    gen.manual_seed(64)
    L = _lib.load()
    s = _lib.stream_handle()
    x = torch.empty((R, dim), dtype=torch.float32, device=DEV)
    _lib.check(L.et_fill_uniform(_lib.ET_F32, x.data_ptr(), x.numel(), 6400, 0, -1.0, 1.0, s))
    delta = torch.empty((Bb, dim), dtype=torch.float32, device=DEV)
    _lib.check(L.et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 6401, 0, -1.0, 1.0,
                                 s))
    I = _zipf(R, (Bb,), gen)
    A = et.SimpleEmbedding(x.clone(), Static(dim))
    et.update_(et.Descent(0.1), A, et.SparseEmbeddingUpdate(A.lookup_type, delta, I))
    torch.cuda.synchronize()
    assert et.check_errors() == 0
    counts = torch.bincount(I, minlength=R + 1)[1:]
    assert int(counts.max()) > 1_500_000
    ref = x.cpu().numpy()
    oracle.sgd(ref, delta.cpu().numpy(), I.cpu().numpy(), 0.1, fused=True)
    assert A.data.cpu().numpy().tobytes() == ref.tobytes()
    # the boundary below it (2^24 - 1 bags: the 24-bit entries) on the same data
    A2 = et.SimpleEmbedding(x.clone(), Static(dim))
    n = Bb - 1
    et.update_(et.Descent(0.1), A2, et.SparseEmbeddingUpdate(A2.lookup_type, delta[:n], I[:n]))
    ref2 = x.cpu().numpy()
    oracle.sgd(ref2, delta[:n].cpu().numpy(), I[:n].cpu().numpy(), 0.1, fused=True)
    assert A2.data.cpu().numpy().tobytes() == ref2.tobytes()


def test_streamed_loop_on_the_regular_list(oracle):
    """The streamed chain loop (S = 8 / 16: per-entry gradient offsets and lane masks written
    by the plan, et_chain_asm.h chain_walk_stream) on the REGULAR list — columns of tables
    above the early-chain size with 257..20,000 occurrences and many adds per bag, walked by
    the shared-SIMD chain kernel — for contiguous, paged and column-pointer tables, and beside
    early chains of the same call: every table bit-identical to the oracle's serial update."""
    Bb, P, D = 2048, 64, 128
    spec = [(300, 0), (257, 7), (400, 1), (60, 0)]  # (rows, cols per page; 0 contiguous)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(607)
    rng = np.random.default_rng(608)
    tabs, idx, base = [], [], []
    for R, cpp in spec:
        x = rng.standard_normal((R, D)).astype(np.float32)
        t = torch.from_numpy(x).to(DEV)
        A = (et.SimpleEmbedding(t, Static(D)) if cpp == 0 else
             et.SplitEmbedding(t, cpp) if cpp > 1 else ColumnPointerTable(t, D + 4, gen))
        tabs.append(A)
        base.append(x)
        idx.append(_zipf(R, (Bb, P), gen))
    d = rng.standard_normal((Bb, D * len(spec))).astype(np.float32)
    dd = torch.from_numpy(d).to(DEV)
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, dd[:, k * D:(k + 1) * D], i)
             for k, (A, i) in enumerate(zip(tabs, idx))]
    et.update_(et.Descent(0.1), tabs, grads)  # default (exact) mode
    torch.cuda.synchronize()
    assert et.check_errors() == 0
    streamed = 0
    for k, ((R, _), A, I) in enumerate(zip(spec, tabs, idx)):
        ref = base[k].copy()
        oracle.sgd(ref, np.ascontiguousarray(d[:, k * D:(k + 1) * D]), I.cpu().numpy(), 0.1,
                   fused=True)
        got = A.data if isinstance(A, et.SimpleEmbedding) else _dense(A)
        assert got.cpu().numpy().tobytes() == ref.tobytes(), (k, R)
        if R > EC_MAX_ROWS:
            counts = torch.bincount(I.view(-1), minlength=R + 1)[1:]
            for c in torch.nonzero((counts > CHUNK) & (counts <= 20000)).view(-1).tolist():
                streamed += _chain_shape(I, c + 1)[0] >= 8
    assert streamed >= 3, streamed  # the regular list holds S >= 8 chains


@pytest.mark.parametrize("Bb", [16382, 16383])
def test_chain_offsets_at_the_32_bit_boundary(oracle, Bb):
    """Gradient offsets at the edge of the asm loops' 32-bit buffer range: a gradient with a
    65,536-float leading dimension, so bag * ld * 4 passes 2^31 from bag 8,192 on.  At 16,382
    bags (batch + 1) * ld * 4 < 2^32: the early (4 rows, S = 8) and regular (200 rows) chains
    take the streamed and packed asm loops with offsets up to 2^32 - 2^18; at 16,383 bags they
    do not fit and take the 64-bit walk (chain_asm_ok).  Both bit-identical to the oracle."""
    ld, dim = 65536, 64
    spec = [(4, 32), (200, 64), (60, 20)]  # (rows, pool)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(609)
    rng = np.random.default_rng(610)
    L = _lib.load()
    s = _lib.stream_handle()
    delta = torch.empty((Bb, ld), dtype=torch.float32, device=DEV)
    _lib.check(L.et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 6110, 0, -1.0, 1.0,
                                 s))
    tabs, idx, base = [], [], []
    for R, P in spec:
        x = rng.standard_normal((R, dim)).astype(np.float32)
        tabs.append(et.SimpleEmbedding(torch.from_numpy(x).to(DEV), Static(dim)))
        base.append(x)
        idx.append(_zipf(R, (Bb, P), gen))
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, k * dim:(k + 1) * dim], i)
             for k, (A, i) in enumerate(zip(tabs, idx))]
    et.update_(et.Descent(0.1), tabs, grads)  # default (exact) mode
    torch.cuda.synchronize()
    assert et.check_errors() == 0
    d = delta[:, :dim * len(spec)].cpu().numpy()
    del delta, grads
    torch.cuda.empty_cache()
    shapes = set()
    for k, ((R, _), A, I) in enumerate(zip(spec, tabs, idx)):
        ref = base[k].copy()
        oracle.sgd(ref, np.ascontiguousarray(d[:, k * dim:(k + 1) * dim]), I.cpu().numpy(), 0.1,
                   fused=True)
        assert A.data.cpu().numpy().tobytes() == ref.tobytes(), (Bb, k, R)
        counts = torch.bincount(I.view(-1), minlength=R + 1)[1:]
        shapes |= {_chain_shape(I, c + 1)[0] for c in torch.nonzero(counts > CHUNK).view(-1).tolist()}
    assert {1, 8} <= shapes or {1, 16} <= shapes, shapes  # packed and streamed loops both ran
