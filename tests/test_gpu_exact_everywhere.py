"""The default update is the reference's exact serial sum at every size and element type
(VERDICT r04 items 2 / weak #1), and the per-XCD queue schedule runs on a caller-owned
queue block.

The reference sums every distinct column's gradient serially in occurrence order
(src/sparseupdate.jl:110-127; :199-238 for the multi-table update, Δ sliced as in
src/lookup.jl:374-389) whatever the batch and the gradient's leading dimension.  Round 4's
default (ET_FLAG_EXACT_IF_FAST) quietly fell back to the reassociating split mode when a
gradient's byte offsets passed 32 bits (batch * ld_delta >= 2^30) and for non-Float32
tables; since ABI v9 those chains run on 64-bit addresses (chain_walk_wide) and the default
stays exact.  Checked here bit for bit against the oracle's serial update."""
import ctypes
import threading

import numpy as np
import pytest
import torch

import embtab as et
from embtab import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _zipf(R, shape, gen):
    u = torch.rand(shape, generator=gen, device=DEV, dtype=torch.float64)
    a1 = 1.0 - 1.05
    x = torch.floor(((float(R) ** a1 - 1.0) * u + 1.0) ** (1.0 / a1)).clamp_(1, R).long()
    return torch.randperm(R, generator=gen, device=DEV)[x - 1] + 1


def _check_columns(oracle, A, W0, I, dl, P, cols, feats):
    """The oracle's serial fused update (reference order) of columns `cols` on the feature
    subset `feats` (features are independent in the reference's sum), bit for bit."""
    for c in cols:
        occ = torch.nonzero(I.view(-1) == c + 1).view(-1)  # occurrence order
        n = len(occ)
        if n == 0:
            continue
        dsub = dl[:, feats][occ // P].cpu().numpy()        # one delta row per occurrence
        w = W0[c:c + 1, feats].cpu().numpy().copy()
        oracle.sgd(w, dsub, np.ones(n, np.int64), 0.1, fused=True)
        got = A.data[c, feats].cpu().numpy()
        assert w[0].tobytes() == got.tobytes(), (c, n)
        del dsub


def test_default_exact_past_32bit_gradient_offsets(oracle):
    """B = 262,144 with a Preallocation gradient of ld 4,352 (k = 1,024
    prepended rows + 26 x 128 features; the checked tables' blocks at the top of it), so a
    chain's gradient byte offsets reach bag * ld * 4 = 4.56e9 > 2^32.  The DEFAULT mode
    (exact=None) is bit-identical to the oracle's serial update on every table's three
    hottest and 8 sampled columns — the early chains of the 3-row table (3.5 M occurrences
    in its hottest column), the early hot columns and the regular chains of the larger
    ones, all on 64-bit addresses."""
    Bb, P, D, k = 262144, 20, 128, 1024
    ld = k + 26 * D
    assert ld == 4352 and Bb * ld >= (1 << 30)
    rows = [3, 1460, 93145, 2202608]
    gen = torch.Generator(device=DEV)
    gen.manual_seed(77)
    L = _lib.load()
    s = _lib.stream_handle()
    tabs, idx = [], []
    for t, R in enumerate(rows):
        x = torch.empty((R, D), dtype=torch.float32, device=DEV)
        _lib.check(L.et_fill_uniform(_lib.ET_F32, x.data_ptr(), x.numel(), 7000 + t, 0, 0.0, 1.0,
                                     s))
        tabs.append(et.SimpleEmbedding(x, et.Static(D)))
        idx.append(_zipf(R, (Bb, P), gen))
    delta = torch.empty((Bb, ld), dtype=torch.float32, device=DEV)  # 4.56 GB
    _lib.check(L.et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 7100, 0, -1.0, 1.0,
                                 s))
    off = [ld - (len(rows) - t) * D for t in range(len(rows))]  # the last rows of the gradient
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, o:o + D], i)
             for A, o, i in zip(tabs, off, idx)]
    before = [A.data.clone() for A in tabs]
    et.update_(et.Descent(0.1), tabs, grads, [et.Indexer() for _ in tabs])  # default mode
    torch.cuda.synchronize()
    assert et.check_errors() == 0
    g = torch.Generator().manual_seed(8)
    feats = torch.tensor([0, 1, 31, 63, 64, 100, 127], device=DEV)
    hottest = 0
    for t, R in enumerate(rows):
        A, I, W0 = tabs[t], idx[t], before[t]
        counts = torch.bincount(I.view(-1), minlength=R + 1)[1:]
        hottest = max(hottest, int(counts.max()))
        touched = torch.nonzero(counts).view(-1)
        mask = torch.ones(R, dtype=torch.bool, device=DEV)
        mask[touched] = False
        assert torch.equal(A.data[mask], W0[mask])  # untouched columns unchanged
        pick = touched[torch.randperm(len(touched), generator=g)[:8].to(DEV)]
        pick = torch.unique(torch.cat([pick, torch.topk(counts, min(3, R)).indices]))
        _check_columns(oracle, A, W0, I, grads[t].delta, P, pick.tolist(), feats)
    assert hottest > 3_000_000
    del delta, grads, before, tabs, idx
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kind", ["f64", "f16", "f16acc", "bf16"])
def test_default_exact_typed_hot_columns(oracle, kind):
    """Float64 / Float16 / BFloat16 tables: the default update is the exact serial sum too
    (round 4 gave them the split mode by default).  A 3-row table (early chains: its
    hottest column has ~40 K occurrences, entries of up to 16 adds) and a 1,000-row one
    (regular chains of > 256 occurrences), Zipf batch, single-table update!: every column
    bit-identical to the oracle's typed model (oracle/embtab_oracle.c)."""
    from oracle import bf16_to_f32, f32_to_bf16  # noqa: F401

    from embtab.tables import fused_update_path

    rng = np.random.default_rng(21)
    Bb, P, dim = 4096, 20, 64
    gen = torch.Generator(device=DEV)
    gen.manual_seed(22)
    npdt = {"f64": np.float64, "f16": np.float16, "f16acc": np.float16}
    for R in (3, 1000):
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
        A = et.SimpleEmbedding(tdev, et.Static(dim))
        g = et.SparseEmbeddingUpdate(A.lookup_type, ddev, I)
        et.update_(et.Descent(0.1), A, g, f16_fp32_acc=kind == "f16acc")  # default mode
        ref = base.copy()
        oracle.sgd(ref, delta, I.cpu().numpy(), 0.1, fused=fused_update_path(A),
                   bf16=kind == "bf16", f16_fp32_acc=kind == "f16acc")
        got = A.data.view(torch.int16) if kind != "f64" else A.data
        got = got.cpu().numpy()
        counts = np.bincount(I.cpu().numpy().ravel(), minlength=R + 1)[1:]
        assert counts.max() > 256  # chains ran
        assert got.tobytes() == ref.view(got.dtype).tobytes(), (kind, R)


def _queue_tables(n=5, R=(1000, 50000, 7, 300000, 64), D=128, B=4096, P=20):
    rng = np.random.default_rng(5)
    hs = [rng.random((r, D), dtype=np.float32) for r in R[:n]]
    hi = [rng.integers(1, r + 1, (B, P)) for r in R[:n]]
    return hs, hi


def test_queue_block_caller_owned(oracle):
    """et_maplookup_prealloc_q (ABI v9): the per-XCD queue schedule on a zeroed block the
    caller owns gives the oracle's concat bit for bit, leaves the block zero after every
    launch (so the next ordered call may reuse it), and NULL is the static schedule."""
    hs, hi = _queue_tables()
    tabs = [torch.from_numpy(h).to(DEV) for h in hs]
    idx = [torch.from_numpy(i).to(DEV) for i in hi]
    B, D = hi[0].shape[0], hs[0].shape[1]
    descs = (_lib.LookupDesc * len(tabs))()
    for t, (A, I) in enumerate(zip(tabs, idx)):
        descs[t] = _lib.LookupDesc(A.data_ptr(), D, A.shape[0], D, I.shape[1], I.data_ptr(),
                                   I.shape[1], t * D, 0)
    ref = oracle.maplookup_prealloc(hs, hi, prependrows=0)
    L = _lib.load()
    q = torch.zeros(_lib.ET_LOOKUP_QUEUE_BYTES // 4, dtype=torch.int32, device=DEV)
    for use_q in (True, True, True, False):
        dst = torch.full((B, D * len(tabs)), float("nan"), dtype=torch.float32, device=DEV)
        _lib.check(L.et_maplookup_prealloc_q(_lib.ET_F32, ctypes.addressof(descs), len(tabs), B,
                                             dst.data_ptr(), D * len(tabs), 1,
                                             q.data_ptr() if use_q else None,
                                             _lib.stream_handle()))
        torch.cuda.synchronize()
        assert dst.cpu().numpy().tobytes() == np.ascontiguousarray(ref).tobytes()
        assert int(q.abs().sum()) == 0
    # a misaligned block is refused before any launch
    rc = L.et_maplookup_prealloc_q(_lib.ET_F32, ctypes.addressof(descs), len(tabs), B,
                                   dst.data_ptr(), D * len(tabs), 1, q.data_ptr() + 4,
                                   _lib.stream_handle())
    assert rc == -1  # ET_ERR_ARG


def test_queue_blocks_per_thread_and_stream(oracle):
    """Two host threads, each with its own stream, run the Preallocation maplookup at the
    same time, 20 times each: each (device, stream, thread) has its own queue block, so the
    per-XCD queues of concurrent launches never mix, and every result equals
    the oracle's concat."""
    hs, hi = _queue_tables()
    tabs = [et.SimpleEmbedding(torch.from_numpy(h).to(DEV), et.Static(128)) for h in hs]
    idx = [torch.from_numpy(i).to(DEV) for i in hi]
    ref = np.ascontiguousarray(oracle.maplookup_prealloc(hs, hi, prependrows=0)).tobytes()
    errs, bad = [], []

    def body(k):
        try:
            st = torch.cuda.Stream(DEV)
            with torch.cuda.stream(st):
                dst = torch.empty((hi[0].shape[0], 128 * len(tabs)), dtype=torch.float32,
                                  device=DEV)
                plan = et.PreallocationPlan(et.PreallocationStrategy(), dst, tabs, idx)
                outs = []
                for _ in range(20):
                    plan()
                    outs.append(dst.clone())
                st.synchronize()
                bad.extend(k for o in outs if o.cpu().numpy().tobytes() != ref)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=body, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    assert not any(t.is_alive() for t in th)
    assert not bad


@pytest.mark.parametrize("kind", ["f64", "f16", "f16acc", "bf16"])
def test_default_exact_typed_early_hot_columns(oracle, kind):
    """the typed chain walk on the EARLY HOT list (k_sgd_chains_x<T, C> and the EH
    plan on non-Float32 tables).  A 3,000-row table at B = 65,536, pool 20: its hottest Zipf
    columns (~140 K occurrences, above the 32,768 the sampled plan needs) are early hot
    columns, the next ones regular chains; single-table default update!, every column
    bit-identical to the oracle's typed model."""
    from oracle import f32_to_bf16

    from embtab.tables import fused_update_path

    rng = np.random.default_rng(31)
    Bb, P, dim, R = 65536, 20, 64, 3000
    gen = torch.Generator(device=DEV)
    gen.manual_seed(32)
    npdt = {"f64": np.float64, "f16": np.float16, "f16acc": np.float16}
    x = rng.standard_normal((R, dim)).astype(np.float32)
    d = rng.standard_normal((Bb, dim)).astype(np.float32)
    if kind == "bf16":
        base, delta = f32_to_bf16(x), f32_to_bf16(d)
    else:
        base, delta = x.astype(npdt[kind]), d.astype(npdt[kind])
    I = _zipf(R, (Bb, P), gen)
    tdev, ddev = torch.from_numpy(base).to(DEV), torch.from_numpy(delta).to(DEV)
    if kind == "bf16":
        tdev, ddev = tdev.view(torch.bfloat16), ddev.view(torch.bfloat16)
    A = et.SimpleEmbedding(tdev, et.Static(dim))
    et.update_(et.Descent(0.1), A, et.SparseEmbeddingUpdate(A.lookup_type, ddev, I),
               f16_fp32_acc=kind == "f16acc")
    ref = base.copy()
    oracle.sgd(ref, delta, I.cpu().numpy(), 0.1, fused=fused_update_path(A), bf16=kind == "bf16",
               f16_fp32_acc=kind == "f16acc")
    counts = np.bincount(I.cpu().numpy().ravel(), minlength=R + 1)[1:]
    assert counts.max() > 2 * 32768  # early hot columns
    got = (A.data.view(torch.int16) if kind != "f64" else A.data).cpu().numpy()
    assert got.tobytes() == ref.view(got.dtype).tobytes(), kind
    assert et.check_errors() == 0


def test_default_exact_f32_wide_walk_for_a_long_gradient_stride(oracle):
    """the Float32 chain walk with 64-bit addresses when the gradient's stride
    reaches 2^22 elements (chain_asm_ok fails on ld, not on the batch): a 3-row table's early
    chains (hottest column ~700 occurrences) at B = 64, pool 20, with the gradient a column
    block of a (64, 2^22 + 256) matrix, bit-identical to the oracle."""
    Bb, P, dim, R = 64, 20, 128, 3
    ld = (1 << 22) + 256
    gen = torch.Generator(device=DEV)
    gen.manual_seed(41)
    big = torch.empty((Bb, ld), dtype=torch.float32, device=DEV)  # 1.07 GB
    L = _lib.load()
    _lib.check(L.et_fill_uniform(_lib.ET_F32, big.data_ptr(), big.numel(), 4100, 0, -1.0, 1.0,
                                 _lib.stream_handle()))
    delta = big[:, ld - dim:]
    assert delta.stride(0) >= (1 << 22)
    x = torch.rand((R, dim), generator=gen, device=DEV, dtype=torch.float32)
    I = _zipf(R, (Bb, P), gen)
    A = et.SimpleEmbedding(x.clone(), et.Static(dim))
    et.update_(et.Descent(0.1), A, et.SparseEmbeddingUpdate(A.lookup_type, delta, I))
    ref = x.cpu().numpy()
    oracle.sgd(ref, delta.cpu().numpy(), I.cpu().numpy(), 0.1, fused=True)
    counts = np.bincount(I.cpu().numpy().ravel(), minlength=R + 1)[1:]
    assert counts.max() > 256  # a chain
    assert A.data.cpu().numpy().tobytes() == ref.tobytes()
    assert et.check_errors() == 0
    del big
    torch.cuda.empty_cache()
