#!/usr/bin/env python3
"""Benchmark of the embedding-table hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], the metric's config): 26 fp32 tables of dim
128 with Criteo-Kaggle cardinalities (public DLRM statistics, NOT from the
reference — labelled as such), matrix-index pooled sum with pool 20, batch 65536,
PreallocationStrategy(0).  A step is one fused maplookup of the whole batch over
all 26 tables (one kernel launch at N = 1), inputs resident in HBM.

N > 1 (launched by torch.distributed.run, one rank per GPU): the tables are split
table-wise over the ranks (4,4,3,3,3,3,3,3 at N = 8); a step is each rank's fused
lookup of its tables + the RCCL all-gather of the slabs + the concat assembly, so
the whole-job throughput is B*T*P lookups per step time ("scaling": "strong").

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel
(k_pooled_vec, HIP events on the launch stream) and the CPU baseline (the oracle's
multithreaded restatement of the reference CPU path, timed on this host's cores on
the same tables and indices, with its output compared bit-for-bit to the GPU's).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "embeddingtables.jl_amd"))

# Criteo-Kaggle (DLRM) cardinalities — public statistics, not from the reference.
CRITEO_KAGGLE_ROWS = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683,
                      8351593, 3194, 27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15,
                      286181, 105, 142572]
DIM, POOL, BATCH = 128, 20, 65536
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
HBM_COPY_GBS = 6290.0  # measured float4-copy ceiling (MI355X_MICROARCH.md:36), SURVEY.md §8d
TABLE_SEED, INDEX_SEED = 1000, 2000


INFINITY_CACHE = 256 << 20  # MI355X die-level L3 (MI355X_MICROARCH.md, Infinity Cache)


def algorithmic_bytes(batch, pool, dims, es=4):
    """Per launch: every gathered row + every index + every output element
    (SURVEY.md §8d), summed over the tables (or table pieces) of the launch."""
    return sum(batch * pool * d * es + batch * pool * 8 + batch * d * es for d in dims)


def hbm_compulsory_bytes(batch, pool, dims, rows, es=4):
    """Per launch, the bytes that MUST come from HBM whatever the caches hold: the
    gathered rows of every table (piece) larger than the 256 MiB Infinity Cache (a
    smaller one can stay on die from one launch to the next), every index and every
    output element.  A lower bound on the launch's DRAM bytes, so bytes / time / 8 TB/s
    is a lower bound on the HBM fraction (<= 1 by construction)."""
    tot = 0
    for d, R in zip(dims, rows):
        tot += batch * pool * 8 + batch * d * es
        if R * d * es > INFINITY_CACHE:
            tot += batch * pool * d * es
    return tot


def host_cpus():
    """(host cores, CPUs this process may run on, cgroup CPU quota or None)."""
    cores = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = cores
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return cores, usable, quota


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=BATCH)
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="target CPU-baseline sample duration (0 disables)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU-baseline threads; 0 = every host core (os.cpu_count())")
    p.add_argument("--no-check", action="store_true", help="skip the CPU/GPU bit comparison")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the config-2 (gather) and config-4 (Zipf + SGD) measurements")
    p.add_argument("--force-shard", action="store_true",
                   help="use the sharded (all-gather + concat) step even on one rank")
    p.add_argument("--plan", choices=["featurewise", "tablewise"], default="tablewise",
                   help="N > 1: whole tables per rank, balanced by count (default, SURVEY.md "
                        "§8e), or equal feature ranges cut at 32-feature granules")
    p.add_argument("--chunks", type=int, default=4,
                   help="N > 1: batch chunks pipelined through lookup / all-gather / concat")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="N > 1 process group: nccl (= RCCL on ROCm) or gloo (rehearsal of "
                        "the N > 1 path with several ranks sharing one GPU)")
    p.add_argument("--p2p", action="store_true",
                   help="N>1: also time the one-sided exchange (IPC-mapped peers, et_push_cols)")
    p.add_argument("--no-alltoall", action="store_true",
                   help="N > 1: skip the extra all-to-all (batch-sliced output) measurement")
    p.add_argument("--subset", choices=["all", "heavy", "light"], default="all",
                   help="calibration only: tables above / below 4 MiB")
    p.add_argument("--rows", type=int, default=0,
                   help="calibration only: give every table this many rows (0 = Criteo)")
    p.add_argument("--min-rows", type=int, default=0,
                   help="calibration only: drop the tables with fewer rows")
    p.add_argument("--max-rows", type=int, default=0,
                   help="calibration only: drop the tables with more rows (0 = no limit)")
    return p.parse_args()


def make_tables(et, L, tids, device):
    import torch
    from embtab import _lib

    tables, idx = [], []
    stream = _lib.stream_handle(device)
    for t in tids:
        R = CRITEO_KAGGLE_ROWS[t]
        data = torch.empty((R, DIM), dtype=torch.float32, device=device)
        _lib.check(L.et_fill_uniform(_lib.ET_F32, data.data_ptr(), data.numel(), TABLE_SEED + t, 0,
                                     0.0, 1.0, stream))
        tables.append(et.SimpleEmbedding(data, et.Static(DIM)))
    return tables


def make_indices(L, tids, batch, device):
    import torch
    from embtab import _lib

    stream = _lib.stream_handle(device)
    idx = []
    for t in tids:
        I = torch.empty((batch, POOL), dtype=torch.int64, device=device)
        _lib.check(L.et_fill_index_uniform(I.data_ptr(), I.numel(), CRITEO_KAGGLE_ROWS[t],
                                           INDEX_SEED + t, 0, stream))
        idx.append(I)
    return idx


def cpu_baseline(gpu_out, idx, batch, seconds, threads, check):
    """Time the oracle's Preallocation maplookup (reference CPU algorithm, C + pthreads,
    atomic work queue with worksize_div = 8) on host copies of the same inputs."""
    import numpy as np

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc

    t0 = time.time()
    tabs = [orc.fill_uniform((R, DIM), np.float32, TABLE_SEED + t, 0, 0.0, 1.0, nthreads=threads)
            for t, R in enumerate(CRITEO_KAGGLE_ROWS)]
    hidx = [i.cpu().numpy() for i in idx]
    setup = time.time() - t0
    out = np.empty((batch, len(tabs) * DIM), np.float32)
    # one untimed pass (page-in), then whole steps until the time budget is spent
    orc.maplookup_prealloc(tabs, hidx, nthreads=threads, out=out)
    same = None
    if check:
        same = bool(np.array_equal(out, gpu_out))
    steps, t0 = 0, orc.now()
    while True:
        orc.maplookup_prealloc(tabs, hidx, nthreads=threads, out=out)
        steps += 1
        el = orc.now() - t0
        if el >= seconds or steps >= 1000:
            break
    lookups = steps * batch * len(tabs) * POOL
    cores, usable, quota = host_cpus()
    return {
        "value": lookups / el,
        "unit": "lookups/s",
        "cores": threads,
        "threads": threads,
        "host_cores": cores,
        "cpus_usable": usable,  # sched_getaffinity of this process
        "cgroup_cpu_quota": quota,  # cpu.max of this process's cgroup (None = no limit)
        "isa": "gcc -O3 -march=x86-64-v4 (AVX-512)",
        "kind": "port",
        "sample": f"{steps} full step(s) of the same workload ({batch} bags x {len(tabs)} tables "
                  f"x pool {POOL}, same tables and indices) in {el:.2f} s; C restatement of "
                  "src/lookup.jl:316-371 + :134-165 (oracle/embtab_oracle.c), pthreads atomic "
                  "work queue, worksize_div 8",
        "ms_per_step": 1e3 * el / steps,
        "gpu_output_bit_identical": same,
        "setup_s": round(setup, 2),
    }


def _timed(fn, steps, warmup, stream):
    """Average HIP-event time (ms) of fn() on `stream` over `steps` launches."""
    import torch

    for _ in range(warmup):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    torch.cuda.synchronize()
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / steps


def table_classes(et, tables, idx, tids, batch, stream, mixed_ms, steps=10, warmup=3):
    """The headline launch split by table class: every class's tables
    alone in one Preallocation launch of their own — heavy (> 256 MiB, rows from HBM), mid
    (4 MiB .. 256 MiB, Infinity-Cache resident), light (<= 4 MiB, one XCD's L2) — with its
    time, its §8d algorithmic rate and (heavy) its HBM-compulsory rate, so the gap between
    the mixed launch and the HBM roofline is traceable to a class."""
    import torch

    out = {}
    classes = (("heavy", lambda b: b > INFINITY_CACHE), ("mid", lambda b: (4 << 20) < b <= INFINITY_CACHE),
               ("light", lambda b: b <= (4 << 20)))
    total = 0.0
    for name, pick in classes:
        sel = [k for k, t in enumerate(tids) if pick(CRITEO_KAGGLE_ROWS[t] * DIM * 4)]
        if not sel:
            continue
        tabs = [tables[k] for k in sel]
        ids = [idx[k] for k in sel]
        dst = torch.empty((batch, DIM * len(sel)), dtype=torch.float32, device=tables[0].data.device)
        strat = et.PreallocationStrategy(0)
        ms = _timed(lambda: et.maplookup_(strat, dst, tabs, ids), steps, warmup, stream)
        rows = [CRITEO_KAGGLE_ROWS[tids[k]] for k in sel]
        alg = algorithmic_bytes(batch, POOL, [DIM] * len(sel))
        hbm = hbm_compulsory_bytes(batch, POOL, [DIM] * len(sel), rows)
        out[name] = {"tables": len(sel), "ms_alone": ms,
                     "algorithmic_GBs": alg / (ms * 1e-3) / 1e9,
                     "hbm_compulsory_GBs": hbm / (ms * 1e-3) / 1e9,
                     "hbm_compulsory_frac": hbm / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        tr = load_class_traffic(name)
        if tr and tr.get("hbm_bytes_per_launch"):  # committed per-class PMC (same launch alone)
            fb = tr["hbm_bytes_per_launch"]
            out[name].update({"fabric_bytes_per_launch": fb, "fabric_GBs": fb / (ms * 1e-3) / 1e9,
                              "fabric_over_compulsory": fb / hbm,
                              "l2_hit_rate": tr.get("l2_hit_rate"), "traffic_source": tr["file"]})
        total += ms
        del dst
    out["sum_alone_ms"] = total
    out["mixed_ms"] = mixed_ms
    return out


def bench_config2(et, L, device, steps, warmup, nsets=16):
    """BASELINE configs[1]: one 128 x 1e7 fp32 table, vector-index (non-reducing) gather,
    B = 65536.  Bytes per lookup: 512 read + 512 written + 8 index.

    Cold-cache method: `nsets` independent index sets (different seeds) are rotated over
    the back-to-back launches, so consecutive uses of one set are nsets - 1 launches
    apart; between them nsets x (33.5 MB of rows + 33.5 MB of output) = 1.07 GB pass
    through the die, 4x the 256 MiB Infinity Cache, so no launch finds its rows on die
    (a single repeated set — the round-1 method — measured the Infinity Cache instead)."""
    import torch
    from embtab import _lib

    R, B = 10_000_000, BATCH
    stream = torch.cuda.current_stream(device)
    data = torch.empty((R, DIM), dtype=torch.float32, device=device)
    _lib.check(L.et_fill_uniform(_lib.ET_F32, data.data_ptr(), data.numel(), 3000, 0, 0.0, 1.0,
                                 stream.cuda_stream))
    sets = []
    for k in range(nsets):
        I = torch.empty(B, dtype=torch.int64, device=device)
        _lib.check(L.et_fill_index_uniform(I.data_ptr(), B, R, 3001 + k, 0, stream.cuda_stream))
        sets.append(I)
    A = et.SimpleEmbedding(data, et.Static(DIM))
    dsts = [torch.empty((B, DIM), dtype=torch.float32, device=device) for _ in range(nsets)]

    def run(n, rotate=True):
        for k in range(n):
            j = k % nsets if rotate else 0
            et.lookup_(dsts[j], A, sets[j])

    run(warmup * nsets)
    # a ~12 us launch is timed over back-to-back launches (one event
    # pair around all of them), so the per-launch event overhead does not count
    n = max(steps, nsets) // nsets * nsets
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(rotate):
        torch.cuda.synchronize()
        a.record(stream)
        run(n, rotate)
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / n

    eager_ms = timed(True)
    warm_ms = timed(False)  # one repeated set: the Infinity-Cache rate, for reference only
    # the same rotated launches captured once in a HIP graph and replayed (a serving loop
    # without the host's per-call launch cost between the ~15 us kernels)
    reps = n // nsets
    graph = None
    if os.environ.get("BENCH_NO_GRAPH"):  # experiments: eager timing only
        ms = eager_ms
    else:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            run(nsets)
        if os.environ.get("BENCH_GRAPH_NOREPLAY"):  # experiments: capture only
            return {"kernel_ms": eager_ms}
        graph.replay()
        torch.cuda.synchronize()
        a.record(stream)
        for _ in range(reps):
            graph.replay()
        b.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / (reps * nsets)
    ok = all(bool(torch.equal(dsts[j], data[sets[j] - 1])) for j in range(nsets))  # bit copy
    nbytes = B * (DIM * 4 * 2 + 8)
    del data, dsts, graph
    return {"workload": "1 table 128 x 1e7 fp32, vector-index gather, B=65536",
            "lookups_per_s": B / (ms * 1e-3), "kernel_ms": ms,
            "timing": f"{reps} replays of a HIP graph of the {nsets} rotated launches, one "
                      "event pair around them (per launch)",
            "eager_ms": eager_ms, "lookups_per_s_eager": B / (eager_ms * 1e-3),
            "eager_timing": f"{n} back-to-back eager launches (Python + ctypes per call)",
            "cold_cache_method": f"{nsets} independent index sets rotated over the launches "
                                 f"({nsets} x 67 MB of rows + output between two uses of a "
                                 "set, 4x the 256 MiB Infinity Cache)",
            "achieved_GBs": nbytes / (ms * 1e-3) / 1e9,
            "frac_of_hbm_peak": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "frac_of_copy_ceiling": nbytes / (ms * 1e-3) / 1e9 / HBM_COPY_GBS,
            "warm_repeated_set_kernel_ms": warm_ms,
            "algorithmic_bytes_per_launch": nbytes, "bit_identical": ok}


def bench_alltoall(plan, rank, world, B, device, tables, idx, steps, warmup):
    """The DLRM layout: same lookups, but rank r keeps only its
    batch slice of the destination (RCCL all-to-all instead of all-gather)."""
    import torch
    import torch.distributed as dist
    from embtab.sharding import ShardedMapLookup

    a2a = ShardedMapLookup(plan, rank, world, B, torch.float32, device, exchange="alltoall")
    try:
        out = torch.empty((a2a.mine, plan.ld), dtype=torch.float32, device=device)
        for _ in range(warmup):
            a2a(tables, idx, out)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            a2a(tables, idx, out)
        torch.cuda.synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                          device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    finally:
        a2a.close()
    ms = 1e3 * float(el.item()) / steps
    return {"ms_per_step": ms, "value": B * len(plan.dims) * POOL / (ms * 1e-3),
            "unit": "lookups/s", "output": "batch slice per rank"}


def bench_p2p(plan, rank, world, B, device, tables, idx, steps, warmup, chunks):
    """One-sided exchange (fused P2P writes): lookups straight
    into this rank's columns of its destination, et_push_cols stores them into every
    peer's IPC-mapped destination, a one-element all-reduce publishes them."""
    import torch
    import torch.distributed as dist
    from embtab.sharding import ShardedMapLookup

    sm = ShardedMapLookup(plan, rank, world, B, torch.float32, device, exchange="p2p",
                          chunks=chunks)
    try:
        for _ in range(warmup):
            sm(tables, idx, None)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            sm(tables, idx, None)
        torch.cuda.synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                          device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    finally:
        torch.cuda.synchronize()
        dist.barrier()
        sm.close()
    ms = 1e3 * float(el.item()) / steps
    return {"ms_per_step": ms, "value": B * len(plan.dims) * POOL / (ms * 1e-3),
            "unit": "lookups/s", "output": "whole destination on every rank",
            "chunks": sm.chunks}


def zipf_indices(R, shape, alpha, gen, device):
    """Bounded Zipf(alpha) ranks over 1..R by the continuous inverse CDF, mapped through
    a seeded random permutation of the table."""
    import torch

    u = torch.rand(shape, generator=gen, device=device, dtype=torch.float64)
    a1 = 1.0 - alpha
    x = torch.floor(((float(R) ** a1 - 1.0) * u + 1.0) ** (1.0 / a1)).clamp_(1, R).long()
    perm = torch.randperm(R, generator=gen, device=device)
    return perm[x - 1] + 1


def bench_config4(et, tables, tids, device, steps, warmup, batch):
    """BASELINE configs[3]: the 26 tables, Zipf(1.05) indices, forward maplookup +
    SparseEmbeddingUpdate fused Descent(0.1) over all tables (one SGD pipeline)."""
    import torch
    from embtab import _lib

    stream = torch.cuda.current_stream(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(4000)
    idx = [zipf_indices(CRITEO_KAGGLE_ROWS[t], (batch, POOL), 1.05, gen, device) for t in tids]
    ld = DIM * len(tables)
    dst = torch.empty((batch, ld), dtype=torch.float32, device=device)
    delta = torch.empty((batch, ld), dtype=torch.float32, device=device)
    _lib.check(_lib.load().et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 4001, 0,
                                           -1.0, 1.0, stream.cuda_stream))
    strat = et.PreallocationStrategy(0)
    opt = et.Descent(0.1)
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, k * DIM:(k + 1) * DIM], i)
             for k, (A, i) in enumerate(zip(tables, idx))]
    indexers = [et.Indexer() for _ in tables]

    def fwd():
        et.maplookup_(strat, dst, tables, idx)

    def upd():
        et.update_(opt, tables, grads, indexers)

    def step():
        fwd()
        upd()

    # (The step with update!'s index phase on a second stream beside the forward —
    # et.PhasedUpdate, src/sparseupdate.jl:210-213 — is no longer timed here: in exact mode
    # the early chains start with the update call, so that ordering measured 6.49-6.60 ms
    # against 5.22-5.46 serial in rounds 3-4)
    fwd_ms = _timed(fwd, steps, warmup, stream)
    upd_ms = _timed(upd, steps, warmup, stream)
    step_ms = _timed(step, steps, warmup, stream)
    # the other update mode, and how far the split mode lies from the exact (reference-
    # order, src/sparseupdate.jl:110-127) result: both from the same tables, every element
    # (the default resolves to the exact mode for these Float32 tables: ET_FLAG_EXACT_IF_FAST)
    other_ms = _timed(lambda: et.update_(opt, tables, grads, indexers, exact=False), steps,
                      warmup, stream)
    w0 = [A.data.clone() for A in tables]
    res = {}
    for mode in (True, False):
        et.update_(opt, tables, grads, None, exact=mode)
        torch.cuda.synchronize()
        res[mode] = [A.data.clone() for A in tables]
        for A, w in zip(tables, w0):
            A.data.copy_(w)
    worst, over, differ = 0.0, 0, 0
    for e, sp in zip(res[True], res[False]):
        rel = (sp.double() - e.double()).abs() / e.double().abs().clamp_min(1e-30)
        worst = max(worst, float(rel.max()))
        over += int((rel > 1e-6).sum())
        differ += int((sp != e).sum())
    del res, w0
    torch.cuda.empty_cache()
    exact_ms, split_ms = upd_ms, other_ms
    U = sum(int(torch.unique(i).numel()) for i in idx)
    occ = batch * POOL * len(tables)
    upd_bytes = occ * 8 + batch * len(tables) * DIM * 4 + 2 * U * DIM * 4
    hot = max(int(torch.bincount(i.view(-1)).max()) for i in idx)
    return {"workload": "26 Criteo tables x 128 fp32, Zipf(1.05) pool-20 indices, B=65536: "
                        "Preallocation forward + fused Descent(0.1) update of every table",
            "lookups_per_s": occ / (step_ms * 1e-3), "step_ms": step_ms,
            "step_order": "serial",
            "forward_ms": fwd_ms, "update_ms": upd_ms,
            "update_mode": "exact",
            "update_exact_ms": exact_ms, "update_split_ms": split_ms,
            "exact_over_split": exact_ms / split_ms,
            # the split mode (long columns as ordered partial sums) against the exact one,
            # over all 26 x 128 x R_t table elements after one update
            "split_vs_exact_max_rel": worst, "split_elements_over_1e-6_rel": over,
            "split_elements_differing": differ,
            "distinct_rows_U": U, "hottest_row_occurrences": hot,
            "update_algorithmic_bytes": upd_bytes,
            "update_achieved_GBs": upd_bytes / (upd_ms * 1e-3) / 1e9,
            "update_delta_gather_bytes": occ * DIM * 4,
            # the bytes the gather-by-column algorithm itself moves: one delta column per
            # occurrence (before the repeated-bag dedupe), the table RMW and the indices
            "update_gather_inclusive_GBs":
                (occ * DIM * 4 + 2 * U * DIM * 4 + occ * 8) / (upd_ms * 1e-3) / 1e9}


def bench_config3_fp16(et, L, tids, idx, device, steps, warmup, batch):
    """SURVEY.md §8f rank 4 / north_star "fp32/fp16 embedding columns": the config-3
    workload with Float16 tables (same seeds, 8.6 GB), in the reference's Float16
    arithmetic (every add rounded to half, as Julia's) and with fp32 accumulation
    (ET_FLAG_F16_FP32_ACC, one rounding).  An extra line, never the headline."""
    import torch
    from embtab import _lib

    stream = torch.cuda.current_stream(device)
    tabs = []
    for t in tids:
        R = CRITEO_KAGGLE_ROWS[t]
        data = torch.empty((R, DIM), dtype=torch.float16, device=device)
        _lib.check(L.et_fill_uniform(_lib.ET_F16, data.data_ptr(), data.numel(), TABLE_SEED + t, 0,
                                     0.0, 1.0, stream.cuda_stream))
        tabs.append(et.SimpleEmbedding(data, et.Static(DIM)))
    dst = torch.empty((batch, DIM * len(tabs)), dtype=torch.float16, device=device)
    strat = et.PreallocationStrategy(0)
    out = {"workload": "config 3 with Float16 tables (26 x 128, pool 20, B = 65536)"}
    rows = [CRITEO_KAGGLE_ROWS[t] for t in tids]
    hbm = hbm_compulsory_bytes(batch, POOL, [DIM] * len(tabs), rows, es=2)
    alg = algorithmic_bytes(batch, POOL, [DIM] * len(tabs), es=2)
    for key, acc in (("julia_f16_arith", False), ("fp32_accumulate", True)):
        plan = et.PreallocationPlan(strat, dst, tabs, idx, True, acc)
        ms = _timed(plan, steps, warmup, stream)
        out[key] = {"kernel_ms": ms, "lookups_per_s": batch * len(tabs) * POOL / (ms * 1e-3),
                    "hbm_compulsory_GBs": hbm / (ms * 1e-3) / 1e9,
                    "hbm_frac": hbm / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                    "algorithmic_GBs": alg / (ms * 1e-3) / 1e9}
    out["hbm_compulsory_bytes_per_launch"] = hbm
    del tabs, dst
    torch.cuda.empty_cache()
    return out


def load_class_traffic(name):
    """The latest committed PMC traffic of one headline table class launched alone
    (profiles/rNN/classpmc/traffic_<class>.json: tools/class_pmc.py + tools/traffic.py)."""
    import glob

    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "classpmc",
                                              f"traffic_{name}.json")), reverse=True):
        try:
            with open(path) as f:
                doc = json.load(f)
            doc["file"] = os.path.relpath(path, REPO)
            return doc
        except (OSError, ValueError):
            continue
    return None


def load_traffic():
    """The latest committed PMC traffic summary of the headline kernel
    (profiles/traffic_rNN.json, written by tools/traffic.py)."""
    import glob

    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "traffic_r*.json")),
                       reverse=True):
        try:
            with open(path) as f:
                doc = json.load(f)
            doc["file"] = os.path.relpath(path, REPO)
            return doc
        except (OSError, ValueError):
            continue
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import embtab as et
    from embtab import _lib
    from embtab.sharding import ShardedMapLookup, ShardPlan, compact_piece_table

    if args.rows:
        CRITEO_KAGGLE_ROWS[:] = [args.rows] * len(CRITEO_KAGGLE_ROWS)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("run N>1 under torch.distributed.run (one rank per GPU)")
    ndev = torch.cuda.device_count()
    local_dev = local_rank % ndev if args.backend == "gloo" else local_rank
    torch.cuda.set_device(local_dev)
    device = torch.device("cuda", local_dev)
    if world > 1:
        if args.backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
    L = _lib.load()
    B = args.batch
    if args.subset != "all":
        keep = [r for r in CRITEO_KAGGLE_ROWS if (r * DIM * 4 > (4 << 20)) == (args.subset == "heavy")]
        CRITEO_KAGGLE_ROWS[:] = keep
    if args.min_rows or args.max_rows:
        CRITEO_KAGGLE_ROWS[:] = [r for r in CRITEO_KAGGLE_ROWS if r >= args.min_rows and
                                 (args.max_rows == 0 or r <= args.max_rows)]
    T = len(CRITEO_KAGGLE_ROWS)
    dims = [DIM] * T
    sharded = world > 1 or args.force_shard
    if sharded:
        # table-wise: dealt by size so the 5 tables above 256 MiB land on distinct ranks
        # (SURVEY.md §8e); counts stay 4,4,3,3,3,3,3,3 at N = 8
        plan = (ShardPlan.featurewise(dims, world) if args.plan == "featurewise"
                else ShardPlan.tablewise(dims, world, sizes=CRITEO_KAGGLE_ROWS))
        mine = plan.tables_of(rank)
        pieces = plan.pieces[rank]
        tables = []
        for t in mine:  # only the owned tables / feature slices stay resident
            (full_t,) = make_tables(et, L, [t], device)
            tables += [(k, compact_piece_table(full_t, p)) for k, p in enumerate(pieces)
                       if p.table == t]
            del full_t
        tables = [tb for _, tb in sorted(tables, key=lambda x: x[0])]
        fidx = dict(zip(mine, make_indices(L, mine, B, device)))
        idx = [fidx[p.table] for p in pieces]
        torch.cuda.empty_cache()
        local_dims = [p.dim for p in pieces]
        shard = ShardedMapLookup(plan, rank, world, B, torch.float32, device,
                                 exchange="allgather", chunks=args.chunks)
    else:
        mine = list(range(T))
        tables = make_tables(et, L, mine, device)
        idx = make_indices(L, mine, B, device)
        local_dims = dims
    dst = torch.empty((B, sum(dims)), dtype=torch.float32, device=device)
    strat = et.PreallocationStrategy(0)

    def step():
        if sharded:
            shard(tables, idx, dst)
        else:
            et.maplookup_(strat, dst, tables, idx)

    torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # kernel-level timing of the dominant launch(es) on the stream they run on
    stream = torch.cuda.current_stream(device)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        if sharded:
            shard(tables, idx, dst)  # lookups on `stream`, exchange on a second stream
        else:
            et.maplookup_(strat, dst, tables, idx)
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=device if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if sharded:  # lookup-only time: the chunked lookups alone, same launches, no exchange
        torch.cuda.synchronize()
        for k in range(args.steps):
            ev[k][0].record(stream)
            for c in range(shard.chunks):
                shard.lookup_chunk(tables, idx, shard.bounds[c], shard.bounds[c + 1])
            ev[k][1].record(stream)
        torch.cuda.synchronize()
    kernel_times = sorted(a.elapsed_time(b) for a, b in ev)
    kernel_ms = sum(kernel_times) / args.steps
    kernel_ms_median = kernel_times[len(kernel_times) // 2]

    lookups_per_step = B * T * POOL
    value = lookups_per_step * args.steps / elapsed
    local_bytes = algorithmic_bytes(B, POOL, local_dims)
    local_rows = ([CRITEO_KAGGLE_ROWS[p.table] for p in pieces] if sharded
                  else [CRITEO_KAGGLE_ROWS[t] for t in mine])
    hbm_bytes = hbm_compulsory_bytes(B, POOL, local_dims, local_rows)
    achieved = hbm_bytes / (kernel_ms * 1e-3) / 1e9
    algorithmic_GBs = local_bytes / (kernel_ms * 1e-3) / 1e9
    traffic = load_traffic()
    traffic_bytes = None
    if traffic and traffic.get("workload") == f"criteo26_b{B}" and world == 1:
        traffic_bytes = traffic.get("hbm_bytes_per_launch")

    result = {
        "metric": "embedding lookups/sec + achieved HBM GB/s (% of roofline), 26 tables x dim128 "
                  "at B=65536",
        "value": value,
        "unit": "lookups/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: counter-hash uniform[0,1) fp32 tables, uniform 1-based Int64 indices "
                "(seeded, identical on CPU and GPU)",
        "config": {
            "workload": "criteo-kaggle 26 tables x dim 128 fp32, pooled sum pool 20, "
                        "PreallocationStrategy(0)",
            "global_batch": B,
            "tables": T,
            "pool": POOL,
            "dim": DIM,
            "table_rows": CRITEO_KAGGLE_ROWS,
            "parallelism": "single GPU" if not sharded else
                           ("feature-wise: equal contiguous feature ranges per GPU, tables "
                            "cut at 32-feature granules" if args.plan == "featurewise"
                            else "table-wise: whole tables per GPU, balanced by count and dealt "
                                 "by size so the largest land on distinct GPUs (SURVEY.md §8e)")
                           + f" x{world} + "
                           f"{'RCCL' if args.backend == 'nccl' else 'gloo'} all-gather concat "
                           f"({shard.chunks} pipelined batch chunks; "
                           f"{'C-ABI et_sharded_maplookup' if shard._native else 'torch.distributed exchange'})",
        },
        "bags_per_s": B * T * args.steps / elapsed,
        "samples_per_s": B * args.steps / elapsed,
        "roofline": {
            "bound": "hbm",
            "kernel": "k_pooled_vec_queued<float,float,128,8,NT,SG=1> (scalar-addressed, per-XCD queues)",
            # achieved = HBM-compulsory bytes (rows of the tables larger than the 256 MiB
            # Infinity Cache + all indices + the output) / average launch time: a lower
            # bound on the DRAM rate, so frac <= 1; the cache-inclusive SURVEY.md §8d
            # figure is algorithmic_GBs / algorithmic_frac below
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "bytes_basis": "HBM-compulsory: gathered rows of tables > 256 MiB + indices + output",
            "hbm_compulsory_bytes_per_launch": hbm_bytes,
            "algorithmic_GBs": algorithmic_GBs,
            "algorithmic_frac": algorithmic_GBs / HBM_PEAK_GBS,
            "traffic": traffic_bytes,
            "traffic_source": traffic.get("file") if traffic_bytes else None,
            # fabric-side bytes (PMC, per launch) over the same launch time: how close the
            # memory system itself runs to the HBM peak (cache-resident tables make the
            # algorithmic rate exceed it)
            "traffic_GBs": (traffic_bytes / (kernel_ms * 1e-3) / 1e9) if traffic_bytes else None,
            "traffic_frac": (traffic_bytes / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                             if traffic_bytes else None),
            # the same fabric rate against the measured float4-copy ceiling (6.29 TB/s)
            "traffic_frac_of_copy_ceiling": (traffic_bytes / (kernel_ms * 1e-3) / 1e9 /
                                             HBM_COPY_GBS if traffic_bytes else None),
            "algorithmic_bytes_per_launch": local_bytes,
            "kernel_ms": kernel_ms,
            "kernel_ms_median": kernel_ms_median,
        },
    }
    if not sharded and world == 1 and not args.no_extra:
        result["roofline"]["classes"] = table_classes(et, tables, idx, mine, B, stream,
                                                      kernel_ms)
    if sharded:
        result["lookup_only_ms"] = kernel_ms
        result["slab_cols"] = plan.slab_ld
        # what every rank holds: its tables (or feature slices) only
        mem = {"rank": rank, "tables": mine, "pieces": [(p.table, p.f0, p.dim) for p in pieces],
               "table_bytes": sum(tb.data.numel() * tb.data.element_size() for tb in tables)}
        every = [None] * world
        if world > 1:
            dist.all_gather_object(every, mem)
        else:
            every = [mem]
        result["per_rank"] = every
        if world > 1 and not args.no_alltoall:
            try:  # an extra measurement: never lose the main line to it
                result["alltoall"] = bench_alltoall(plan, rank, world, B, device, tables, idx,
                                                    max(5, args.steps // 2), 2)
            except Exception as e:  # noqa: BLE001
                result["alltoall"] = {"error": f"{type(e).__name__}: {e}"}
        if world > 1 and args.p2p:
            try:
                result["p2p"] = bench_p2p(plan, rank, world, B, device, tables, idx,
                                          max(5, args.steps // 2), 2, args.chunks)
            except Exception as e:  # noqa: BLE001
                result["p2p"] = {"error": f"{type(e).__name__}: {e}"}
    if world == 1 and not args.no_extra and not sharded:
        # config 3 also at prependrows k = 16 (dst ld = 16 + 3328)
        dst16 = torch.empty((B, 16 + sum(dims)), dtype=torch.float32, device=device)
        ms16 = _timed(lambda: et.maplookup_(et.PreallocationStrategy(16), dst16, tables, idx),
                      max(10, args.steps // 2), 2, stream)
        result["config3_prepend16"] = {"kernel_ms": ms16,
                                       "lookups_per_s": lookups_per_step / (ms16 * 1e-3)}
        del dst16
    if world == 1 and not args.no_extra:
        result["config3_fp16"] = bench_config3_fp16(et, L, mine, idx, device, 20, 3, B)
        # config 2 (which captures a HIP graph) before config 4: since round 5 the library
        # opens the exact update's side queues at its first call, so queues opened later (a
        # capture's, another stream's) no longer land on the caller's pipe
        result["config2_gather"] = bench_config2(et, L, device, 320, 2)
        result["config4_zipf_update"] = bench_config4(et, tables, mine, device, 10, 2, B)
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        gpu_out = None if args.no_check else dst.cpu().numpy()
        if args.cpu_threads:
            result["cpu_baseline"] = cpu_baseline(gpu_out, idx, B, args.cpu_seconds,
                                                  args.cpu_threads, not args.no_check)
        else:
            # every host core, and the CPUs the job's cgroup may actually use (the GPU
            # box caps a job at 16 CPUs of its 256: cpu.max); the faster run is the
            # baseline, both are reported
            cores, _, quota = host_cpus()
            widths = [cores] + ([int(quota)] if quota and int(quota) < cores else [])
            runs = [cpu_baseline(gpu_out, idx, B, args.cpu_seconds if k == 0 else
                                 max(2.0, args.cpu_seconds / 3), w, not args.no_check and k == 0)
                    for k, w in enumerate(widths)]
            best = max(runs, key=lambda r: r["value"])
            best["widths_tried"] = {str(r["threads"]): r["value"] for r in runs}
            if best is not runs[0]:
                best["gpu_output_bit_identical"] = runs[0]["gpu_output_bit_identical"]
            result["cpu_baseline"] = best
    if _lib.EXPERIMENT_BUILD:  # tools/ A/B runs only (ET_TOOLS_EXPERIMENT=1): say so
        result["library"] = f"EXPERIMENT BUILD {_lib.LIB_PATH} (not the shipped library)"
    if rank == 0:
        print(json.dumps(result), flush=True)
    if sharded:
        shard.close()  # the native step's stream, events and RCCL communicator
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
