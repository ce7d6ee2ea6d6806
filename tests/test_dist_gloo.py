"""Table-wise sharded Preallocation maplookup on 2 CPU ranks (gloo): the real
plan / layout / all-gather / assembly-plan code of embtab.sharding, with the oracle
standing in for the two device kernels (et_maplookup_prealloc into the slab and
et_concat_slabs), checked against the single-process Preallocation result."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from embtab.sharding import ShardLayout, ShardedPreallocation, plan_tables


def test_plan_tables_counts():
    a = plan_tables(26, 8)
    assert [len(x) for x in a] == [4, 4, 3, 3, 3, 3, 3, 3]
    assert sorted(t for x in a for t in x) == list(range(26))
    rows = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194,
            27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572]
    b = plan_tables(26, 8, sizes=rows)
    big5 = sorted(range(26), key=lambda t: -rows[t])[:5]
    owners = [next(r for r, x in enumerate(b) if t in x) for t in big5]
    assert len(set(owners)) == 5  # the five largest tables on distinct GPUs
    assert [len(x) for x in b] == [4, 4, 3, 3, 3, 3, 3, 3]
    assert plan_tables(26, 2) == [list(range(13)), list(range(13, 26))]


def _concat_numpy(gathered, slab_ld, shift, rows, offs, dst):
    """et_concat_slabs semantics (include/embtab.h) on host arrays."""
    for r, (n, o) in enumerate(zip(rows, offs)):
        if n:
            dst[:, o:o + n] = gathered[r][:, shift:shift + n]


def _worker(rank, world, port, sizes, result_q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import oracle as orc

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(0)
    dims = [16, 32, 16, 48, 16]
    B, P, k = 40, 6, 3
    tabs = [rng.random((r, d), dtype=np.float32) for r, d in zip(sizes, dims)]
    idx = [rng.integers(1, r + 1, (B, P)) for r in sizes]
    for spread in (False, True):
        assignment = plan_tables(len(dims), world, sizes=sizes if spread else None)
        layout = ShardLayout(dims, k, assignment)
        sp = ShardedPreallocation(layout, rank, world, B, torch.float32, torch.device("cpu"))
        mine = assignment[rank]
        # stand-in for et_maplookup_prealloc into the slab (dst_row_off 0 + running)
        slab = orc.maplookup_prealloc([tabs[t] for t in mine], [idx[t] for t in mine])
        sp.slab[:, :slab.shape[1]] = torch.from_numpy(slab)
        g = sp.exchange().numpy()
        dst = np.zeros((B, layout.ld), np.float32)
        for shift, rows, offs in sp.assembly_launches():
            _concat_numpy(g, layout.slab_ld, shift, rows, offs, dst)
        ref = orc.maplookup_prealloc(tabs, idx, prependrows=k)
        result_q.put((rank, spread, bool(np.array_equal(dst[:, k:], ref[:, k:]))))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_prealloc_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    sizes = [50, 400, 30, 70, 1000]
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    res = [q.get(timeout=5) for _ in range(4)]
    assert len(res) == 4 and all(ok for _, _, ok in res), res
