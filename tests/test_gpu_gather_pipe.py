"""The vector-index gather (k_gather_one, et_lookup.hip; round 5's pipelined k_gather_pipe
before it): one round of 8 rows per lane group, each row stored as it arrives.  Bit copies of
the oracle's gather (src/lookup.jl:51-87) at every row size the kernel takes (128 .. 1024
bytes), batches that end inside a workgroup and a row group, a strided destination, several
tables in one launch and out-of-range indices (zero rows, counted)."""
import numpy as np
import pytest
import torch

import embtab as et

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


def host(x):
    return x.cpu().numpy()


@pytest.mark.parametrize("dim,dtype", [(128, np.float32), (32, np.float32), (64, np.float32),
                                       (256, np.float32), (128, np.float16), (64, np.float64)])
@pytest.mark.parametrize("batch", [65536, 40000 + 37, 32768 + 1])
def test_pipelined_gather_bits(oracle, dim, dtype, batch):
    rng = np.random.default_rng(dim * 7 + batch)
    R = 50_000
    h = (rng.standard_normal((R, dim)) * 10).astype(dtype)
    A = et.SimpleEmbedding(dev(h), et.Static(dim))
    v = rng.integers(1, R + 1, batch)
    got = host(et.lookup(A, dev(v)))
    assert got.tobytes() == oracle.gather(h, v).tobytes()


def test_pipelined_gather_strided_dst_bad_indices_and_tables(oracle):
    rng = np.random.default_rng(11)
    B, R, D = 65536 + 300, 20_000, 128
    hs = [rng.standard_normal((R, D)).astype(np.float32) for _ in range(3)]
    tabs = [et.SimpleEmbedding(dev(h), et.Static(D)) for h in hs]
    vs = [rng.integers(1, R + 1, B) for _ in hs]
    vs[1][[0, 777, B - 1]] = [R + 1, 0, -5]  # out of range: zero rows, counted
    et.check_errors()
    big = torch.full((B, 3 * D + 8), -2.0, dtype=torch.float32, device=DEV)
    for k, (A, v) in enumerate(zip(tabs, vs)):
        et.lookup_(big[:, 4 + k * D:4 + (k + 1) * D], A, dev(v))
    assert et.check_errors() == 3
    got = host(big)
    for k, (h, v) in enumerate(zip(hs, vs)):
        ok = (v >= 1) & (v <= R)
        ref = np.zeros((B, D), np.float32)
        ref[ok] = oracle.gather(h, v[ok])
        assert got[:, 4 + k * D:4 + (k + 1) * D].tobytes() == ref.tobytes()
    assert (got[:, :4] == -2.0).all() and (got[:, 4 + 3 * D:] == -2.0).all()
    # the same three gathers in one launch (maplookup of vector indices)
    out = et.maplookup(et.PreallocationStrategy(0), tabs, [dev(v) for v in vs])
    et.check_errors()
    o = host(out)
    for k, (h, v) in enumerate(zip(hs, vs)):
        ok = (v >= 1) & (v <= R)
        assert o[ok, k * D:(k + 1) * D].tobytes() == oracle.gather(h, v[ok]).tobytes()
