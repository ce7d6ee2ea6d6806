"""Exact config-4 update on a subset of the Criteo tables (rows in [lo, hi]): isolates the
chains of the small tables (early chains) from the rest of the update for a kernel trace.
Usage: python tools/exact_subset.py LO HI"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    import embtab as et
    from embtab import _lib

    lo, hi = int(sys.argv[1]), int(sys.argv[2])
    dev = torch.device("cuda", 0)
    L = _lib.load()
    mine = [t for t, r in enumerate(bench.CRITEO_KAGGLE_ROWS) if lo <= r <= hi]
    tables = bench.make_tables(et, L, mine, dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(4000)
    B, P, D = bench.BATCH, bench.POOL, bench.DIM
    idx = [bench.zipf_indices(bench.CRITEO_KAGGLE_ROWS[t], (B, P), 1.05, gen, dev) for t in mine]
    delta = torch.empty((B, D * len(tables)), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    _lib.check(L.et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 4001, 0, -1.0, 1.0,
                                 stream.cuda_stream))
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, k * D:(k + 1) * D], i)
             for k, (A, i) in enumerate(zip(tables, idx))]
    opt = et.Descent(0.1)
    ms = bench._timed(lambda: et.update_(opt, tables, grads, None, exact=True), 5, 2, stream)
    print(json.dumps({"tables": mine, "exact_ms": ms}))


if __name__ == "__main__":
    main()
