"""Config-4 exact update timed with and without Indexers (the snapshot path,
et_sparse_sgd_snap), as bench.py's config4_zipf_update times it.
Usage: python tools/upd_ix.py [steps] [warmup]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    import embtab as et
    from embtab import _lib

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    L = _lib.load()
    churn = os.environ.get("UPD_IX_CHURN", "")
    if "alloc" in churn:  # the bench's earlier legs: a 5 GB table and 16 index sets, freed
        big = torch.empty((10_000_000, 128), dtype=torch.float32, device=dev)
        sets = [torch.empty((65536, 1), dtype=torch.int64, device=dev) for _ in range(16)]
        big.fill_(1.0)
        del big, sets
    if "free" in churn:
        torch.cuda.empty_cache()
    mine = list(range(len(bench.CRITEO_KAGGLE_ROWS)))
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
    ix = [et.Indexer() for _ in tables]
    out = {}
    for name, fn in [("plain", lambda: et.update_(opt, tables, grads, None)),
                     ("indexers", lambda: et.update_(opt, tables, grads, ix)),
                     ("plain2", lambda: et.update_(opt, tables, grads, None))]:
        out[name + "_ms"] = bench._timed(fn, steps, warmup, stream)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
