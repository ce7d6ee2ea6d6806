"""Config-4 exact mode, index phase only, with ET_CHAIN_CHECK=1: validates every chain's
entries (bounds, mask indices, counts) on the device; prints the error word and the
chain statistics it can reach from the host."""
import os
import sys

os.environ["ET_CHAIN_CHECK"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    import embtab as et
    from embtab import _lib

    dev = torch.device("cuda", 0)
    L = _lib.load()
    mine = list(range(len(bench.CRITEO_KAGGLE_ROWS)))
    tables = bench.make_tables(et, L, mine, dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(4000)
    B, P, D = bench.BATCH, bench.POOL, bench.DIM
    idx = [bench.zipf_indices(bench.CRITEO_KAGGLE_ROWS[t], (B, P), 1.05, gen, dev) for t in mine]
    delta = torch.zeros((B, D * len(tables)), dtype=torch.float32, device=dev)
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, k * D:(k + 1) * D], i)
             for k, (A, i) in enumerate(zip(tables, idx))]
    et.check_errors()
    pu = et.PhasedUpdate(tables, grads, exact=True)
    pu.index_()
    torch.cuda.synchronize()
    print("chain check error word:", et.check_errors(), "(0 = every chain entry valid)")


if __name__ == "__main__":
    main()
