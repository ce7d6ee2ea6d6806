"""Diagnostics of the exact Float32 update at BASELINE config 4.
  index   : index phase only, ET_CHAIN_CHECK=1 (plan, entries and order validated)
  plain   : full exact update with ET_CHAIN_ASM=0 (chains summed in plain C++)
Prints the device error word and, for `plain`, the time of one update."""
import os
import sys

mode = sys.argv[1] if len(sys.argv) > 1 else "index"
os.environ["ET_CHAIN_CHECK"] = "1"
if mode == "plain":
    os.environ["ET_CHAIN_ASM"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import time

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
    delta = torch.empty((B, D * len(tables)), dtype=torch.float32, device=dev)
    _lib.check(L.et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 4001, 0, -1.0, 1.0,
                                 _lib.stream_handle(dev)))
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, k * D:(k + 1) * D], i)
             for k, (A, i) in enumerate(zip(tables, idx))]
    et.check_errors()
    pu = et.PhasedUpdate(tables, grads, exact=True)
    pu.index_()
    torch.cuda.synchronize()
    print(mode, "index-phase check word:", et.check_errors(), flush=True)
    if mode == "plain":
        t0 = time.perf_counter()
        pu.update_(et.Descent(0.1))
        torch.cuda.synchronize()
        print("plain exact update phase: %.2f ms, error word %d" %
              (1e3 * (time.perf_counter() - t0), et.check_errors()), flush=True)


if __name__ == "__main__":
    main()
