"""Host-side cost of one config-4 update call against its GPU time.

Times et.update_ (exact, bench.py's config-4 tables and Zipf batch) three ways: the host
wall time of the call alone (perf_counter around it; the GPU runs behind), HIP events around
back-to-back calls (bench.py's method), and events around calls separated by a synchronize
(the GPU time of one call with no queue ahead of it).  If the host time per call approaches
the event time, the update is host-bound.  Usage: python tools/host_cost.py [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    import embtab as et
    from embtab import _lib

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
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
                                 _lib.stream_handle()))
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, k * D:(k + 1) * D], i)
             for k, (A, i) in enumerate(zip(tables, idx))]
    opt = et.Descent(0.1)
    indexers = [et.Indexer() for _ in tables]
    upd = lambda: et.update_(opt, tables, grads, indexers)  # noqa: E731
    for _ in range(3):
        upd()
    torch.cuda.synchronize()
    host = []
    for _ in range(steps):
        t0 = time.perf_counter()
        upd()
        host.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for a, b in ev:
        a.record()
        upd()
        b.record()
    torch.cuda.synchronize()
    b2b = [a.elapsed_time(b) for a, b in ev]
    iso = []
    for a, b in ev:
        torch.cuda.synchronize()
        a.record()
        upd()
        b.record()
        torch.cuda.synchronize()
        iso.append(a.elapsed_time(b))
    med = lambda x: sorted(x)[len(x) // 2]  # noqa: E731
    print(json.dumps({"host_ms_median": med(host), "host_ms_mean": sum(host) / steps,
                      "events_back_to_back_ms": sum(b2b) / steps,
                      "events_isolated_ms_median": med(iso)}))


if __name__ == "__main__":
    main()
