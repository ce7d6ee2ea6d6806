"""One table class of the headline launch, alone, for per-class PMC passes.

Builds bench.py's 26 Criteo tables and indices (same seeds), keeps the tables of one class —
heavy (> 256 MiB), mid (4 MiB .. 256 MiB), light (<= 4 MiB), or all — and runs that class's
Preallocation launch (et.maplookup_) `steps` times after a warm-up, so rocprofv3 --pmc sees
only those dispatches (tools/gpu_run.sh classpmc step; tools/traffic.py sums per dispatch).
Prints the class's kernel time (HIP events) as one JSON line.
Usage: python tools/class_pmc.py CLASS [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

PICK = {
    "heavy": lambda b: b > bench.INFINITY_CACHE,
    "mid": lambda b: (4 << 20) < b <= bench.INFINITY_CACHE,
    "light": lambda b: b <= (4 << 20),
    "all": lambda b: True,
}


def main():
    import torch

    import embtab as et
    from embtab import _lib

    cls = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    L = _lib.load()
    tids = list(range(len(bench.CRITEO_KAGGLE_ROWS)))
    tables = bench.make_tables(et, L, tids, dev)
    idx = bench.make_indices(L, tids, bench.BATCH, dev)
    sel = [k for k in tids if PICK[cls](bench.CRITEO_KAGGLE_ROWS[k] * bench.DIM * 4)]
    tabs, ids = [tables[k] for k in sel], [idx[k] for k in sel]
    dst = torch.empty((bench.BATCH, bench.DIM * len(sel)), dtype=torch.float32, device=dev)
    strat = et.PreallocationStrategy(0)
    for _ in range(3):
        et.maplookup_(strat, dst, tabs, ids)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for a, b in ev:
        a.record()
        et.maplookup_(strat, dst, tabs, ids)
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    rows = [bench.CRITEO_KAGGLE_ROWS[k] for k in sel]
    print(json.dumps({"class": cls, "tables": len(sel), "rows": rows,
                      "ms_median": ms[len(ms) // 2], "ms_mean": sum(ms) / len(ms),
                      "algorithmic_bytes": bench.algorithmic_bytes(bench.BATCH, bench.POOL,
                                                                   [bench.DIM] * len(sel)),
                      "hbm_compulsory_bytes": bench.hbm_compulsory_bytes(
                          bench.BATCH, bench.POOL, [bench.DIM] * len(sel), rows)}))


if __name__ == "__main__":
    main()
