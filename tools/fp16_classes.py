"""The config-3 Float16 leg split by table class (as bench.table_classes for fp32): heavy /
mid / light tables (by their Float16 bytes: > 256 MiB, 4 MiB .. 256 MiB, <= 4 MiB) each alone
in one Preallocation launch, beside the mixed launch.  Prints JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    import embtab as et
    from embtab import _lib

    dev = torch.device("cuda", 0)
    L = _lib.load()
    tids = list(range(len(bench.CRITEO_KAGGLE_ROWS)))
    idx = bench.make_indices(L, tids, bench.BATCH, dev)
    stream = torch.cuda.current_stream(dev)
    tabs = []
    for t in tids:
        R = bench.CRITEO_KAGGLE_ROWS[t]
        data = torch.empty((R, bench.DIM), dtype=torch.float16, device=dev)
        _lib.check(L.et_fill_uniform(_lib.ET_F16, data.data_ptr(), data.numel(), bench.TABLE_SEED + t,
                                     0, 0.0, 1.0, stream.cuda_stream))
        tabs.append(et.SimpleEmbedding(data, et.Static(bench.DIM)))
    strat = et.PreallocationStrategy(0)
    out = {}
    B = bench.BATCH
    classes = (("mixed", lambda b: True), ("heavy", lambda b: b > (256 << 20)),
               ("mid", lambda b: (4 << 20) < b <= (256 << 20)), ("light", lambda b: b <= (4 << 20)))
    for name, pick in classes:
        sel = [k for k in tids if pick(bench.CRITEO_KAGGLE_ROWS[k] * bench.DIM * 2)]
        ts = [tabs[k] for k in sel]
        ids = [idx[k] for k in sel]
        dst = torch.empty((B, bench.DIM * len(sel)), dtype=torch.float16, device=dev)
        ms = bench._timed(lambda: et.maplookup_(strat, dst, ts, ids), 20, 3, stream)
        rows = [bench.CRITEO_KAGGLE_ROWS[k] for k in sel]
        hbm = bench.hbm_compulsory_bytes(B, bench.POOL, [bench.DIM] * len(sel), rows, es=2)
        out[name] = {"tables": len(sel), "ms": ms, "hbm_compulsory_frac":
                     hbm / (ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBS}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
