"""Config-4 update only (for rocprofv3 kernel stats of the SGD pipeline)."""
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
    mine = list(range(len(bench.CRITEO_KAGGLE_ROWS)))
    tables = bench.make_tables(et, L, mine, dev)
    r = bench.bench_config4(et, tables, mine, dev, 5, 2, bench.BATCH)
    print({k: r[k] for k in ("forward_ms", "update_ms", "step_ms")})


if __name__ == "__main__":
    main()
