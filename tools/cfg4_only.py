"""bench.py's config-4 leg alone (or after the legs named on the command line) (bench_config4 on freshly made tables), to separate its
timing from the legs that run before it in the full bench."""
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
    mine = list(range(len(bench.CRITEO_KAGGLE_ROWS)))
    tables = bench.make_tables(et, L, mine, dev)
    legs = sys.argv[1:]  # legs to run first, as the full bench does: fp16, config2
    if legs:
        gen = torch.Generator(device=dev)
        gen.manual_seed(1234)
        idx = [torch.randint(1, bench.CRITEO_KAGGLE_ROWS[t] + 1, (bench.BATCH, bench.POOL),
                             generator=gen, device=dev) for t in mine]
        if "fp16" in legs:
            bench.bench_config3_fp16(et, L, mine, idx, dev, 20, 3, bench.BATCH)
        if "config2" in legs:
            bench.bench_config2(et, L, dev, 320, 2)
    r = bench.bench_config4(et, tables, mine, dev, 10, 2, bench.BATCH)
    print(json.dumps({k: r[k] for k in ("forward_ms", "update_ms", "update_split_ms", "step_ms")}))


if __name__ == "__main__":
    main()
