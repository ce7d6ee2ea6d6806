"""The bench's config-3 Float16 leg alone (bench.bench_config3_fp16): 26 Float16 tables x 128,
pool 20, B = 65536, Julia Float16 arithmetic and fp32 accumulation; prints its JSON."""
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
    print(json.dumps(bench.bench_config3_fp16(et, L, tids, idx, dev, 20, 3, bench.BATCH)))


if __name__ == "__main__":
    main()
