"""Config-4 step: index phase of the update beside the forward, launch-order and stream
priority variants (experiment; DESIGN.md §4 "Two phases")."""
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
    tables = bench.make_tables(et, L, tids, dev)
    B, DIM, POOL = bench.BATCH, bench.DIM, bench.POOL
    stream = torch.cuda.current_stream(dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(4000)
    idx = [bench.zipf_indices(bench.CRITEO_KAGGLE_ROWS[t], (B, POOL), 1.05, gen, dev) for t in tids]
    dst = torch.empty((B, DIM * len(tables)), dtype=torch.float32, device=dev)
    delta = torch.randn((B, DIM * len(tables)), dtype=torch.float32, device=dev)
    strat, opt = et.PreallocationStrategy(0), et.Descent(0.1)
    grads = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, k * DIM:(k + 1) * DIM], i)
             for k, (A, i) in enumerate(zip(tables, idx))]
    pu = et.PhasedUpdate(tables, grads)

    def fwd():
        et.maplookup_(strat, dst, tables, idx)

    res = {}
    for name, prio in (("normal", 0), ("high", -1)):
        side = torch.cuda.Stream(dev, priority=prio)

        def idx_first():
            side.wait_stream(stream)
            pu.index_(side)
            fwd()
            pu.update_(opt)

        def fwd_first():
            side.wait_stream(stream)
            fwd()
            pu.index_(side)
            pu.update_(opt)

        res[f"{name}/index_first"] = bench._timed(idx_first, 20, 3, stream)
        res[f"{name}/fwd_first"] = bench._timed(fwd_first, 20, 3, stream)

    def serial():
        pu.index_(stream)
        fwd()
        pu.update_(opt)

    def idx_only():
        pu.index_(stream)

    def apply_only():
        pu.update_(opt)

    res["serial"] = bench._timed(serial, 20, 3, stream)
    res["forward"] = bench._timed(fwd, 20, 3, stream)
    res["index_phase"] = bench._timed(idx_only, 20, 3, stream)
    res["apply_phase"] = bench._timed(apply_only, 20, 3, stream)
    print({k: round(v, 3) for k, v in res.items()})


if __name__ == "__main__":
    main()
