"""Config-4 update: the split (chunked) mode against the exact serial mode.

Times both update modes on the Zipf(1.05) 26-table batch and reports how far the split
mode's result lies from the exact one (the reference's serial order,
src/sparseupdate.jl:110-127) over every table element, as a relative deviation."""
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
    w0 = [A.data.clone() for A in tables]
    out = {}
    modes = [("exact", True), ("split", False)]
    if len(sys.argv) > 1:
        modes = [m for m in modes if m[0] in sys.argv[1:]]
    res = {}
    for name, exact in modes:
        ms = bench._timed(lambda: et.update_(opt, tables, grads, None, exact=exact), 10, 2, stream)
        out[f"{name}_ms"] = ms
        for A, w in zip(tables, w0):
            A.data.copy_(w)
        et.update_(opt, tables, grads, None, exact=exact)
        torch.cuda.synchronize()
        res[name] = [A.data.clone() for A in tables]
        for A, w in zip(tables, w0):
            A.data.copy_(w)
    if "exact" in res and "split" in res:
        worst, n_over, n_diff, n_el = 0.0, 0, 0, 0
        per_table = []
        for t in mine:
            e, s = res["exact"][t].double(), res["split"][t].double()
            rel = (s - e).abs() / e.abs().clamp_min(1e-30)
            m = float(rel.max())
            per_table.append(m)
            worst = max(worst, m)
            n_over += int((rel > 1e-6).sum())
            n_diff += int((s != e).sum())
            n_el += e.numel()
        out.update({"split_vs_exact_max_rel": worst, "elements_over_1e-6_rel": n_over,
                    "elements_differing": n_diff, "elements": n_el,
                    "per_table_max_rel": per_table})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
