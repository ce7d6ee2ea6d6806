"""Per-workgroup completion timeline of the headline launch (config 3: 26 Criteo tables,
B = 65536, pool 20) from the profiling build (tools/wg_timeline.sh -> tools/tl/).

Every workgroup of the striped kernel stamps its start and end (s_memrealtime, 100 MHz)
with its table, XCC and hardware slot.  Reported per XCC and per table class (heavy:
> 256 MiB, mid: > 4 MiB, light): when the class's workgroups start and end, so one can
see whether the L2-bound light stripes run after the heavy stripes have drained (the
launch's tail) or beside them.  Usage (GPU box): python tools/wg_timeline.py OUT.json"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "embeddingtables.jl_amd"))


def main():
    os.environ["ET_LIBRARY"] = os.path.join(REPO, "tools", "tl", "libembtab_hip.so")
    import torch

    import bench
    from embtab import _lib
    import embtab as et

    L = _lib.load()
    L.et_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    L.et_debug_timeline.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    tids = list(range(len(bench.CRITEO_KAGGLE_ROWS)))
    tables = bench.make_tables(et, L, tids, dev)
    idx = bench.make_indices(L, tids, bench.BATCH, dev)
    strat = et.PreallocationStrategy(0)
    dst = torch.empty((bench.BATCH, bench.DIM * len(tids)), dtype=torch.float32, device=dev)
    runs = []
    for it in range(6):
        et.maplookup_(strat, dst, tables, idx)
        torch.cuda.synchronize()
        buf = np.zeros((1 << 17, 8), dtype=np.uint32)
        n = L.et_debug_timeline(buf.ctypes.data, buf.shape[0])
        assert n > 0
        grid = int(buf[0, 7])
        rec = buf[:grid]
        t0 = rec[:, 0].astype(np.uint64) | (rec[:, 1].astype(np.uint64) << np.uint64(32))
        t1 = rec[:, 2].astype(np.uint64) | (rec[:, 3].astype(np.uint64) << np.uint64(32))
        runs.append((grid, t0, t1, rec[:, 4].copy(), rec[:, 5].copy(), rec[:, 6].copy()))
    grid, t0, t1, tab, xcc, hw = runs[-1]  # a warm launch
    base = int(t0.min())
    s = (t0.astype(np.int64) - base) / 100.0  # us (100 MHz clock)
    e = (t1.astype(np.int64) - base) / 100.0
    rows = bench.CRITEO_KAGGLE_ROWS
    nbytes = [r * bench.DIM * 4 for r in rows]

    def cls(t):
        if t == 0xff:
            return "idle"
        return "heavy" if nbytes[t] > (256 << 20) else "mid" if nbytes[t] > (4 << 20) else "light"

    c = np.array([cls(int(t)) for t in tab])
    out = {"grid": grid, "launch_us": float(e.max()), "classes": {}, "per_xcc": {},
           "class_tables": {k: [t for t in tids if cls(t) == k] for k in ("heavy", "mid", "light")}}
    for k in ("heavy", "mid", "light", "idle"):
        m = c == k
        if not m.any():
            continue
        d = e[m] - s[m]
        out["classes"][k] = {"workgroups": int(m.sum()), "first_start_us": float(s[m].min()),
                             "last_end_us": float(e[m].max()),
                             "end_p50_us": float(np.percentile(e[m], 50)),
                             "end_p90_us": float(np.percentile(e[m], 90)),
                             "wg_us_mean": float(d.mean()), "wg_us_p90": float(np.percentile(d, 90)),
                             "wg_time_sum_us": float(d.sum())}
    for x in sorted(set(int(v) for v in xcc)):
        mx = xcc == x
        ent = {"workgroups": int(mx.sum()), "last_end_us": float(e[mx].max())}
        for k in ("heavy", "mid", "light"):
            m = mx & (c == k)
            if m.any():
                ent[k] = {"n": int(m.sum()), "last_end_us": float(e[m].max()),
                          "end_p90_us": float(np.percentile(e[m], 90))}
        out["per_xcc"][str(x)] = ent
    # what is running in each 50 us bin: workgroup-time by class (occupancy profile)
    T = float(e.max())
    nb = int(T // 50) + 1
    prof = {k: [0.0] * nb for k in ("heavy", "mid", "light")}
    for k in prof:
        m = c == k
        for a, b in zip(s[m], e[m]):
            for q in range(int(a // 50), int(b // 50) + 1):
                lo, hi = max(a, q * 50.0), min(b, (q + 1) * 50.0)
                if hi > lo:
                    prof[k][q] += (hi - lo) / 50.0
    out["resident_wg_per_50us"] = {k: [round(v, 1) for v in p] for k, p in prof.items()}
    out["xcc_of_blockIdx_mod8_agrees"] = float(np.mean((np.arange(grid) % 8) == xcc))
    out["launch_us_all_runs"] = [float((r[2].astype(np.int64) - r[1].astype(np.int64).min()).max())
                                 / 100.0 for r in runs]
    json.dump(out, open(sys.argv[1], "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("grid", "launch_us", "classes", "launch_us_all_runs")}))


if __name__ == "__main__":
    main()
