"""Chain-item timeline of one exact config-4 update (experiment build only).

Runs bench.bench_config4's tables and Zipf batch through the exact update with the
experiment library (ET_LIBRARY=tools/exp/libembtab_hip_exp.so, built by tools/exp_build.sh),
reads every chain item's start / end (s_memrealtime, 100 MHz) from et_debug_chain_timeline
and prints, per chain list (0 early, 1 regular, 2 early hot): items, first start and last end
relative to the earliest item, the busy wave count over time, and the longest items.
Usage: ET_LIBRARY=tools/exp/libembtab_hip_exp.so python tools/chain_timeline.py [out.json]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

NAMES = {0: "early", 1: "regular", 2: "early-hot"}


def main():
    import torch

    import embtab as et
    from embtab import _lib

    dev = torch.device("cuda", 0)
    L = _lib.load()
    f = L.et_debug_chain_timeline
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    f.restype = ctypes.c_int
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
    cap = 1 << 17
    buf = np.zeros((cap, 8), dtype=np.uint32)
    n = ctypes.c_int64(0)
    for _ in range(3):  # warm, then the recorded call
        f(buf.ctypes.data, cap, ctypes.byref(n))
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        et.update_(et.Descent(0.1), tables, grads, None)
        ev1.record()
        torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1)
    assert f(buf.ctypes.data, cap, ctypes.byref(n)) == 0
    k = min(n.value, cap)
    r = buf[:k]
    t0 = (r[:, 0].astype(np.uint64) | (r[:, 1].astype(np.uint64) << 32)).astype(np.int64)
    t1 = (r[:, 2].astype(np.uint64) | (r[:, 3].astype(np.uint64) << 32)).astype(np.int64)
    lst, S, ngr, it, hw = r[:, 4] >> 24, r[:, 4] & 0xffffff, r[:, 5], r[:, 6], r[:, 7]
    base = t0.min()
    us0, us1 = (t0 - base) / 100.0, (t1 - base) / 100.0  # 100 MHz -> us
    out = {"update_ms_events": ms, "items": int(k), "lists": {}}
    print(f"update {ms:.3f} ms (events), {k} chain items recorded")
    for l in sorted(set(lst.tolist())):
        m = lst == l
        d = us1[m] - us0[m]
        order = np.argsort(-d)[:12]
        bins = np.arange(0, us1.max() + 100, 100)
        busy = [int(((us0[m] < b + 100) & (us1[m] > b)).sum()) for b in bins]
        info = {"items": int(m.sum()), "first_start_us": float(us0[m].min()),
                "last_end_us": float(us1[m].max()), "sum_item_us": float(d.sum()),
                "busy_waves_per_100us": busy,
                "longest": [{"S": int(S[m][j]), "groups": int(ngr[m][j]), "item": int(it[m][j]),
                             "start_us": float(us0[m][j]), "dur_us": float(d[j])}
                            for j in order]}
        out["lists"][NAMES.get(l, str(l))] = info
        print(f"[{NAMES.get(l, l)}] items {info['items']} start {info['first_start_us']:.0f} "
              f"end {info['last_end_us']:.0f} us, item-us {info['sum_item_us']:.0f}")
        print("  busy waves / 100 us:", busy)
        for x in info["longest"][:6]:
            print(f"  S={x['S']:2d} groups={x['groups']:5d} start {x['start_us']:7.0f} "
                  f"dur {x['dur_us']:7.0f} us  ({x['dur_us'] / max(1, x['groups'] * 64):.3f} us/entry)")
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            json.dump(out, fh)


if __name__ == "__main__":
    main()
