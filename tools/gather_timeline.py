"""Per-workgroup timeline of the config-2 gather (k_gather_one: one 128 x 1e7 fp32 table,
vector-index gather, B = 65,536) from the profiling build (tools/wg_timeline.sh -> tools/tl/,
-DET_WG_TIMELINE), VERDICT r05 item 6: where the launch's time goes beyond the byte floor.

The 16 rotated index sets of bench.bench_config2 run back to back (cold rows, as the bench);
the last launch's workgroups leave their records: wave 0's start, the moment its row loads
are issued (its index loads have returned), and the workgroup's end once every store has
completed (s_memrealtime, 100 MHz).  Prints the launch span, the start ramp, the index
latency, the row + store phase and the end tail as one JSON object.
Usage (GPU box): python tools/gather_timeline.py [OUT.json]"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "embeddingtables.jl_amd"))


def pct(x, q):
    return round(float(np.percentile(x, q)), 2)


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
    R, B, nsets = 10_000_000, bench.BATCH, 16
    stream = torch.cuda.current_stream(dev)
    data = torch.empty((R, bench.DIM), dtype=torch.float32, device=dev)
    _lib.check(L.et_fill_uniform(_lib.ET_F32, data.data_ptr(), data.numel(), 3000, 0, 0.0, 1.0,
                                 stream.cuda_stream))
    sets = []
    for k in range(nsets):
        I = torch.empty(B, dtype=torch.int64, device=dev)
        _lib.check(L.et_fill_index_uniform(I.data_ptr(), B, R, 3001 + k, 0, stream.cuda_stream))
        sets.append(I)
    A = et.SimpleEmbedding(data, et.Static(bench.DIM))
    dsts = [torch.empty((B, bench.DIM), dtype=torch.float32, device=dev) for _ in range(nsets)]
    out = []
    for rep in range(3):
        for j in range(nsets):
            et.lookup_(dsts[j], A, sets[j])
        torch.cuda.synchronize()
        buf = np.zeros((1 << 17, 8), dtype=np.uint32)
        assert L.et_debug_timeline(buf.ctypes.data, buf.shape[0]) > 0
        grid = int(buf[0, 7])
        rec = buf[:grid]
        t0 = rec[:, 0].astype(np.uint64) | (rec[:, 1].astype(np.uint64) << np.uint64(32))
        t1 = rec[:, 2].astype(np.uint64) | (rec[:, 3].astype(np.uint64) << np.uint64(32))
        t2 = rec[:, 4].astype(np.uint64) | (rec[:, 5].astype(np.uint64) << np.uint64(32))
        base = int(t0.min())
        s = (t0.astype(np.int64) - base) / 100.0
        i = (t1.astype(np.int64) - base) / 100.0
        e = (t2.astype(np.int64) - base) / 100.0
        out.append({
            "workgroups": grid, "span_us": round(float(e.max()), 2),
            "start_us": {"p50": pct(s, 50), "p90": pct(s, 90), "max": pct(s, 100)},
            "index_wait_us": {"p10": pct(i - s, 10), "p50": pct(i - s, 50), "p90": pct(i - s, 90)},
            "rows_and_stores_us": {"p10": pct(e - i, 10), "p50": pct(e - i, 50),
                                   "p90": pct(e - i, 90)},
            "end_us": {"p10": pct(e, 10), "p50": pct(e, 50), "p90": pct(e, 90), "max": pct(e, 100)},
            "xcc_end_max_us": [round(float(e[rec[:, 6] == x].max()), 2) for x in range(8)
                               if (rec[:, 6] == x).any()],
        })
    text = json.dumps(out[-1])
    print(text)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
