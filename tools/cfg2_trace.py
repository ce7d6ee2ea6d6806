"""Config 2 (BASELINE configs[1]: one 128 x 1e7 fp32 table, vector-index gather, B = 65536)
as bench.bench_config2 runs it — 16 rotated index sets, captured once in a HIP graph and
replayed — for a rocprofv3 kernel trace (per-launch kernel time against the replay period)
or PMC passes.  Prints the per-launch time of the replays (HIP events) as one JSON line.
Usage: python tools/cfg2_trace.py [replays] [--eager]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    import embtab as et
    from embtab import _lib

    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10
    eager = "--eager" in sys.argv
    dev = torch.device("cuda", 0)
    L = _lib.load()
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

    def run():
        for j in range(nsets):
            et.lookup_(dsts[j], A, sets[j])

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if eager:
        a.record(stream)
        for _ in range(reps):
            run()
        b.record(stream)
    else:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            run()
        g.replay()
        torch.cuda.synchronize()
        a.record(stream)
        for _ in range(reps):
            g.replay()
        b.record(stream)
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / (reps * nsets)
    print(json.dumps({"mode": "eager" if eager else "graph", "us_per_launch": us,
                      "GBs": B * (bench.DIM * 8 + 8) / (us * 1e-6) / 1e9}))


if __name__ == "__main__":
    main()
