"""Why a HIP graph capture slows the multi-stream exact update.

Times the config-4 exact update (bench.bench_config4's tables and Zipf batch) in one
fresh process per mode:
  none            the update alone
  pool            torch.cuda.Stream() first (initialises torch's per-device stream pools)
  capture         a tiny torch.cuda.graph capture first (never replayed)
  capture_after   one update first (the library's side streams exist), then the capture
  dummyN          N torch streams (normal priority) that have each run one kernel, first
  hidummyN        the same with high-priority streams
  capture+dummyN  a capture, then N used streams
  firstN          N used torch streams and a graph capture BEFORE any library call (as a
                  training process that opens its data-loader / communicator streams first)
  firstN+shard    the same, then a world-1 sharded step (et_sharded_create's side stream)
                  run once before the update
Prints one JSON line per process.  Run under rocprofv3 --kernel-trace to get the queue
and stream id of every dispatch (tools/queue_map.py reads them).
Usage: python tools/capture_effect.py MODE [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    import embtab as et
    from embtab import _lib

    mode = sys.argv[1] if len(sys.argv) > 1 else "none"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)

    def capture():
        x = torch.ones(1024, device=dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = x * 2  # noqa: F841
        torch.cuda.synchronize()
        return g

    def used_streams(k, prio=0):  # k streams that have each run one kernel
        out = []
        for _ in range(k):
            st = torch.cuda.Stream(device=dev, priority=prio)
            with torch.cuda.stream(st):
                torch.ones(16, device=dev).mul_(2)
            out.append(st)
        torch.cuda.synchronize()
        return out

    first = None
    if mode.startswith("first"):  # before the library's first stream-taking call
        first = used_streams(int(mode[5:].split("+")[0])) + [capture()]
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

    def upd():
        et.update_(opt, tables, grads, None)

    keep = first
    if mode.startswith("first") and mode.endswith("+shard"):
        from embtab.sharding import ShardedMapLookup, ShardPlan

        dims = [D] * len(tables)
        plan = ShardPlan.tablewise(dims, 1, sizes=bench.CRITEO_KAGGLE_ROWS)
        sh = ShardedMapLookup(plan, 0, 1, B, torch.float32, dev, exchange="allgather", chunks=4)
        out = torch.empty((B, sum(dims)), dtype=torch.float32, device=dev)
        sh(tables, idx, out)
        torch.cuda.synchronize()
        keep = [first, sh, out]
    elif mode.startswith("dummy"):  # dummyN: N used normal-priority streams first
        keep = used_streams(int(mode[5:]))
    elif mode.startswith("hidummy"):  # hidummyN: N used high-priority streams first
        keep = used_streams(int(mode[7:]), -1)
    elif mode.startswith("capture+dummy"):  # a capture, then N used streams
        keep = [capture()] + used_streams(int(mode[len("capture+dummy"):]))
    elif mode == "pool":
        keep = torch.cuda.Stream(device=dev)
    elif mode == "capture":
        keep = capture()
    elif mode == "capture_after":
        upd()
        torch.cuda.synchronize()
        keep = capture()
    ms = bench._timed(upd, steps, 2, stream)
    print(json.dumps({"mode": mode, "update_ms": ms, "kept": type(keep).__name__}), flush=True)


if __name__ == "__main__":
    main()
