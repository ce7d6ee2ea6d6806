"""One rank of the one-sided (p2p) sharded maplookup parity test
(tests/test_gpu_p2p.py).  Launched by torch.distributed.run with the gloo backend,
every rank on cuda:0: the peers' destinations are IPC mappings of memory on the same
device, so the exchange kernel (et_push_cols), the handle exchange and the barriers
run exactly as across GPUs; only the xGMI link itself is absent.  Writes one JSON
result per rank to argv[1]."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "embeddingtables.jl_amd"), os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import embtab as et  # noqa: E402
import oracle as orc  # noqa: E402
from embtab.sharding import ShardedMapLookup, ShardPlan, piece_table  # noqa: E402


def main():
    out_path = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    rng = np.random.default_rng(0)
    dims = [16, 32, 16, 48, 16, 128, 96]
    sizes = [50, 400, 30, 70, 1000, 20, 333]
    B, P, k = 97, 6, 3
    hs = [rng.random((r, d), dtype=np.float32) for r, d in zip(sizes, dims)]
    hidx = [rng.integers(1, r + 1, (B, P)) for r in sizes]
    ref = orc.maplookup_prealloc(hs, hidx, prependrows=k)
    full = [et.SimpleEmbedding(torch.from_numpy(h).to(dev)) for h in hs]
    didx = [torch.from_numpy(i).to(dev) for i in hidx]
    plans = {"table": ShardPlan.tablewise(dims, world, k),
             "table_spread": ShardPlan.tablewise(dims, world, k, sizes=sizes),
             "feature": ShardPlan.featurewise(dims, world, k, granule=16)}
    results = []
    for name, plan in plans.items():
        ps = plan.pieces[rank]
        tabs = [piece_table(full[p.table], p) for p in ps]
        idx = [didx[p.table] for p in ps]
        for chunks in (1, 3):
            sm = ShardedMapLookup(plan, rank, world, B, torch.float32, dev, exchange="p2p",
                                  chunks=chunks)
            ok = True
            for rep in range(2):  # the second step rewrites the same buffers
                sm.out.fill_(float("nan"))
                torch.cuda.synchronize()
                dist.barrier()
                out = sm(tabs, idx, None)
                torch.cuda.synchronize()
                got = out.cpu().numpy()[:, k:]
                ok = ok and got.tobytes() == np.ascontiguousarray(ref[:, k:]).tobytes()
            # backward: column views of the full gradient, as for the all-gather layout
            delta = torch.arange(B * plan.ld, dtype=torch.float32, device=dev).view(B, plan.ld)
            for p, g in zip(ps, sm.piece_grads(tabs, idx, delta)):
                ok = ok and torch.equal(g.delta, delta[:, p.col:p.col + p.dim])
            dist.barrier()  # nobody unmaps while a peer may still push
            sm.close()
            results.append({"rank": rank, "plan": name, "chunks": chunks, "ok": bool(ok)})
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(results, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
